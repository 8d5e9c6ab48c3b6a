#!/usr/bin/env python3
"""A/B of drop-in encoder builds on the bench's FS + sub-pel row (1080p, encoder_baseline.cfg's sub-pel keys,
JMME_PHASES=1), the builds alternating round by round.  GPU box.
Usage: python3 tools/ab_fs_subpel.py ROUNDS ENCODER[:LIBDIR] ...   (paths relative to the repo; LIBDIR: a libjmme
build taken through LD_LIBRARY_PATH ahead of the encoder's runpath)"""
import json
import os
import re
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)
import bench_blocks  # noqa: E402
from jmme import synth  # noqa: E402
from test_jm_dropin_gpu import CFG  # noqa: E402

rounds = int(sys.argv[1])
encoders = sys.argv[2:]
params = dict(bench_blocks.BASELINE_SUBPEL, SearchMode=-1, SearchRange=32, NumberReferenceFrames=1)
w, h, frames = 1920, 1080, 2
with tempfile.TemporaryDirectory() as d:
    yuv = os.path.join(d, "in.yuv")
    synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=2024, gmv=(5, 3)))
    for r in range(rounds):
        for spec in encoders:
            e, _, libdir = spec.partition(":")
            env = {"JMME_PHASES": "1"}
            if libdir:
                env["LD_LIBRARY_PATH"] = os.path.join(REPO, libdir) + ":" + os.environ.get("LD_LIBRARY_PATH", "")
            res = bench_blocks._lencod(os.path.join(REPO, e), d, f"r{r}", yuv, w, h, frames, params, CFG, env=env)
            sp = re.search(r"([\d.]+) ms in sub-pel batches[^\n]*", res.get("stderr", ""))
            ch = re.search(r"([\d.]+) ms in chain-only calls", res.get("stderr", ""))
            print(json.dumps({"encoder": spec, "round": r, "me_s": res["me_s"], "md5": res.get("md5"),
                              "subpel": sp.group(0) if sp else None, "chain_only_ms": ch.group(1) if ch else None}),
                  flush=True)
