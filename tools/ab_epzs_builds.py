#!/usr/bin/env python3
"""A/B of drop-in encoder builds on the bench's EPZS row (1080p, encoder_baseline.cfg's EPZS keys), the builds
alternating round by round.  GPU box.
Usage: python3 tools/ab_epzs_builds.py ROUNDS ENCODER[:NAME=VALUE,...] ...   (paths relative to the repo; the
assignments: extra environment for that arm)"""
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)
import bench_blocks  # noqa: E402
from jmme import synth  # noqa: E402
from test_jm_dropin_epzs_gpu import BASELINE_EPZS  # noqa: E402
from test_jm_dropin_gpu import CFG  # noqa: E402

rounds = int(sys.argv[1])
encoders = sys.argv[2:]
params = dict(BASELINE_EPZS, SearchRange=32, NumberReferenceFrames=1)
w, h, frames = 1920, 1080, 2
with tempfile.TemporaryDirectory() as d:
    yuv = os.path.join(d, "in.yuv")
    synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=2024, gmv=(5, 3)))
    for r in range(rounds):
        for spec in encoders:
            e, _, kv = spec.partition(":")
            env = dict(x.split("=", 1) for x in kv.split(",")) if kv else {}
            res = bench_blocks._lencod(os.path.join(REPO, e), d, f"r{r}", yuv, w, h, frames, params, CFG, env=env)
            print(json.dumps({"encoder": spec, "round": r, "me_s": res["me_s"], "wall_s": res.get("wall_s"),
                              "md5": res.get("md5")}), flush=True)
