#!/usr/bin/env python3
"""One drop-in encode of the bench's FS + sub-pel row (1080p, encoder_baseline.cfg's sub-pel keys) with the
adapter's miss trace on (JMME_TRACE_MISS): every failed guess with the guesses held for it.  GPU box.
Usage: python3 tools/trace_fs_subpel.py OUTDIR [FS|FFS]"""
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)
import bench_blocks  # noqa: E402
from jmme import synth  # noqa: E402
from test_jm_dropin_gpu import CFG  # noqa: E402

out = os.path.abspath(sys.argv[1])
mode = sys.argv[2] if len(sys.argv) > 2 else "FS"
os.makedirs(out, exist_ok=True)
params = dict(bench_blocks.BASELINE_SUBPEL, SearchMode=-1 if mode == "FS" else 0, SearchRange=32, NumberReferenceFrames=1)
w, h, frames = 1920, 1080, 2
with tempfile.TemporaryDirectory() as d:
    yuv = os.path.join(d, "in.yuv")
    synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=2024, gmv=(5, 3)))
    r = bench_blocks._lencod(os.path.join(REPO, "integration", "_build", "lencod_jmme"), d, "t", yuv, w, h, frames, params,
                             CFG, env={"JMME_TRACE_MISS": os.path.join(out, "miss.txt"), "JMME_TRACE": os.path.join(out, "batches.txt"),
                                       "JMME_PHASES": "1"})
print(json.dumps({k: v for k, v in r.items() if k != "md5"}))
