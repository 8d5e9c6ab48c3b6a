#!/usr/bin/env python3
"""Phase breakdown of the unit kernel from a -DJMME_STAMPS build (diagnostic).
Usage: JMME_LIB=<stamps build> python3 tools/stamps.py"""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = [sys.argv[0], "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
from jmme import _lib, FULL_SEARCH, MotionEstimator, BLOCK_RES, NSLOT  # noqa: E402
cur, ref, req, unit_of, slots, expect, meta = bench.load_workload()
me = MotionEstimator({"SearchRange": 32, "SearchMode": -1})
me.upload_cur(cur); me.upload_ref(0, 0, ref)
out = me.search(FULL_SEARCH, req)
st = np.zeros((len(req), 8), np.uint64)
n = _lib.lib().jmme_debug_stamps(me._ctx, _lib.ptr(st), len(req))
st = st[:n].astype(np.float64)
names = ["wait", "expand", "sweep", "reduce", "refine", "output"]
tot = st[:, :6].sum(1)
print("units", n, "items", int(st[:, 7].sum()), "mean cycles per unit", tot.mean())
for i, nm in enumerate(names):
    print(f"{nm:8s} mean {st[:, i].mean():12.0f} cyc  {100 * st[:, i].sum() / tot.sum():5.1f}%")
