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
NWG_ROWS = 2048   # kStampWGs * 4 words / 8
raw = np.zeros((len(req) + NWG_ROWS, 8), np.uint64)
n = _lib.lib().jmme_debug_stamps(me._ctx, _lib.ptr(raw), len(req) + NWG_ROWS)
st = raw[:len(req)].astype(np.float64)
wg = raw[len(req):n].reshape(-1, 4)
names = ["wait", "expand", "sweep", "reduce", "refine", "output"]
tot = st[:, :6].sum(1)
print("units", n, "items", int(st[:, 7].sum()), "mean cycles per unit", tot.mean())
for i, nm in enumerate(names):
    print(f"{nm:8s} mean {st[:, i].mean():12.0f} cyc  {100 * st[:, i].sum() / tot.sum():5.1f}%")

# per-workgroup records: start, end (100 MHz realtime), HW_ID, XCC_ID << 32 | items
wg = wg[wg[:, 3] != 0]
if len(wg):
    t0, t1 = wg[:, 0].astype(np.int64), wg[:, 1].astype(np.int64)
    base = t0.min()
    t0, t1 = (t0 - base) * 10, (t1 - base) * 10   # ns
    hw = wg[:, 2].astype(np.int64)
    xcc = (wg[:, 3] >> 32).astype(np.int64)
    items = (wg[:, 3] & 0xffffffff).astype(np.int64)
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    print("workgroups", len(wg), "span ns", t1.max(), "start spread ns", t0.max(), "end min/med/max ns",
          t1.min(), int(np.median(t1)), t1.max())
    print("items per wg: hist", np.bincount(items).tolist())
    for k in sorted(set(items.tolist())):
        sel = items == k
        print(f"  wgs with {k} items: {sel.sum()}  end ns mean {t1[sel].mean():.0f} max {t1[sel].max()}")
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    ucu, inv = np.unique(key, return_inverse=True)
    per_cu_items = np.bincount(inv, weights=items)
    per_cu_wgs = np.bincount(inv)
    per_cu_end = np.zeros(len(ucu)); np.maximum.at(per_cu_end, inv, t1)
    print("CUs", len(ucu), "wgs per CU hist", np.bincount(per_cu_wgs).tolist(),
          "items per CU hist", np.bincount(per_cu_items.astype(int)).tolist())
    for k in sorted(set(per_cu_items.astype(int).tolist())):
        sel = per_cu_items.astype(int) == k
        print(f"  CUs with {k} items: {sel.sum()}  last end ns mean {per_cu_end[sel].mean():.0f} max {per_cu_end[sel].max():.0f}")
    np.save(os.path.join(REPO, "gpurun_out", "stamps_wg.npy"), raw[len(req):n])

