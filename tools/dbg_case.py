#!/usr/bin/env python3
"""Debug aid: run one golden case through the async path (no status check)
and summarise mismatches per slot.  Usage: python3 tools/dbg_case.py [case]"""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "--h.264-by-zhaodongyu_amd"))
import torch  # noqa: E402
import golden_io as g  # noqa: E402
from jmme import MotionEstimator, BLOCK_RES, NSLOT  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c1_foreman_qcif_fs16"
c = g.Case(name)
ov = g.manifest()[name]["cfg_overrides"]
mode = ov["SearchMode"]
me = MotionEstimator({"SearchRange": ov["SearchRange"], "SearchMode": mode})
bad = tot = 0
for f, lst, rf, idx in c.groups():
    me.upload_cur(c.cur[f]); me.upload_ref(lst, rf, c.ref[(f, lst, rf)])
    req, unit_of, slots = c.units(idx, mode)
    d_req = torch.from_numpy(req.view(np.uint8).copy()).cuda()
    d_out = torch.zeros(len(req) * NSLOT * BLOCK_RES.itemsize, dtype=torch.uint8, device="cuda")
    me.search_async(mode, d_req.data_ptr(), len(req), d_out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy().view(BLOCK_RES).reshape(len(req), NSLOT)
    res = out[unit_of, slots]
    ok = (res["mv_x"] == c.r["out_mv_x"][idx]) & (res["mv_y"] == c.r["out_mv_y"][idx]) & (res["cost"] == c.r["out_cost"][idx])
    bad += int((~ok).sum()); tot += len(idx)
    if not ok.all():
        k = np.nonzero(~ok)[0]
        print("frame", f, "ref", rf, "bad", len(k), "of", len(idx), "bad slots hist", np.bincount(slots[k], minlength=NSLOT).tolist())
        for i in k[:6]:
            print("  unit", unit_of[i], "slot", slots[i], "got", res[i]["mv_x"], res[i]["mv_y"], res[i]["cost"],
                  "want", c.r["out_mv_x"][idx[i]], c.r["out_mv_y"][idx[i]], c.r["out_cost"][idx[i]])
print("TOTAL bad", bad, "of", tot)
