#!/usr/bin/env python3
"""Diagnostic: repeat the 10-bit JM golden search (c2_syn_1080p_fs32_10bit) in one
process and report, per repetition, which units / slots differ from JM and how
(looking for a result that depends on timing).  GPU box.
Usage: python3 tools/flake_hbd.py [--reps 20] [--case c2_syn_1080p_fs32_10bit]"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--case", default="c2_syn_1080p_fs32_10bit")
    a = ap.parse_args()
    import golden_io as g
    from jmme import MotionEstimator
    c = g.Case(a.case)
    ov = g.manifest()[a.case]["cfg_overrides"]
    cfg = {"SearchRange": ov["SearchRange"], "SearchMode": ov["SearchMode"]}
    if c.bits > 8:
        cfg["SourceBitDepthLuma"] = c.bits
    mode = ov["SearchMode"]
    bad_total = 0
    with MotionEstimator(cfg) as me:
        groups = list(c.groups())
        for rep in range(a.reps):
            for f, lst, rf, idx in groups:
                me.upload_cur(c.cur[f])
                me.upload_ref(lst, rf, c.ref[(f, lst, rf)])
                req, unit_of, slots = c.units(idx, mode)
                try:
                    out = me.search(mode, req)
                except Exception as e:   # (a diagnostic build's checks fail loudly)
                    print(json.dumps({"rep": rep, "error": str(e)}), flush=True)
                    bad_total += 1
                    continue
                res = out[unit_of, slots]
                ok = ((res["mv_x"] == c.r["out_mv_x"][idx]) & (res["mv_y"] == c.r["out_mv_y"][idx]) &
                      (res["cost"] == c.r["out_cost"][idx]))
                nb = int((~ok).sum())
                bad_total += nb
                rec = {"rep": rep, "frame": int(f), "ref": int(rf), "differ": nb}
                if nb:
                    k = np.nonzero(~ok)[0]
                    units = sorted(set(int(unit_of[i]) for i in k))
                    rec["units"] = units[:20]
                    rec["slots_of_first"] = sorted(int(slots[i]) for i in k if int(unit_of[i]) == units[0])
                    u0 = units[0]
                    rec["req_first"] = {n: int(req[n][u0]) for n in req.dtype.names if req[n][u0].ndim == 0}
                    # where the wrong answers come from: units whose JM answer for the same slot is
                    # exactly the GPU's (another unit's results written here?)
                    jm_by_slot = {}
                    for i in k[:64]:
                        sl = int(slots[i])
                        if sl not in jm_by_slot:
                            sel = np.nonzero(slots == sl)[0]
                            jm_by_slot[sl] = (sel, c.r["out_mv_x"][idx[sel]], c.r["out_mv_y"][idx[sel]],
                                              c.r["out_cost"][idx[sel]])
                        sel, mx, my, co = jm_by_slot[sl]
                        hit = sel[(mx == res["mv_x"][i]) & (my == res["mv_y"][i]) & (co == res["cost"][i])]
                        rec.setdefault("source_units", []).append(
                            (int(unit_of[i]), sl, [int(unit_of[h]) for h in hit[:4]]))
                    rec["slots_by_unit"] = {str(un): sorted(int(slots[i]) for i in k if int(unit_of[i]) == un)
                                            for un in units[:6]}
                    rec["examples"] = [(int(slots[i]), int(res["mv_x"][i]), int(res["mv_y"][i]), int(res["cost"][i]),
                                        int(c.r["out_mv_x"][idx[i]]), int(c.r["out_mv_y"][idx[i]]),
                                        int(c.r["out_cost"][idx[i]])) for i in k[:8]]
                print(json.dumps(rec), flush=True)
    print(json.dumps({"reps": a.reps, "bad_total": bad_total}))


if __name__ == "__main__":
    main()
