#!/usr/bin/env python3
"""Latency of one EPZS search alone (the drop-in's misses: jmme_epzs_speculate
with n = 1, the fused search + refinement kernel), split into what the launch
costs, what the search costs and what the chained refinement costs.  JM's own
1080p EPZSSubPelGrid requests (tests/golden/epzs_grid_syn_1080p_r32), sampled
by block type.  GPU box; run under `rocprofv3 --kernel-trace` and give the
kernel trace to --trace afterwards for per-category kernel durations.

Usage: python3 tools/ubench_epzs_single.py [--per 200]
       python3 tools/ubench_epzs_single.py --trace DIR/t_kernel_trace.csv --log OUT"""
import argparse
import csv
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)

CATS = ("floor", "floor/unfused", "floor/small map", "search", "search/unfused", "search+refine")


def trace_summary(path, log):
    plan = [json.loads(l) for l in open(log) if l.startswith("{\"phase\"")]
    rows = [r for r in csv.DictReader(open(path)) if "epzs_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    k = 0
    for ph in plan:
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[k:k + ph["calls"]]]
        k += ph["calls"]
        if ph["phase"] != "warmup":
            print(json.dumps({"phase": ph["phase"], "bt": ph["bt"], "calls": len(d),
                              "kernel_us_mean": round(float(np.mean(d)) / 1e3, 2),
                              "kernel_us_p50": round(float(np.median(d)) / 1e3, 2)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per", type=int, default=200)
    ap.add_argument("--trace")
    ap.add_argument("--log")
    a = ap.parse_args()
    if a.trace:
        trace_summary(a.trace, a.log)
        return
    from epzs_cases import EpzsCase
    from test_epzs_gpu import _cfg_for
    from test_epzs_spec_gpu import _req_for_engine

    from jmme import SUBPEL_REQ, MotionEstimator
    c = EpzsCase("epzs_grid_syn_1080p_r32")
    rng = np.random.default_rng(3)
    with MotionEstimator(_cfg_for(c)) as me:
        for f, cur, refs, req, exp in c.frames():
            me.upload_cur(cur)
            for k, r in enumerate(refs):
                me.upload_ref(0, k, r)
            break
        q_all = _req_for_engine(req)

        def single(i, phase):
            q = q_all[i:i + 1].copy()
            o, n = int(q["pred_off"][0]), int(q["n_pred"][0])
            preds = c.preds[o:o + n]
            so, ns = int(q["stale_off"][0]), int(q["n_stale"][0])
            stale = c.stale[so:so + ns]
            q["pred_off"], q["stale_off"] = 0, 0
            if phase.startswith("floor"):
                q["medthres"] = 1 << 40
            if phase == "floor/small map":
                q["max_x"] = q["max_y"] = 8
            sp = np.zeros(1, SUBPEL_REQ)
            sp["pos_x"], sp["pos_y"] = q["pos_x"], q["pos_y"]
            sp["blocktype"] = q["blocktype"] if phase == "search+refine" else 0
            sp["ref_slot"] = q["ref_slot"]
            sp["pred_x"], sp["pred_y"] = q["pred_x"], q["pred_y"]
            sp["lambda_h"] = sp["lambda_q"] = int(q["lambda"][0])
            sp["subthres"] = 2048
            sp["variant"] = 1
            sp["metric_h"] = sp["metric_q"] = 2
            sp["start_hp"] = sp["start_qp"] = 1
            sp["search_pos2"] = sp["search_pos4"] = 9
            return q, preds, stale, sp

        def run(phase, bt, idx):
            t0 = time.perf_counter()
            for i in idx:
                q, preds, stale, sp = single(i, phase)
                me.epzs_speculate(q, preds, None, stale, max_visited=256,
                                  sp_req=None if phase.endswith("unfused") else sp)
            dt = (time.perf_counter() - t0) / max(len(idx), 1)
            print(json.dumps({"phase": phase, "bt": bt, "calls": len(idx), "host_us_per_call": round(dt * 1e6, 1)}),
                  flush=True)

        ok = np.nonzero((q_all["n_pred"] <= 128) & (q_all["n_stale"] <= 64))[0]
        run("warmup", 0, ok[:100])
        for bt in (1, 4, 7):
            sel = ok[q_all["blocktype"][ok] == bt]
            idx = rng.choice(sel, min(a.per, len(sel)), replace=False)
            for ph in CATS:
                run(ph, bt, idx)


if __name__ == "__main__":
    main()
