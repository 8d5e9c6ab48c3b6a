#!/usr/bin/env python3
"""BASELINE configs[4], per GPU: one frame of the joint fractal + H.264 codec
(ZhangLing_Yu path) at 1080p, all on one MI355X, inputs resident:

  fractal   encode_one_macroblock quadtree (ZL/src/block_enc.c:508) for the Y plane
            (1920x1088) and both chroma planes (960x544), thesis search range 7,
            4 reference views (C, H, M, N), then decode_one_macroblock
            (ZL/src/block_dec.c:20) of the three planes from the trees;
  H.264     JM 18.5 full-search integer-pel ME (FS +-32, the 334,560 searches JM ran
            for the bench clip's P-frame: tests/golden/c2_syn_1080p_fs32).

Parity: the ME against JM's own results (every search); the U plane's fractal
trees and reconstruction against the C restatement (every macroblock).  The
frames of a GOP are sequential (each P-frame refers to the previous
reconstruction), so N GPUs run N GOPs: the per-GPU frame time below is the
scaling unit (bench.py --gpus N measures that replica scaling for the ME).
Usage (GPU): python3 tools/bench_hybrid.py [--iters 10]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "--h.264-by-zhaodongyu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from jmme import BLOCK_RES, FRACTAL_MB, FULL_SEARCH, NSLOT, MotionEstimator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--range", type=int, default=7)
    ap.add_argument("--tol16", type=float, default=8.0)
    ap.add_argument("--tol8", type=float, default=5.0)
    a = ap.parse_args()
    import bench
    import oracle_lib as ol
    from fractal_scenes import gate_scene
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    me = MotionEstimator({"SearchRange": 32, "SearchMode": -1, "RDOptimization": 0})

    # ---- fractal planes: Y and U, V with four views each ----
    planes = []
    for comp, (W, H, seed) in enumerate([(1920, 1088, 11), (960, 544, 12), (960, 544, 13)], start=1):
        org, refs = gate_scene(W, H, seed, 4, scale=6)
        d_org = torch.from_numpy(org).to(dev)
        d_refs = [torch.from_numpy(r).to(dev) for r in refs]
        d_words = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in refs]
        n_mb = (W // 16) * (H // 16)
        d_tree = torch.empty(n_mb * FRACTAL_MB.itemsize, dtype=torch.uint8, device=dev)
        d_rec = torch.empty((H, W), dtype=torch.uint8, device=dev)
        planes.append(dict(comp=comp, W=W, H=H, org=org, refs=refs, d_org=d_org, d_refs=d_refs, d_words=d_words,
                           d_tree=d_tree, d_rec=d_rec, n_mb=n_mb))

    def fractal_encode():
        for p in planes:
            for r, wd in zip(p["d_refs"], p["d_words"]):
                me.fractal_words_async(r.data_ptr(), p["W"], p["W"], p["H"], wd.data_ptr(), st)
            me.fractal_encode_mbs_async(p["d_org"].data_ptr(), p["d_refs"][0].data_ptr(), p["W"],
                                        [wd.data_ptr() for wd in p["d_words"]], p["W"], p["H"], a.range, a.tol16,
                                        a.tol8, p["d_tree"].data_ptr(), st)

    def fractal_decode():
        for p in planes:
            me.fractal_decode_mbs_async(p["d_tree"].data_ptr(), [r.data_ptr() for r in p["d_refs"]], p["W"],
                                        p["W"], p["H"], p["comp"], p["d_rec"].data_ptr(), 0, st)

    # ---- H.264 ME: the headline workload ----
    cur, ref, req, unit_of, slots, expect, meta = bench.load_workload()
    me.upload_cur(cur)
    me.upload_ref(0, 0, ref)
    n = len(req)
    d_req = torch.from_numpy(req.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n * NSLOT * BLOCK_RES.itemsize, dtype=torch.uint8, device=dev)

    def h264_me():
        me.search_async(FULL_SEARCH, d_req.data_ptr(), n, d_out.data_ptr(), st)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    ms_enc = timed(fractal_encode)
    ms_dec = timed(fractal_decode)
    ms_me = timed(h264_me)
    ms_frame = timed(lambda: (fractal_encode(), fractal_decode(), h264_me()))

    # parity
    out = d_out.cpu().numpy().view(BLOCK_RES).reshape(n, NSLOT)[unit_of, slots]
    me_exact = int(np.sum((out["mv_x"] == expect[0]) & (out["mv_y"] == expect[1]) & (out["cost"] == expect[2])))
    pu = planes[1]
    got = pu["d_tree"].cpu().numpy().view(FRACTAL_MB)
    t0 = time.time()
    exp = ol.fractal_encode_mbs(pu["org"], pu["refs"], a.range, a.tol16, a.tol8)
    cpu_enc_s = time.time() - t0
    g, e = got.copy(), exp.copy()
    g["chun"][np.isnan(g["chun"])] = 0
    e["chun"][np.isnan(e["chun"])] = 0
    tree_exact = int((g.view(np.uint8).reshape(len(g), -1) == e.view(np.uint8).reshape(len(e), -1)).all(1).sum())
    rc, rec_exp = ol.fractal_decode_mbs(exp, pu["refs"], 2)
    rec_exact = rc == 0 and bool(np.array_equal(pu["d_rec"].cpu().numpy(), rec_exp))
    nodes = {}
    for p in planes:
        t = p["d_tree"].cpu().numpy().view(FRACTAL_MB)
        nodes[f"comp{p['comp']}_split_mbs"] = int((t["mb"]["partition"] == 3).sum())
    me.close()
    print(json.dumps({
        "metric": "hybrid fractal + H.264 frames/sec per GPU (1080p, configs[4])",
        "value": round(1e3 / ms_frame, 1), "unit": "frames/sec", "ms_per_frame": round(ms_frame, 4),
        "stages_ms": {"fractal_encode_YUV_4views": round(ms_enc, 4), "fractal_decode_YUV": round(ms_dec, 4),
                      "h264_fs32_me": round(ms_me, 4)},
        "fractal": {"R": a.range, "tol_16": a.tol16, "tol_8": a.tol8, "views": 4,
                    "macroblocks": sum(p["n_mb"] for p in planes), **nodes},
        "parity": {"h264_me_vs_jm": {"searches": int(len(expect[0])), "bit_exact": me_exact},
                   "u_plane_trees_vs_restatement": {"macroblocks": pu["n_mb"], "exact": tree_exact},
                   "u_plane_reconstruction_vs_restatement": rec_exact},
        "cpu_baseline": {"value": round(pu["n_mb"] / cpu_enc_s, 1), "unit": "macroblocks/sec", "cores": 1,
                         "kind": "port", "sample": f"fractal encode of the U plane ({pu['n_mb']} MBs, 4 views), "
                                                   "oracle/fractal_oracle.c"},
        "scaling": "GOP replicas (frames of a GOP are sequential)"}))


if __name__ == "__main__":
    main()
