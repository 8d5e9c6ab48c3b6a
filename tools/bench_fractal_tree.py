#!/usr/bin/env python3
"""Fractal macroblock encoder throughput: the thesis's
encode_one_macroblock quadtree (16x16 -> 8x8 -> 8x4/4x8 pairs -> 4x4, each
level searched over n_views reference views) for every macroblock of a
synthetic plane, on one MI355X, next to the C restatement on the same plane
(bounded: only the first rows of macroblocks).  One JSON line per (size, views).
Usage (GPU): python3 tools/bench_fractal_tree.py [--iters 5] [--range 7]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "--h.264-by-zhaodongyu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from jmme import FRACTAL_MB, MotionEstimator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--range", type=int, default=7)
    ap.add_argument("--tol16", type=float, default=8.0)   # configfile.h:100-101 defaults
    ap.add_argument("--tol8", type=float, default=5.0)
    ap.add_argument("--cpu-rows", type=int, default=2)
    ap.add_argument("--sizes", default="352x288,1920x1088")
    ap.add_argument("--views", default="1,4")
    a = ap.parse_args()
    import oracle_lib as ol
    from fractal_scenes import gate_scene
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    me = MotionEstimator()
    R = a.range
    for size in a.sizes.split(","):
        W, H = (int(v) for v in size.split("x"))
        for K in (int(v) for v in a.views.split(",")):
            org, refs = gate_scene(W, H, 5, K, scale=6)
            n_mb = (W // 16) * (H // 16)
            d_org = torch.from_numpy(org).to(dev)
            d_refs = [torch.from_numpy(r).to(dev) for r in refs]
            d_words = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in refs]
            d_out = torch.empty(n_mb * FRACTAL_MB.itemsize, dtype=torch.uint8, device=dev)

            def step():
                for r, wd in zip(d_refs, d_words):
                    me.fractal_words_async(r.data_ptr(), W, W, H, wd.data_ptr(), st)
                me.fractal_encode_mbs_async(d_org.data_ptr(), d_refs[0].data_ptr(), W,
                                            [wd.data_ptr() for wd in d_words], W, H, R, a.tol16, a.tol8,
                                            d_out.data_ptr(), st)
            step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                step()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            got = d_out.cpu().numpy().view(FRACTAL_MB)
            # CPU restatement on the first cpu_rows macroblock rows (a plane of
            # its own: bound_chk then clips at that plane's bottom edge, so the
            # comparison covers the rows above it that stay in range)
            hc = 16 * a.cpu_rows
            t0 = time.time()
            exp = ol.fractal_encode_mbs(org[:hc], [r[:hc] for r in refs], R, a.tol16, a.tol8)
            cpu_s = time.time() - t0
            split = got["mb"]["partition"] == 3
            b8 = got["b8"]["partition"][split].ravel()
            nodes = {"16x16": n_mb, "8x8": int(4 * split.sum()), "pairs": int((b8 != 0).sum()),
                     "4x4_groups": int((b8 == 3).sum())}
            # full-plane parity on the GPU result vs the oracle over the same plane, when cheap
            exact = None
            if n_mb <= 10000:
                full = ol.fractal_encode_mbs(org, refs, R, a.tol16, a.tol8)
                g, e = got.copy(), full.copy()
                g["chun"][np.isnan(g["chun"])] = 0
                e["chun"][np.isnan(e["chun"])] = 0
                exact = int((g.view(np.uint8).reshape(n_mb, -1) == e.view(np.uint8).reshape(n_mb, -1)).all(1).sum())
            print(json.dumps({
                "metric": "fractal macroblocks/sec (encode_one_macroblock quadtree, full_search)",
                "plane": f"{W}x{H}", "views": K, "R": R, "tol_16": a.tol16, "tol_8": a.tol8,
                "macroblocks": n_mb, "ms_per_plane": round(ms, 4), "value": round(n_mb / (ms * 1e-3), 1),
                "unit": "macroblocks/sec", "nodes": nodes,
                "parity_vs_restatement": {"macroblocks": n_mb if exact is not None else 0, "exact": exact},
                "cpu_baseline": {"value": round(len(exp) / cpu_s, 1), "unit": "macroblocks/sec", "cores": 1,
                                 "kind": "port",
                                 "sample": f"{len(exp)} macroblocks ({W}x{hc}), oracle/fractal_oracle.c"}}))
            sys.stdout.flush()
    me.close()


if __name__ == "__main__":
    main()
