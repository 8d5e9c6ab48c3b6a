#!/usr/bin/env python3
"""getSubImagesLuma (jmme_interpolate_ref) at 1080p (1920x1088 coded): per-launch time issued from a
Python loop (one ctypes call per launch, as bench.py's subpel block does) against
the same launches replayed from a captured graph (the kernel's own rate, no host
issue in between).  Prints one JSON line.
Usage (GPU): python3 tools/ubench_interp.py [--iters 50] [--w 1920 --h 1088]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "--h.264-by-zhaodongyu_amd"))
from jmme import MotionEstimator, _lib  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1088)
    a = ap.parse_args()
    rng = np.random.default_rng(5)
    pic = rng.integers(0, 256, (a.h, a.w)).astype(np.uint16)
    dev = torch.device("cuda", 0)
    me = MotionEstimator({"SourceWidth": a.w, "SourceHeight": a.h}, device=0)
    me.upload_cur(pic)
    me.upload_ref(0, 0, pic)
    st = torch.cuda.Stream(dev)
    launch = lambda: _lib.check(_lib.lib().jmme_interpolate_ref(me._ctx, 0, 0, st.cuda_stream))  # noqa: E731
    with torch.cuda.stream(st):
        launch()
    torch.cuda.synchronize(dev)

    def events(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn(n)
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / n

    def loop(n):
        for _ in range(n):
            launch()
    ms_loop = min(events(loop, a.iters) for _ in range(3))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        loop(a.iters)
    g.replay()
    torch.cuda.synchronize(dev)
    ms_graph = min(events(lambda n: g.replay(), a.iters) for _ in range(5))
    pw, ph = a.w + 64, a.h + 40
    nbytes = a.w * a.h + 16 * pw * ph
    frac = lambda ms: round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)  # noqa: E731
    print(json.dumps({"picture": [a.w, a.h], "bytes": nbytes, "iters": a.iters,
                      "us_loop": round(ms_loop * 1e3, 2), "frac_loop": frac(ms_loop),
                      "us_graph": round(ms_graph * 1e3, 2), "frac_graph": frac(ms_graph)}))
    me.close()


if __name__ == "__main__":
    main()
