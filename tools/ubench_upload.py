#!/usr/bin/env python3
"""Plane upload latency (jmme_upload_cur / jmme_upload_ref: JM's uint16 imgpel
rows -> pinned 8-bit staging -> one DMA), 1080p, mean per call (GPU box)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "--h.264-by-zhaodongyu_amd"))


def main():
    from jmme import MotionEstimator
    w, h = 1920, 1088
    rng = np.random.default_rng(0)
    planes = [rng.integers(0, 256, (h, w)).astype(np.uint16) for _ in range(4)]
    out = []
    with MotionEstimator({"SourceWidth": w, "SourceHeight": h, "SearchRange": 32, "SearchMode": -1}) as me:
        for name, fn in (("cur", lambda p: me.upload_cur(p)), ("ref", lambda p: me.upload_ref(0, 0, p))):
            t0 = time.perf_counter()
            fn(planes[0])
            first = (time.perf_counter() - t0) * 1e6
            n = 40
            t0 = time.perf_counter()
            for i in range(n):
                fn(planes[i & 3])
            out.append({"plane": name, "first_us": round(first, 1), "us_per_upload": round((time.perf_counter() - t0) / n * 1e6, 1)})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
