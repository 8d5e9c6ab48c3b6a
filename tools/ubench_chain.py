#!/usr/bin/env python3
"""Latency of jmme_search_mbs_chains (the drop-in's chained guesses inside a
macroblock): chains of 1..4 steps with fixed neighbours, alone and beside a
one-unit batch, mean wall time per call (GPU box)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "--h.264-by-zhaodongyu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


W, H, R = 1920, 1088, 32
SLOTS = {1: [5], 2: [9, 11], 4: [25, 26, 29, 30]}


def setup():
    from jmme import MotionEstimator, synth
    from test_gpu_parity import _random_units
    luma = synth.luma_sequence(W, H, 2, seed=5, gmv=(0, 0), adversarial=True)
    me = MotionEstimator({"SearchRange": R, "SearchMode": -1, "RDOptimization": 0})
    me.upload_cur(luma[1])
    me.upload_ref(0, 0, luma[0])
    return me, _random_units(np.random.default_rng(1), W, H, 1, R)


def make_chains(steps, n_chains, r=R):
    """n_chains chains of `steps` steps (slots SLOTS[steps]) with fixed neighbours, range r"""
    from jmme._lib import CHAIN
    ch = np.zeros(n_chains, CHAIN)
    for i in range(n_chains):
        ch[i]["mb_x"], ch[i]["mb_y"] = 16 * (5 + i), 16 * 7
        ch[i]["n_steps"] = steps
        ch[i]["lambda"] = 100
        ch[i]["mv_lim_x0"], ch[i]["mv_lim_x1"], ch[i]["mv_lim_y0"], ch[i]["mv_lim_y1"] = -2048, 2047, -512, 511
        for k, s in enumerate(SLOTS[steps]):
            st = ch[i]["steps"][k]
            st["slot"] = s
            for j in range(3):
                st["nb"][j]["src"] = k - 1 if (k and j == 0) else -2
                st["nb"][j]["mv_x"], st["nb"][j]["mv_y"] = 4 * (3 * j - 2), 4 * (j - 1)
            st["sr_min_x"] = st["sr_min_y"] = -4 * r
            st["sr_max_x"] = st["sr_max_y"] = 4 * r
            ch[i]["steps"][k] = st
    return ch


def main():
    from jmme import FULL_SEARCH, MB_REQ
    out = []
    me, unit = setup()
    with me:
        for steps in SLOTS:
            for n_chains in (1, 4):
                ch = make_chains(steps, n_chains)
                for batch in (False, True):
                    req = unit if batch else np.zeros(0, MB_REQ)
                    for _ in range(20):
                        me.search_chains(FULL_SEARCH, req, ch)
                    t0 = time.perf_counter()
                    n = 300
                    for _ in range(n):
                        me.search_chains(FULL_SEARCH, req, ch)
                    us = (time.perf_counter() - t0) / n * 1e6
                    out.append({"steps": steps, "chains": n_chains, "with_batch": batch, "us_per_call": round(us, 1)})
        # fixed costs: one step at range 1 (a 3x3 window)
        ch = make_chains(1, 1, r=1)
        for _ in range(20):
            me.search_chains(FULL_SEARCH, np.zeros(0, MB_REQ), ch)
        t0 = time.perf_counter()
        for _ in range(300):
            me.search_chains(FULL_SEARCH, np.zeros(0, MB_REQ), ch)
        out.append({"steps": 1, "chains": 1, "range": 1, "us_per_call": round((time.perf_counter() - t0) / 300 * 1e6, 1)})
        # the batch alone, for reference
        for _ in range(20):
            me.search(FULL_SEARCH, unit)
        t0 = time.perf_counter()
        for _ in range(300):
            me.search(FULL_SEARCH, unit)
        out.append({"batch_alone_us": round((time.perf_counter() - t0) / 300 * 1e6, 1)})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
