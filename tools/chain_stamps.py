#!/usr/bin/env python3
"""Phase breakdown of the chain kernel from a -DJMME_CHAIN_PROF build
(diagnostic).  Usage: JMME_LIB=<that build> python3 tools/chain_stamps.py
Prints block 0's phase times in ns (copy-in; per step: derive, stage, sweep,
reduce; write-out) and the shader clock over the kernel."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "--h.264-by-zhaodongyu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    from jmme import FULL_SEARCH, MB_REQ, _lib
    from ubench_chain import make_chains, setup
    me, unit = setup()
    lib = _lib.lib()
    raw = (ctypes.c_ulonglong * 32)()
    for steps in (1, 4):
        ch = make_chains(steps, 1)
        rows = []
        for _ in range(50):
            me.search_chains(FULL_SEARCH, np.zeros(0, MB_REQ), ch)
            lib.jmme_debug_chain_prof(raw)
            rows.append(np.array(raw[:], np.int64))
        a = np.array(rows[10:])
        t = (a[:, :19] - a[:, :1]) * 10
        names = ["copy-in"]
        idx = [1]
        for k in range(steps):
            names += [f"s{k} derive", f"s{k} stage", f"s{k} sweep", f"s{k} reduce"]
            idx += [2 + 4 * k, 3 + 4 * k, 4 + 4 * k, 5 + 4 * k]
        names.append("write-out")
        idx.append(18)
        prev = 0
        parts = []
        for nm, i in zip(names, idx):
            m = float(np.median(t[:, i]))
            parts.append(f"{nm} {m - prev:.0f}")
            prev = m
        clk = np.median((a[:, 31] - a[:, 30]) / np.maximum(1, (a[:, 18] - a[:, 0]) * 10)) * 1e3
        print(f"steps {steps}: total {prev:.0f} ns, shader clock ~{clk:.0f} MHz |", ", ".join(parts))


if __name__ == "__main__":
    main()
