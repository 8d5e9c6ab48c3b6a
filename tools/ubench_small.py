#!/usr/bin/env python3
"""Latency of jmme_search_mbs on small batches (the drop-in's speculative
batches after a failed guess): JM's own requests of a captured case sent
`--units` macroblocks at a time, mean wall time per call.  Run once per
JMME_SMALL_VARIANT to compare the small path's variants (GPU box)."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "--h.264-by-zhaodongyu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="c2_syn_1080p_fs32")
    ap.add_argument("--units", default="1,3,8")
    ap.add_argument("--calls", type=int, default=300)
    a = ap.parse_args()
    import golden_io as g
    from jmme import MotionEstimator
    c = g.Case(a.case)
    mode = g.manifest()[a.case]["cfg_overrides"]["SearchMode"]
    (f, lst, rf, idx), = list(c.groups())[:1]
    req, unit_of, slots = c.units(idx, mode)
    out = {"variant": os.environ.get("JMME_SMALL_VARIANT", "0"), "case": a.case}
    with MotionEstimator({"SearchRange": 32, "SearchMode": mode}) as me:
        me.upload_cur(c.cur[f])
        me.upload_ref(lst, rf, c.ref[(f, lst, rf)])
        for lim, tag in ((1 << 20, "small"), (0, "throughput")):
            me.set_small_batch_limit(lim)
            for u in (int(x) for x in a.units.split(",")):
                for k in range(20):
                    me.search(mode, req[k * u:(k + 1) * u])
                t0 = time.perf_counter()
                for k in range(a.calls):
                    o = (k * 37) % (len(req) - u)
                    me.search(mode, req[o:o + u])
                out[f"{tag}_{u}_us"] = round((time.perf_counter() - t0) / a.calls * 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
