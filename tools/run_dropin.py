#!/usr/bin/env python3
"""The bench's in-encoder block alone (stock lencod vs lencod_jmme on the 1080p
clip), one JSON line.  GPU box.
Usage: python3 tools/run_dropin.py [TAG ...] [--reps N] [--host N]
TAG: FS FFS FS_subpel FFS_subpel EPZS (default: all of bench_blocks.dropin_modes())."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)

import bench_blocks  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("tags", nargs="*")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--host", type=int, default=None, help="concurrent stock encoders (default: host_cores())")
a = ap.parse_args()
modes = [m for m in bench_blocks.dropin_modes() if not a.tags or m[0] in a.tags]
print(json.dumps(bench_blocks.dropin_block(modes=tuple(modes), reps=a.reps, host_procs=a.host)))
