#!/usr/bin/env python3
"""The bench's in-encoder block alone (stock lencod vs lencod_jmme, 1080p FS and
FFS; add EPZS with --epzs), one JSON line.  GPU box."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)

import bench_blocks  # noqa: E402

modes = [(-1, "FS"), (0, "FFS")] + ([(3, "EPZS")] if "--epzs" in sys.argv else [])
print(json.dumps(bench_blocks.dropin_block(modes=tuple(modes))))
