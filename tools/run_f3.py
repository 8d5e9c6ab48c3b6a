#!/usr/bin/env python3
"""bench.py's (f)3 block alone (GPU box): one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)
import bench_blocks  # noqa: E402

print(json.dumps(bench_blocks.f3_block()))
