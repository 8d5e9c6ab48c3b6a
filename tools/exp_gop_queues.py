#!/usr/bin/env python3
"""Concurrency experiment for the configs[3] GOP encoder block: the same 4K EPZS
GOPs through lencod_jmme with several encoders per GPU, under different HIP
hardware-queue limits per encoder process (GPU_MAX_HW_QUEUES) -- no stock leg.
Usage (GPU box): python3 tools/exp_gop_queues.py [gops] [per_gpu] [queue/queue/...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)
import bench_blocks  # noqa: E402

gops = int(sys.argv[1]) if len(sys.argv) > 1 else 8
per = int(sys.argv[2]) if len(sys.argv) > 2 else 8
queues = (sys.argv[3] if len(sys.argv) > 3 else "default/1/2").split("/")
for qv in queues:
    if qv == "default":
        os.environ.pop("GPU_MAX_HW_QUEUES", None)
    else:
        os.environ["GPU_MAX_HW_QUEUES"] = qv
    b = bench_blocks.encoder_gop_block(gops=gops, gop=2, per_gpu=per, preset="epzs4k", check_stock=False)
    print(json.dumps({"queues": qv, "per_gpu": per, "wall_s": b["wall_s"], "me_s_per_gop": b["me_s_per_gop"]}),
          flush=True)
