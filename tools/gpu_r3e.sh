#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3e
mkdir -p $o
for v in 0 1 2 3; do JMME_SMALL_VARIANT=$v timeout -k 10 120 python tools/ubench_small.py >> $o/ubench_small.jsonl; done
JMME_SMALL_VARIANT=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -k "small" -x -q --timeout 100 --timeout-method thread > $o/pytest_v1.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_gop_launch.py -x -q --timeout 150 --timeout-method thread > $o/pytest_gop.log 2>&1
echo r3e done
