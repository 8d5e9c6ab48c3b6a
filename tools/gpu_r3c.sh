#!/bin/bash
# round 3: small-batch path parity, drop-in parity, bench (all blocks)
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3c
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_jm_dropin_gpu.py -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
JMME_TRACE=$PWD/$o/dropin_trace.txt timeout -k 10 400 python bench.py > $o/bench.json 2> $o/bench.err
echo r3c done
