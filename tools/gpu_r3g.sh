#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3g
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "small or contract or golden" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
timeout -k 10 120 python tools/ubench_small.py > $o/ubench_small.jsonl
SUBPEL=0 OUT=r3g/prof tools/prof_dropin.sh > /dev/null
echo r3g done
