#!/bin/bash
# small-batch kernel v2: parity (small path + drop-in) then the drop-in profile
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3d
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "small or golden or contract" -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_jm_dropin_gpu.py -x -q --timeout 200 --timeout-method thread > $o/pytest_dropin.log 2>&1
SUBPEL=0 OUT=r3d/prof JMME_TRACE=$PWD/$o/trace.txt tools/prof_dropin.sh
echo r3d done
