#!/bin/bash
# Round 3: high-bit-depth sub-pel (16-bit sub-images + refinement) on the GPU.
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3m
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hbd_gpu.py \
  tests/test_subpel_gpu.py tests/test_jm_dropin_hbd_gpu.py tests/test_epzs_gpu.py tests/test_jm_dropin_epzs_gpu.py > $o/pytest.log 2>&1
echo r3m done
