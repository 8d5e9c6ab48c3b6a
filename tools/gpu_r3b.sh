#!/bin/bash
# round 3: new GPU tests (configs[2] full frame, configs[4] frame, fractal bands),
# the bench line with its new blocks, and a traced drop-in encode.
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3b
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_hybrid_gpu.py "tests/test_fractal_pool_gpu.py::test_pool_1080p_every_4x4_full_pool" \
  -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err
JMME_TRACE=$PWD/$o/dropin_trace.txt timeout -k 10 200 python tools/bench_dropin.py > $o/dropin.json 2> $o/dropin.err
echo r3b done
