#!/bin/bash
# Round-start GPU check: gpu tests, smoke, bench (each step time-limited, chained).
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/check
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/check/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/check/bench.json 2> gpurun_out/check/bench.err
echo check done
