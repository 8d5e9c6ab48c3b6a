#!/bin/bash
# Sub-pel GPU session: parity tests, bench, kernel-trace profile (each step time-limited).
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/subpel
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_subpel_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/subpel/pytest.log 2>&1
timeout -k 10 300 python tools/bench_subpel.py > gpurun_out/subpel/bench.json 2> gpurun_out/subpel/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/subpel/trace -o t -- python3 tools/bench_subpel.py --iters 20 --no-cpu > gpurun_out/subpel/bench_trace.json 2> gpurun_out/subpel/trace.err
echo subpel done
