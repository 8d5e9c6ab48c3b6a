#!/bin/bash
# Fractal pool-search GPU session: parity tests, then the full-pool bench lines.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pool
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fractal_pool_gpu.py tests/test_fractal_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pool/pytest.log 2>&1
timeout -k 10 300 python tools/bench_fractal.py --ranges 7,16,32,full --iters 3 --check-windowed > gpurun_out/pool/bench.jsonl 2> gpurun_out/pool/bench.err
timeout -k 10 200 python tools/bench_fractal.py --ranges full --iters 1 --content unrelated > gpurun_out/pool/bench_unrelated.jsonl 2> gpurun_out/pool/bench_unrelated.err
echo pool done
