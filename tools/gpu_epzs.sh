#!/bin/bash
# EPZS GPU session: parity tests (integer + quarter-pel grid), EPZS benches.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/epzs
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_epzs_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/epzs/pytest.log 2>&1
timeout -k 10 300 python tools/bench_epzs.py > gpurun_out/epzs/bench.json 2> gpurun_out/epzs/bench.err
timeout -k 10 300 python tools/bench_epzs.py --case epzs_grid_syn_1080p_r32 > gpurun_out/epzs/bench_grid.json 2> gpurun_out/epzs/bench_grid.err
timeout -k 10 300 python tools/bench_epzs.py --case epzs_syn_4k_r32 > gpurun_out/epzs/bench_4k.json 2> gpurun_out/epzs/bench_4k.err
echo epzs done
