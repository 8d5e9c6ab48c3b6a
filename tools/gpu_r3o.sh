#!/bin/bash
# Round 3: 256x8 interpolation tiles -- sub-image parity (8/16-bit), sub-pel bench
# block, rocprof kernel stats of the interpolation, then the sub-pel drop-in at 1080p.
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3o
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_subpel_gpu.py \
  tests/test_hbd_gpu.py -k "sub_images or refinement or chained" > $o/pytest.log 2>&1
timeout -k 10 200 python3 tools/bench_subpel.py --no-cpu > $o/bench_subpel.json 2> $o/bench_subpel.err
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$o/trace" -o t -- \
  python3 tools/bench_subpel.py --iters 20 --no-cpu > $o/bench_subpel_traced.json 2>&1
bash tools/gpu_r3n.sh
echo r3o done
