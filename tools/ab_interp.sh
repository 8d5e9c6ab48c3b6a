#!/bin/bash
# A/B of lib variants on the quarter-pel interpolation (tools/bench_subpel.py), interleaved rounds,
# then the sub-image parity tests under each variant.  Usage (GPU box): bash tools/ab_interp.sh V1 V2 ...
set -e
mkdir -p gpurun_out/abi
for round in 1 2; do
  for v in "$@"; do
    JMME_LIB=--h.264-by-zhaodongyu_amd/lib/variants/$v/libjmme.so timeout -k 10 180 python3 tools/bench_subpel.py --iters 50 \
      > gpurun_out/abi/${v}_${round}.json 2> gpurun_out/abi/${v}_${round}.err
    python3 -c "import json; d=json.load(open('gpurun_out/abi/${v}_${round}.json')); print('$v', $round, d['interpolation'], {k: v for k, v in d.items() if k != 'interpolation'})"
  done
done
for v in "$@"; do
  JMME_LIB=--h.264-by-zhaodongyu_amd/lib/variants/$v/libjmme.so timeout -k 10 300 python3 -m pytest tests/test_subpel_gpu.py \
    -m gpu -x -q -k "sub_image or interp" > gpurun_out/abi/tests_$v.log 2>&1
  echo "$v: $(tail -1 gpurun_out/abi/tests_$v.log)"
done
