#!/bin/bash
# A/B the lib variants on the bench (one process each, interleaved rounds).
set -e
for round in 1 2; do
  for v in "$@"; do
    JMME_LIB=--h.264-by-zhaodongyu_amd/lib/variants/$v/libjmme.so timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --headline-only > gpurun_out/ab_${v}_${round}.json 2> gpurun_out/ab_${v}_${round}.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${v}_${round}.json')); print('$v', $round, d['ms_per_step'], d['roofline']['kernel_ms'], d['parity']['bit_exact'])"
  done
done
