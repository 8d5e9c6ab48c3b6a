#!/bin/bash
# A/B lib variants on the EPZS bench (one process each, interleaved rounds).
set -e
for round in 1 2; do
  for v in "$@"; do
    JMME_LIB=--h.264-by-zhaodongyu_amd/lib/variants/$v/libjmme.so timeout -k 10 120 python3 tools/bench_epzs.py --iters 30 > gpurun_out/abe_${v}_${round}.json 2> gpurun_out/abe_${v}_${round}.err
    python3 -c "import json; d=json.load(open('gpurun_out/abe_${v}_${round}.json')); print('$v', $round, d['ms_per_frame'], d['parity_vs_jm']['exact'])"
  done
done
