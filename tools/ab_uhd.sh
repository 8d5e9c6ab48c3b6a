#!/bin/bash
# A/B lib variants on the 1080p step and the 4K (uhd) block of bench.py.
set -e
for round in 1 2; do
  for v in "$@"; do
    JMME_LIB=--h.264-by-zhaodongyu_amd/lib/variants/$v/libjmme.so timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-subpel > gpurun_out/abu_${v}_${round}.json 2> gpurun_out/abu_${v}_${round}.err
    python3 -c "import json; d=json.load(open('gpurun_out/abu_${v}_${round}.json')); print('$v', $round, d['ms_per_step'], d['roofline']['kernel_ms'], d['uhd']['ms_per_frame'], d['uhd']['kernel_ms'], d['parity']['bit_exact'], d['uhd']['parity']['bit_exact'])"
  done
done
