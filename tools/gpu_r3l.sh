#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3l
mkdir -p $o
timeout -k 10 200 python bench.py --workload fractal --steps 5 --warmup 1 > $o/fractal_n1.json 2> $o/fractal_n1.err
echo r3l done
