#!/bin/bash
# Round 3: the drop-in at high bit depth, 1080p (10-bit High 10), FS and FFS, sub-pel off and on.
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3p
mkdir -p $o
timeout -k 10 300 python3 tools/bench_dropin.py --frames 3 --mode -1 --bits 10 > $o/dropin_10bit_fs.json 2> $o/a.err
timeout -k 10 300 python3 tools/bench_dropin.py --frames 3 --mode 0 --bits 10 > $o/dropin_10bit_ffs.json 2> $o/b.err
timeout -k 10 400 python3 tools/bench_dropin.py --frames 3 --mode 0 --bits 10 --subpel > $o/dropin_10bit_ffs_subpel.json 2> $o/c.err
echo r3p done
