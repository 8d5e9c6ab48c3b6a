#!/bin/bash
# Round 3: the drop-in at 1080p with sub-pel refinement on (JM's default; SATD quarter-pel),
# FS and FFS, stock lencod vs lencod_jmme, JM's own ME time, byte identity.
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3n
mkdir -p $o
timeout -k 10 400 python3 tools/bench_dropin.py --frames 3 --mode -1 --subpel > $o/dropin_subpel_fs.json 2> $o/fs.err
timeout -k 10 400 python3 tools/bench_dropin.py --frames 3 --mode 0 --subpel > $o/dropin_subpel_ffs.json 2> $o/ffs.err
echo r3n done
