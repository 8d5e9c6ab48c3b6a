#!/bin/bash
# Profile the fractal full-pool search: kernel trace + stats, then SQ counter passes (one --pmc group per run).
set -e
cd "$(dirname "$0")/.."
OUT=gpurun_out/poolprof
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 tools/bench_fractal.py --ranges full --iters 2 --cpu-seconds 0.2"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o p -- $CMD > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq1 -o p -- $CMD > $OUT/sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq2 -o p -- $CMD > $OUT/sq2.log 2>&1
echo prof done
