#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 pass per group;
# --pmc never combined with sys/runtime traces).  Stops at the first failure.
# Usage (GPU box, repo root): [JMME_LIB=...] [PMC_CMD="python3 tools/bench_tq.py"] tools/pmc.sh OUTDIR [groups...]
# (PMC_CMD: the program profiled; default the headline bench)
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
GROUPS_=${@:-tcc1 tcc2 sq1 sq2}
mkdir -p "$OUT"
export TMPDIR=/tmp
declare -A G
G[sq1]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
G[sq2]="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
G[sq3]="SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_WAVES"
G[tcc1]="FETCH_SIZE"
G[tcc2]="WRITE_SIZE"
CMD=${PMC_CMD:-python3 bench.py --steps 5 --warmup 1 --headline-only}
for g in $GROUPS_; do
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc ${G[$g]} --output-format csv -d "$OUT/$g" -o p -- \
    $CMD > "$OUT/$g.log" 2>&1
done
echo pmc done
