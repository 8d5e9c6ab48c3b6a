#!/bin/bash
# One GPU session of round evidence: VALU microbench, kernel-trace stats of
# the bench, PMC passes, and the full bench line (with the JM CPU baseline).
# Usage (GPU box): bash tools/profile_round.sh OUTDIR
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$R/${1:-gpurun_out/prof}"
mkdir -p "$OUT"
timeout -k 10 120 "$R/tools/ubench_valu" > "$OUT/ubench_valu.jsonl"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- \
  python3 bench.py --steps 20 --warmup 3 --headline-only > "$OUT/bench_under_trace.json"
bash tools/pmc.sh "$OUT/pmc" tcc1 tcc2 sq1 sq2
python3 tools/pmc_summary.py "$OUT/pmc" --traffic-json "$OUT/pmc_traffic.json" > "$OUT/pmc_summary.txt"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json"
echo profile done
