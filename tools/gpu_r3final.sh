#!/bin/bash
# Round-3 closing evidence on one GPU: the full GPU suite, smoke, a kernel-trace
# profile of the headline bench, PMC passes, and the full bench line.
set -e
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r3final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o t -- \
  python3 bench.py --steps 20 --warmup 3 --headline-only > $O/bench_under_trace.json
bash tools/pmc.sh "$O/pmc" tcc1 tcc2 sq1 sq2
python3 tools/pmc_summary.py "$O/pmc" --traffic-json "$O/pmc_traffic.json" > "$O/pmc_summary.txt"
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
echo r3final done
