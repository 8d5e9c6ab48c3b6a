#!/bin/bash
# One GPU lease, any sequence of steps, each under its own time limit, stopping at
# the first failure (gpurun: `gpurun --timeout 1200 -- bash tools/gpu_run.sh OUT STEP...`).
#
#   OUT                 output directory under gpurun_out/
#   tests[:FILES]       pytest -m gpu (all GPU tests, or the comma-separated test files / node ids)
#   smoke               __graft_entry__.smoke()
#   trace               rocprofv3 --kernel-trace --stats of the headline bench (20 steps)
#   pmc                 the four PMC passes of the headline bench + their summary (tools/pmc.sh)
#   bench[:ARGS]        python bench.py (ARGS: comma-separated extra arguments)
#   dropin:MODE[:ARGS]  tools/bench_dropin.py --mode MODE (ARGS: comma-separated extra arguments)
#   py:SCRIPT[:ARGS]    python3 SCRIPT (a tools/ benchmark) with comma-separated arguments
#   env:NAME=VALUE      export NAME=VALUE for the steps after it (env:NAME= unsets)
#   info                the box's host placement facts (CPUs, affinity, cgroup limits, the GPU's NUMA cores)
set -e
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/$1
shift
mkdir -p "$O"
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=""
  [ "$kind" != "$step" ] && arg=${step#*:}
  echo "[$n] $step" >&2
  case $kind in
    tests)
      sel="tests"
      [ -n "$arg" ] && sel=$(echo "$arg" | tr ',' ' ')
      timeout -k 10 900 python -u -m pytest $sel -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$O/pytest_gpu_$n.log" 2>&1 ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o t -- \
        python3 bench.py --steps 20 --warmup 3 --headline-only > "$O/bench_under_trace.json" ;;
    pmc)
      bash tools/pmc.sh "$O/pmc" tcc1 tcc2 sq1 sq2
      python3 tools/pmc_summary.py "$O/pmc" --traffic-json "$O/pmc_traffic.json" > "$O/pmc_summary.txt" ;;
    bench)
      timeout -k 10 1100 python3 bench.py $(echo "$arg" | tr ',' ' ') > "$O/bench_$n.json" 2> "$O/bench_$n.err" ;;
    info)
      { nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))";
        cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null || true;
        python3 -c "import sys; sys.path.insert(0, 'tools'); sys.path.insert(0, 'tests'); import bench_blocks as b; print('gpu0 local cpus', b._kfd_gpu_cpus(0)); print('placement', b.gpu_local_cpus(0, 1))";
        lscpu | head -30; } > "$O/info.txt" 2>&1 ;;
    dropin)
      mode=${arg%%:*}
      extra=""
      [ "$mode" != "$arg" ] && extra=$(echo "${arg#*:}" | tr ',' ' ')
      timeout -k 10 600 python3 tools/bench_dropin.py --mode "$mode" $extra > "$O/dropin_${n}_m$mode.json" \
        2> "$O/dropin_${n}_m$mode.err" ;;
    py)
      script=${arg%%:*}
      extra=""
      [ "$script" != "$arg" ] && extra=$(echo "${arg#*:}" | tr ',' ' ')
      timeout -k 10 600 python3 "$script" $extra > "$O/py_$n.out" 2> "$O/py_$n.err" ;;
    env)
      name=${arg%%=*}
      if [ -n "${arg#*=}" ]; then export "$arg"; else unset "$name"; fi ;;
    *)
      echo "unknown step $step" >&2
      exit 2 ;;
  esac
done
echo "gpu_run $O done"
