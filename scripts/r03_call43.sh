#!/bin/bash
# round 3, call 43: steady-state kernel trace (eager, as call 27) of configs[2] on the final
# library (level budget, counter update without reload)
set -u
mkdir -p gpurun_out/r03ap
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ap/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ap/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ap/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ap/$name.log"; exit $rc; fi
}
run prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_c3 -o run -- python3 bench.py --skip-cpu --skip-kernel --no-graph --steps 2000 --warmup 24000
cp /tmp/p_c3/run_kernel_stats.csv gpurun_out/r03ap/kernel_stats.csv
run tail 120 python scripts/trace_tail.py /tmp/p_c3/run_kernel_trace.csv 2000
exit 0
