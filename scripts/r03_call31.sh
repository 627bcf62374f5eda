#!/bin/bash
# round 3, call 31: the bench's kernel timing on fence-free HIP events (the default events'
# system-scope cache writeback reported beside), then the same bench command under rocprofv3
# (eager: the tracer faulted on graph replay with this library) for the kernels' own durations
set -u
mkdir -p gpurun_out/r03ae
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ae/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ae/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ae/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ae/$name.log"; exit $rc; fi
}
run bench 600 python bench.py
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_k -o run -- python3 bench.py --skip-cpu --no-graph --steps 200 --warmup 200 --warmup-exact
cp /tmp/p_k/run_kernel_stats.csv gpurun_out/r03ae/kernel_stats.csv
cp /tmp/p_k/run_kernel_trace.csv gpurun_out/r03ae/kernel_trace.csv
exit 0
