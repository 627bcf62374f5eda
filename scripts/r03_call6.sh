#!/bin/bash
# round 3, call 6: steady-state kernel profile of configs[2] (trace reduced on the box), the
# default bench line with the whole-host cpu_baseline, configs[1]/[3]/[4] bench lines
set -u
mkdir -p gpurun_out/r03f
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03f/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03f/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03f/steps.log
  tail -2 "gpurun_out/r03f/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run prof_c3 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c3 -o run -- python3 bench.py --skip-cpu --skip-kernel --steps 2000 --warmup 24000
run tail_c3 120 python scripts/trace_tail.py /tmp/prof_c3/run_kernel_trace.csv 2000
cp /tmp/prof_c3/run_kernel_stats.csv gpurun_out/r03f/prof_c3_kernel_stats.csv
run bench_default 500 python bench.py
run bench_c4 400 python bench.py --workload c4 --skip-cpu --skip-kernel --steps 4000
run bench_c5 400 python bench.py --workload c5 --skip-cpu --skip-kernel --steps 8000
run bench_c2 400 python bench.py --workload c2 --skip-cpu --skip-kernel --steps 4000
exit 0
