#!/bin/bash
# round 3, call 29: final bench lines on the round-3 library: configs[2] default (roofline,
# cpu_baseline), configs[3] / configs[4] / configs[1] workloads
set -u
mkdir -p gpurun_out/r03ac
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ac/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ac/$name.json" 2> "gpurun_out/r03ac/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ac/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ac/$name.err"; exit $rc; fi
}
run c3 600 python bench.py
run c4 400 python bench.py --skip-cpu --skip-kernel --workload c4
run c5 400 python bench.py --skip-cpu --skip-kernel --workload c5
run c2 400 python bench.py --skip-cpu --skip-kernel --workload c2
exit 0
