#!/bin/bash
# round 3, call 44: configs[3] / configs[4] / configs[1] workloads on the last library
set -u
mkdir -p gpurun_out/r03aq
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03aq/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03aq/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03aq/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03aq/$name.log"; exit $rc; fi
}
B="--skip-cpu --skip-kernel"
run c3 300 python bench.py $B
run c4 400 python bench.py $B --workload c4
run c5 400 python bench.py $B --workload c5
run c2 400 python bench.py $B --workload c2
exit 0
