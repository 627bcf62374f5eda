#!/bin/bash
# round 3, call 20: configs[2] bench with two-board wino4 workgroups (AZ_W4_BOARDS=2) against
# the four-board default, same box, alternating
set -u
mkdir -p gpurun_out/r03t
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03t/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03t/$name.json" 2> "gpurun_out/r03t/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03t/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03t/$name.err"; exit $rc; fi
}
B="--skip-cpu --skip-kernel"
run b4a 300 python bench.py $B
AZ_W4_BOARDS=2 run b2a 300 python bench.py $B
run b4b 300 python bench.py $B
AZ_W4_BOARDS=2 run b2b 300 python bench.py $B
exit 0
