#!/bin/bash
# round 3, call 42: does the default bench's roofline / CPU-baseline work move the self-play
# window?  default vs --skip-kernel vs --skip-cpu vs both skipped, two alternating rounds
set -u
mkdir -p gpurun_out/r03ao
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ao/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ao/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ao/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ao/$name.log"; exit $rc; fi
}
for r in a b; do
  run default_$r 400 python bench.py
  run nokernel_$r 400 python bench.py --skip-kernel
  run nocpu_$r 400 python bench.py --skip-cpu
  run none_$r 300 python bench.py --skip-cpu --skip-kernel
done
exit 0
