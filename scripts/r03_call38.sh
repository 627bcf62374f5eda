#!/bin/bash
# round 3, call 38: a level budget for the select wave's descents (AZ_SEL_LEVELS builds: another
# descent only while the launch's descents walked fewer levels) against the product (cap of 4
# descents alone), configs[2], alternating
set -u
mkdir -p gpurun_out/r03ak
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ak/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ak/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ak/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ak/$name.log"; exit $rc; fi
}
B="--skip-cpu --skip-kernel"
for r in a b; do
  run base_$r 300 python bench.py $B
  for v in lv10 lv14 lv18; do
    AZ_LIB_PATH=expbuild/$v/libaz_othello.so run ${v}_$r 300 python bench.py $B
  done
done
exit 0
