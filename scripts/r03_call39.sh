#!/bin/bash
# round 3, call 39: the level budget (AZ_SEL_LEVELS builds) with a larger descent cap
# (AZ_MAX_DESCENTS), configs[2], three alternating rounds
set -u
mkdir -p gpurun_out/r03al
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03al/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03al/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03al/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03al/$name.log"; exit $rc; fi
}
B="--skip-cpu --skip-kernel"
for r in a b c; do
  run base_$r 300 python bench.py $B
  AZ_LIB_PATH=expbuild/lv14/libaz_othello.so run lv14_$r 300 python bench.py $B
  AZ_MAX_DESCENTS=8 AZ_LIB_PATH=expbuild/lv14/libaz_othello.so run lv14md8_$r 300 python bench.py $B
  AZ_MAX_DESCENTS=8 AZ_LIB_PATH=expbuild/lv10/libaz_othello.so run lv10md8_$r 300 python bench.py $B
done
exit 0
