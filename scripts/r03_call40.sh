#!/bin/bash
# round 3, call 40: the level budget (AZ_SEL_LEVELS = 14, K = 1) as the product: GPU tests and
# smoke on it, then configs[2] against the same library without it (AZ_SEL_LEVELS=0 build),
# three alternating rounds
set -u
mkdir -p gpurun_out/r03am
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03am/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03am/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03am/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03am/$name.log"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run smoke 200 python -c 'import __graft_entry__ as g; g.smoke()'
B="--skip-cpu --skip-kernel"
for r in a b c; do
  run lv14_$r 300 python bench.py $B
  AZ_LIB_PATH=expbuild/lv0/libaz_othello.so run lv0_$r 300 python bench.py $B
done
exit 0
