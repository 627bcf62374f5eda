#!/bin/bash
# round 3, call 22: compile-time knobs of the (now default) two-board conv: weight prefetch
# distance 2 / 4 (product 3), input slices two chunks ahead, plain float ops (no packed asm)
set -u
mkdir -p gpurun_out/r03v
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03v/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03v/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03v/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03v/$name.log"; exit $rc; fi
}
export CONV_AB_ONLY=wino4
run ab_prod 300 python scripts/conv_ab.py 1024 4096
for v in v_pd2 v_pd4 v_ipd2 v_pk0; do
  AZ_LIB_PATH=expbuild/$v/libaz_othello.so run ab_$v 300 python scripts/conv_ab.py 1024 4096
done
run ab_prod2 300 python scripts/conv_ab.py 1024 4096
exit 0
