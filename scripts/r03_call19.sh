#!/bin/bash
# round 3, call 19: what bounds the wino4 loop -- half the weight wave-loads (AZ_W4_EXP=32:
# only waves 0-3 load, results wrong), two-board workgroups two per CU (AZ_W4_BOARDS=2),
# four waves of two row tiles (AZ_W4_NRT=2), against the product
set -u
mkdir -p gpurun_out/r03s
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03s/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03s/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03s/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03s/$name.log"; exit $rc; fi
}
export CONV_AB_ONLY=wino4
run ab_prod 300 python scripts/conv_ab.py 1024 4096
AZ_LIB_PATH=expbuild/w4exp32/libaz_othello.so run ab_exp32 300 python scripts/conv_ab.py 1024 4096
AZ_W4_BOARDS=2 run ab_boards2 300 python scripts/conv_ab.py 1024 4096
AZ_W4_NRT=2 run ab_nrt2 300 python scripts/conv_ab.py 1024 4096
run ab_prod2 300 python scripts/conv_ab.py 1024 4096
exit 0
