#!/bin/bash
# round 3, call 14: wino4 after the VALU diet -- weight-stream ablations (half / no weight
# loads) and SQ counters of the product loop
set -u
mkdir -p gpurun_out/r03n
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03n/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03n/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03n/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03n/$name.log"; exit $rc; fi
}
export CONV_AB_ONLY=wino4
run ab_prod 300 python scripts/conv_ab.py 1024 4096
AZ_LIB_PATH=expbuild/w4_exp32/libaz_othello.so run ab_exp32 300 python scripts/conv_ab.py 1024 4096
AZ_LIB_PATH=expbuild/w4_exp1/libaz_othello.so run ab_exp1 300 python scripts/conv_ab.py 1024 4096
run ab_prod2 300 python scripts/conv_ab.py 1024 4096
unset CONV_AB_ONLY
TAG=r03n_wino4_fp16x2 run sq 400 bash scripts/pmc_conv_sq.sh az_conv3x3_wino4_gpu fp16x2 1024
exit 0
