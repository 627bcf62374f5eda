#!/bin/bash
# round 3, call 17: wino4 with the step's MFMAs interleaved one by one with N VALU, one LDS
# read and one LDS write (AZ_W4_SCHED=N sched_group_barrier pattern), against the product
set -u
mkdir -p gpurun_out/r03q
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03q/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03q/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03q/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03q/$name.log"; exit $rc; fi
}
export CONV_AB_ONLY=wino4
run ab_prod 300 python scripts/conv_ab.py 1024 4096
AZ_LIB_PATH=expbuild/w4_sched2/libaz_othello.so run ab_sched2 300 python scripts/conv_ab.py 1024 4096
AZ_LIB_PATH=expbuild/w4_sched4/libaz_othello.so run ab_sched4 300 python scripts/conv_ab.py 1024 4096
run ab_prod2 300 python scripts/conv_ab.py 1024 4096
exit 0
