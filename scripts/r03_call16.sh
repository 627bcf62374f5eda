#!/bin/bash
# round 3, call 16: wino4 prefetch depths -- input slices two chunks ahead (AZ_W4_IPD3=2),
# weights four steps ahead (AZ_W4_PD3=4), against the product
set -u
mkdir -p gpurun_out/r03p
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03p/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03p/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03p/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03p/$name.log"; exit $rc; fi
}
export CONV_AB_ONLY=wino4
run ab_prod 300 python scripts/conv_ab.py 1024 4096
AZ_LIB_PATH=expbuild/w4_ipd2/libaz_othello.so run ab_ipd2 300 python scripts/conv_ab.py 1024 4096
AZ_LIB_PATH=expbuild/w4_pd4/libaz_othello.so run ab_pd4 300 python scripts/conv_ab.py 1024 4096
run ab_prod2 300 python scripts/conv_ab.py 1024 4096
AZ_LIB_PATH=expbuild/w4_ipd2/libaz_othello.so run ab_ipd2b 300 python scripts/conv_ab.py 1024 4096
exit 0
