#!/bin/bash
# round 3, call 18: wino4 ping-pong chunk orders (AZ_W4_PP: 1 = waves 0-3 MFMA-first / 4-7
# transform-first, 2 = all MFMA-first, 3 = all transform-first) against the product order;
# k_step2 variants (AZ_STEP_EARLY, AZ_LEGAL_V2) same-box
set -u
mkdir -p gpurun_out/r03r
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03r/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03r/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03r/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03r/$name.log"; exit $rc; fi
}
export CONV_AB_ONLY=wino4
for v in w4pp0 w4pp1 w4pp2 w4pp3 w4pp0; do
  AZ_LIB_PATH=expbuild/$v/libaz_othello.so run ab_$v 300 python scripts/conv_ab.py 1024 4096
done
run step_ab 300 python scripts/step_ab.py expbuild/st_base/libaz_othello.so expbuild/st_early/libaz_othello.so expbuild/st_l2/libaz_othello.so expbuild/st_both/libaz_othello.so
exit 0
