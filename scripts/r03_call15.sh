#!/bin/bash
# round 3, call 15: in-kernel clock of the wino4 loop (s_memtime / s_memrealtime stamps):
# product, MFMA-only (AZ_W4_EXP=27) and no-MFMA (AZ_W4_EXP=4) builds
set -u
mkdir -p gpurun_out/r03o
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03o/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03o/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03o/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03o/$name.log"; exit $rc; fi
}
for v in stamp stamp_mfma stamp_nomfma; do
  for B in 1024 4096; do
    AZ_LIB_PATH=expbuild/$v/libaz_othello.so run ${v}_fp16x2_$B 200 python scripts/w4_stamps.py fp16x2 $B
  done
done
AZ_LIB_PATH=expbuild/stamp/libaz_othello.so run stamp_fp16_1024 200 python scripts/w4_stamps.py fp16 1024
exit 0
