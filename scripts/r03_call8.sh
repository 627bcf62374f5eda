#!/bin/bash
# round 3, call 8: ablations of the current wino4 loop (AZ_W4_EXP bits: 1 no weight loads,
# 2 no transform / input work, 4 no MFMAs, 8 no barrier, 16 no A-fragment reads) and the
# SQ counters of the product kernel (fp16x2, B = 1,024)
set -u
mkdir -p gpurun_out/r03h
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03h/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03h/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03h/steps.log
  tail -1 "gpurun_out/r03h/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run ab_prod 200 env CONV_AB_ONLY=wino4 python scripts/conv_ab.py 1024 4096
for v in exp1 exp2 exp3 exp4 exp6 exp19 exp27; do
  run ab_$v 200 env CONV_AB_ONLY=wino4 AZ_LIB_PATH=expbuild/$v/libaz_othello.so python scripts/conv_ab.py 1024 4096
done
run ab_prod2 200 env CONV_AB_ONLY=wino4 python scripts/conv_ab.py 1024 4096
run sq 400 bash scripts/pmc_conv_sq.sh az_conv3x3_wino4_gpu fp16x2 1024
run sqsum 60 python scripts/sq_summary.py gpurun_out/sq_wino4_fp16x2
cp -r gpurun_out/sq_wino4_fp16x2_* gpurun_out/r03h/ 2>/dev/null
exit 0
