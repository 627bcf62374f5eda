#!/bin/bash
# round 3, call 35: what bounds the two-board wino4 conv (AZ_W4_EXP bits: 1 no weight loads,
# 2 no transform/input work, 4 no MFMAs, 8 no chunk barrier -- results wrong) and two
# scheduling knobs on it (AZ_W4_PRIO=2 MFMA-cluster priority, AZ_W4_SCHED=2/4 interleave);
# conv_ab.py at B = 1,024, two alternating rounds
set -u
mkdir -p gpurun_out/r03ai
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ai/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ai/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ai/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ai/$name.log"; exit $rc; fi
}
export CONV_AB_ONLY=wino4
for r in a b; do
  run ab_base_$r 200 python scripts/conv_ab.py 1024
  for v in e1 e2 e4 e8 p2 s2 s4; do
    AZ_LIB_PATH=expbuild/$v/libaz_othello.so run ab_${v}_$r 200 python scripts/conv_ab.py 1024
  done
done
exit 0
