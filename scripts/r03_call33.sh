#!/bin/bash
# round 3, call 33: streaming (nt) cache hints on the wino4 conv's activation traffic
# (AZ_W4_NT builds, scripts/build_variants.py) -- conv A/B, HBM reads per launch (FETCH_SIZE),
# then the configs[2] bench with the default library and the best variant, alternating
set -u
mkdir -p gpurun_out/r03ag
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ag/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ag/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ag/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ag/$name.log"; exit $rc; fi
}
export CONV_AB_ONLY=wino4
for r in a b; do
  run ab_base_$r 200 python scripts/conv_ab.py 1024
  for v in nt1 nt2 nt3; do
    AZ_LIB_PATH=expbuild/$v/libaz_othello.so run ab_${v}_$r 200 python scripts/conv_ab.py 1024
  done
done
for v in base nt1 nt2 nt3; do
  L=alphazero-othello_amd/libaz_othello.so; [ $v != base ] && L=expbuild/$v/libaz_othello.so
  AZ_LIB_PATH=$L run pmc_$v 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03ag/pmc_$v -o pmc -- \
    python3 scripts/conv_one.py az_conv3x3_wino4_gpu fp16x2 1024 20
done
B="--skip-cpu --skip-kernel"
run c3_base_a 300 python bench.py $B
AZ_LIB_PATH=expbuild/nt1/libaz_othello.so run c3_nt1_a 300 python bench.py $B
AZ_LIB_PATH=expbuild/nt3/libaz_othello.so run c3_nt3_a 300 python bench.py $B
run c3_base_b 300 python bench.py $B
AZ_LIB_PATH=expbuild/nt1/libaz_othello.so run c3_nt1_b 300 python bench.py $B
AZ_LIB_PATH=expbuild/nt3/libaz_othello.so run c3_nt3_b 300 python bench.py $B
exit 0
