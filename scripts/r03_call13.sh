#!/bin/bash
# round 3, call 13: conv_wino4 with packed / mixed-precision transform ops and zero-free
# accumulator starts -- bit identity and timing A/B against the previous loop, nn tests, bench
set -u
mkdir -p gpurun_out/r03m
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03m/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03m/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03m/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03m/$name.log"; exit $rc; fi
}
export CONV_AB_ONLY=wino4
AZ_LIB_PATH=expbuild/w4_old/libaz_othello.so run ab_old1 300 python scripts/conv_ab.py 1024 4096
run ab_new1 300 python scripts/conv_ab.py 1024 4096
AZ_LIB_PATH=expbuild/w4_zf/libaz_othello.so run ab_zf 300 python scripts/conv_ab.py 1024 4096
AZ_LIB_PATH=expbuild/w4_old/libaz_othello.so run ab_old2 300 python scripts/conv_ab.py 1024 4096
run ab_new2 300 python scripts/conv_ab.py 1024 4096
unset CONV_AB_ONLY
run nn_tests 600 python -u -m pytest tests/test_nn_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
run bench_new 400 python bench.py --skip-cpu --skip-kernel --steps 4000
AZ_LIB_PATH=expbuild/w4_old/libaz_othello.so run bench_old 400 python bench.py --skip-cpu --skip-kernel --steps 4000
run bench_new2 400 python bench.py --skip-cpu --skip-kernel --steps 4000
exit 0
