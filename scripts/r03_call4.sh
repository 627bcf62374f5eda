#!/bin/bash
# round 3, call 4: wino4 loop variants A/B (triple buffer, A prefetch distance 2, unrolled
# groups) at the bench batch, interleaved with the product build
set -u
mkdir -p gpurun_out/r03d
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03d/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03d/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03d/steps.log
  tail -2 "gpurun_out/r03d/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run t_apdu 300 env AZ_LIB_PATH=expbuild/tbapdu/libaz_othello.so python -u -m pytest tests/test_nn_gpu.py -k "winograd4_fp16x2" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for rep in 1 2; do
  run ab_prod_$rep 200 env CONV_AB_ONLY=wino4 python scripts/conv_ab.py 1024 4096
  for v in tb tbu tbapd tbapdu; do
    run ab_${v}_$rep 200 env CONV_AB_ONLY=wino4 AZ_LIB_PATH=expbuild/$v/libaz_othello.so python scripts/conv_ab.py 1024 4096
  done
done
run cst_apdu 120 env AZ_LIB_PATH=expbuild/tbapducst/libaz_othello.so python scripts/w4_chunk_stamps.py fp16x2 1024
exit 0
