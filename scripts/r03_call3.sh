#!/bin/bash
# round 3, call 3: the triple-buffered wino4 loop (AZ_W4_TB) -- accuracy tests, A/B, chunk
# timeline; configs[4] kernel profile without graphs; the c4 tracer crash with the address map
set -u
mkdir -p gpurun_out/r03c
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03c/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03c/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03c/steps.log
  tail -2 "gpurun_out/r03c/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run tb_tests 300 env AZ_LIB_PATH=expbuild/tb/libaz_othello.so python -u -m pytest tests/test_nn_gpu.py -k "winograd4 or inference_copy" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run ab_prod 200 env CONV_AB_ONLY=wino4 python scripts/conv_ab.py 1024 4096
run ab_tb 200 env CONV_AB_ONLY=wino4 AZ_LIB_PATH=expbuild/tb/libaz_othello.so python scripts/conv_ab.py 1024 4096
run ab_prod2 200 env CONV_AB_ONLY=wino4 python scripts/conv_ab.py 1024 4096
run cst_tb 120 env AZ_LIB_PATH=expbuild/tbcst/libaz_othello.so python scripts/w4_chunk_stamps.py fp16x2 1024
P="rocprofv3 --kernel-trace --stats --output-format csv"
B="python3 bench.py --skip-cpu --skip-kernel"
run p_c5eager 300 $P -d gpurun_out/r03c/p_c5eager -o run -- $B --workload c5 --no-graph --steps 400 --warmup 1600 --warmup-exact
run p_c4maps 300 env AZ_FAULTHANDLER=1 AZ_DUMP_MAPS=gpurun_out/r03c/maps_c4.txt $P -d gpurun_out/r03c/p_c4 -o run -- $B --workload c4 --steps 1000 --warmup 3000 --warmup-exact
exit 0
