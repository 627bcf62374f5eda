#!/bin/bash
# round 3, call 2: chunk timeline of the wino4 conv; diet vs round-2 loop bit-identity; the
# configs[4] rocprofv3 crash bisected (stops at the first fault)
set -u
mkdir -p gpurun_out/r03b
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03b/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03b/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03b/steps.log
  tail -2 "gpurun_out/r03b/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run cst_fp16x2 120 env AZ_LIB_PATH=expbuild/cstamp/libaz_othello.so python scripts/w4_chunk_stamps.py fp16x2 1024
run cst_fp16 120 env AZ_LIB_PATH=expbuild/cstamp/libaz_othello.so python scripts/w4_chunk_stamps.py fp16 1024
run ab_new 200 env CONV_AB_ONLY=wino4 python scripts/conv_ab.py 1024
run ab_old 200 env CONV_AB_ONLY=wino4 AZ_LIB_PATH=expbuild/diet0/libaz_othello.so python scripts/conv_ab.py 1024
P="rocprofv3 --kernel-trace --stats --output-format csv"
B="python3 bench.py --skip-cpu --skip-kernel --steps 1000 --warmup 3000 --warmup-exact"
run p_c4 300 $P -d gpurun_out/r03b/p_c4 -o run -- $B --workload c4
run p_c5x2 300 $P -d gpurun_out/r03b/p_c5x2 -o run -- $B --workload c5 --conv-precision fp16x2
run p_c5w4 300 env AZ_CONV_ALGO=wino4 $P -d gpurun_out/r03b/p_c5w4 -o run -- $B --workload c5
run p_c5eager 300 $P -d gpurun_out/r03b/p_c5eager -o run -- $B --workload c5 --no-graph --steps 300 --warmup 300
run p_c5 300 env AZ_FAULTHANDLER=1 AZ_DUMP_MAPS=gpurun_out/r03b/maps_c5.txt $P -d gpurun_out/r03b/p_c5 -o run -- $B --workload c5
exit 0
