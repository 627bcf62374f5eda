#!/bin/bash
# round 3, call 24: the persistent fp16x2 trunk (az_trunk_wino4_gpu): NN GPU tests, then
# configs[2] and configs[3] benches with and without it (AZ_FUSE_TRUNK4=0), alternating
set -u
mkdir -p gpurun_out/r03x
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03x/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03x/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03x/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03x/$name.log"; exit $rc; fi
}
run nn_tests 600 python -u -m pytest tests/test_nn_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
B="--skip-cpu --skip-kernel"
run c3_t4a 300 python bench.py $B
AZ_FUSE_TRUNK4=0 run c3_l_a 300 python bench.py $B
run c3_t4b 300 python bench.py $B
AZ_FUSE_TRUNK4=0 run c3_l_b 300 python bench.py $B
run c4_t4 300 python bench.py $B --workload c4
AZ_FUSE_TRUNK4=0 run c4_l 300 python bench.py $B --workload c4
exit 0
