#!/bin/bash
# round 3, call 26: expansion fused into the next step's select launch (az_select_move_expand):
# GPU tests, then configs[2] / configs[3] benches against the separate k_expand
# (AZ_FUSE_EXPAND=0), alternating
set -u
mkdir -p gpurun_out/r03z
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03z/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03z/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03z/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03z/$name.log"; exit $rc; fi
}
run tests 800 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
B="--skip-cpu --skip-kernel"
run fx_a 300 python bench.py $B
AZ_FUSE_EXPAND=0 run sx_a 300 python bench.py $B
run fx_b 300 python bench.py $B
AZ_FUSE_EXPAND=0 run sx_b 300 python bench.py $B
run fx_c4 300 python bench.py $B --workload c4
AZ_FUSE_EXPAND=0 run sx_c4 300 python bench.py $B --workload c4
exit 0
