#!/bin/bash
# round 3, call 25: the stem inside the persistent trunk launch (engine stem off): GPU tests,
# then configs[2] benches against the engine stem (AZ_TRUNK_STEM=0), alternating
set -u
mkdir -p gpurun_out/r03y
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03y/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03y/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03y/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03y/$name.log"; exit $rc; fi
}
run tests 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
B="--skip-cpu --skip-kernel"
run ts_a 300 python bench.py $B
AZ_TRUNK_STEM=0 run es_a 300 python bench.py $B
run ts_b 300 python bench.py $B
AZ_TRUNK_STEM=0 run es_b 300 python bench.py $B
exit 0
