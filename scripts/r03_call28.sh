#!/bin/bash
# round 3, call 28: the heads-fused last conv on two-board workgroups (heads scratch moved past
# the conv's LDS): GPU tests, then configs[2] benches against the four-board heads conv
# (AZ_W4_HEADS_BOARDS=4), alternating
set -u
mkdir -p gpurun_out/r03ab
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ab/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ab/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ab/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ab/$name.log"; exit $rc; fi
}
run tests 800 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run dbg 200 python scripts/heads_dbg.py
B="--skip-cpu --skip-kernel"
run h2_a 300 python bench.py $B
AZ_W4_HEADS_BOARDS=4 run h4_a 300 python bench.py $B
run h2_b 300 python bench.py $B
AZ_W4_HEADS_BOARDS=4 run h4_b 300 python bench.py $B
exit 0
