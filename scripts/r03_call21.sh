#!/bin/bash
# round 3, call 21: two-board conv workgroups as the default (incl. the heads-fused conv):
# GPU tests, conv A/B against AZ_W4_BOARDS=4 (fp16x2 and fp16), configs[4] bench both ways
set -u
mkdir -p gpurun_out/r03u
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03u/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03u/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03u/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03u/$name.log"; exit $rc; fi
}
run pytest 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
export CONV_AB_ONLY=wino4
run ab_b2 300 python scripts/conv_ab.py 1024 4096
AZ_W4_BOARDS=4 run ab_b4 300 python scripts/conv_ab.py 1024 4096
B="--skip-cpu --skip-kernel --workload c5"
run c5_b2 300 python bench.py $B
AZ_W4_BOARDS=4 run c5_b4 300 python bench.py $B
run c5_b2b 300 python bench.py $B
exit 0
