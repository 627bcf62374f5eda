#!/bin/bash
# round 3, call 36: heads fused into the (four-board) last conv against the whole tower in the
# persistent two-board trunk + the separate heads kernel (AZ_FUSE_HEADS=0), configs[2], alternating
set -u
mkdir -p gpurun_out/r03aj
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03aj/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03aj/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03aj/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03aj/$name.log"; exit $rc; fi
}
B="--skip-cpu --skip-kernel"
for r in a b c; do
  run fused_$r 300 python bench.py $B
  AZ_FUSE_HEADS=0 run sep_$r 300 python bench.py $B
done
exit 0
