#!/bin/bash
# round 3, call 32: the drop-in search with fused select+expand iterations (az_select_expand):
# GPU tests, then the drop-in one_self_play / play_match rates with and without it
set -u
mkdir -p gpurun_out/r03af
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03af/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03af/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03af/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03af/$name.log"; exit $rc; fi
}
run tests 800 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run dropin_fused 300 python -u scripts/dropin_bench.py
AZ_FUSE_EXPAND=0 run dropin_plain 300 python -u scripts/dropin_bench.py
run dropin_fused2 300 python -u scripts/dropin_bench.py
exit 0
