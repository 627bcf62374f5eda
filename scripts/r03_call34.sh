#!/bin/bash
# round 3, call 34: persistent-trunk stress (bit-identity over many evaluations), then the
# round-end validation on this library: GPU tests, smoke, the default bench line
set -u
mkdir -p gpurun_out/r03ah
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ah/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ah/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ah/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ah/$name.log"; exit $rc; fi
}
run stress 300 python -u scripts/trunk4_stress.py
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run smoke 200 python -c 'import __graft_entry__ as g; g.smoke()'
run bench 400 python bench.py
exit 0
