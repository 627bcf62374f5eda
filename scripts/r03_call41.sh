#!/bin/bash
# round 3, call 41: the select launch's end-of-launch counter update without a reload
# (sims_done / sims_acc kept from the launch's first loads): GPU tests, smoke, default bench
set -u
mkdir -p gpurun_out/r03an
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03an/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03an/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03an/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03an/$name.log"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run smoke 200 python -c 'import __graft_entry__ as g; g.smoke()'
run bench 400 python bench.py
run bench_b 300 python bench.py --skip-cpu --skip-kernel
exit 0
