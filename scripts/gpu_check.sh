#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel-trace summary.
# Stops at the first step that faults, aborts or times out (exit codes >= 124 or signals).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping after $name (rc=$rc)"; exit $rc
  fi
  return 0
}
STEPS=${STEPS:-all}
[[ $STEPS == *pytest* || $STEPS == all ]] && run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
[[ $STEPS == *smoke* || $STEPS == all ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* || $STEPS == all ]] && run bench 900 python bench.py ${BENCH_ARGS:-}
[[ $STEPS == *prof* || $STEPS == all ]] && run rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --skip-cpu ${PROF_ARGS:---steps 400 --warmup 200}
exit 0
