#!/bin/bash
# round 3, call 12: the engine stem without per-tap branches -- parity, kernel profiles
set -u
mkdir -p gpurun_out/r03l
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03l/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03l/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03l/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03l/$name.log"; exit $rc; fi
}
prof() {
  local name=$1; shift
  run prof_$name 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$name -o run -- python3 bench.py --skip-cpu --skip-kernel --steps 2000 --warmup 24000 "$@"
  run tail_$name 120 python scripts/trace_tail.py /tmp/p_$name/run_kernel_trace.csv 2000
  rm -rf /tmp/p_$name
}
run stem_tests 600 python -u -m pytest tests/test_engine_stem_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
prof stem
prof nostem --no-engine-stem
AZ_LIB_PATH=expbuild/stem_nostore/libaz_othello.so prof nostore
exit 0
