#!/bin/bash
# round 3, call 11: where the select launch's time goes with the engine stem (steady-state
# kernel profiles of configs[2]: stem on / off / compiled out / without its stores)
set -u
mkdir -p gpurun_out/r03k
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03k/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03k/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03k/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03k/$name.log"; exit $rc; fi
}
prof() {
  local name=$1; shift
  run prof_$name 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$name -o run -- python3 bench.py --skip-cpu --skip-kernel --steps 2000 --warmup 24000 "$@"
  run tail_$name 120 python scripts/trace_tail.py /tmp/p_$name/run_kernel_trace.csv 2000
  rm -rf /tmp/p_$name
}
prof stem
prof nostem --no-engine-stem
AZ_LIB_PATH=expbuild/stem_nocode/libaz_othello.so prof nocode --no-engine-stem
AZ_LIB_PATH=expbuild/stem_nostore/libaz_othello.so prof nostore
exit 0
