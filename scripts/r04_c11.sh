#!/bin/bash
# round 4: Params back by value (global_* codegen): engine + bench-path tests, smoke; bench A/B
# of the heads inside the (waterfall-free) trunk; the configs[2] window traced alone in graph
# mode (--selected-regions); arena bench + its kernel trace
set -u
export OUT=gpurun_out/r04k TMPDIR=/tmp
mkdir -p $OUT
STEPS=pytest,smoke PYTEST_TIMEOUT=900 bash scripts/gpu_check.sh || exit $?
grep -q " failed" $OUT/pytest_gpu.log && { echo "suite failed"; exit 1; }
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" >> "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -1 "$OUT/$name.log" | cut -c1-250
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
}
for r in 1 2; do
  run net 120 python scripts/net_time.py 1024 40
  AZ_TRUNK_HEADS=1 run net 120 python scripts/net_time.py 1024 40
done
run bench 400 python bench.py --skip-cpu
AZ_TRUNK_HEADS=1 run bench_th 400 python bench.py --skip-cpu --skip-kernel
run arena 600 python bench.py --workload arena --matches 1024
AZ_PROF_WINDOW=1 timeout -k 10 600 rocprofv3 --selected-regions --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --skip-cpu --skip-kernel --steps 2000 > $OUT/trace_bench.log 2>&1
echo "window trace rc=$?"; tail -1 $OUT/trace_bench.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_arena -o run -- python3 bench.py --workload arena --matches 256 > $OUT/trace_arena.log 2>&1
echo "arena trace rc=$?"; tail -1 $OUT/trace_arena.log | cut -c1-200
exit 0
