#!/bin/bash
# round 4, call 2: bench-path goldens, heads two-board form, arena graphs; full GPU suite;
# smoke; a graph-mode rocprofv3 kernel trace of configs[2] (Params by pointer); leaf-row
# occupancy; arena bench line
set -u
export OUT=gpurun_out/r04b TMPDIR=/tmp
mkdir -p $OUT
STEPS=pytest PYTEST_TIMEOUT=900 PYTEST_TARGET="tests/test_bench_path_gpu.py tests/test_arena_gpu.py tests/test_nn_gpu.py" bash scripts/gpu_check.sh || exit $?
mv $OUT/pytest_gpu.log $OUT/pytest_first.log
STEPS=pytest,smoke bash scripts/gpu_check.sh || exit $?
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
}
run rocprof_graph 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --skip-cpu --steps 400 --warmup 2000 --warmup-exact
run occupancy 300 python scripts/row_occupancy.py 2000
run arena 600 python bench.py --workload arena --matches 1024
exit 0
