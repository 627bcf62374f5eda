#!/bin/bash
# round 4: chunked persistent trunk for batches above the resident capacity (configs[3] 4,096
# slots, the arena's 2,048-row evaluations): suite + smoke, A/B bench lines; an eager
# steady-state kernel trace of configs[2]
set -u
export OUT=gpurun_out/r04l TMPDIR=/tmp
mkdir -p $OUT
STEPS=pytest,smoke PYTEST_TIMEOUT=900 bash scripts/gpu_check.sh || exit $?
grep -q " failed" $OUT/pytest_gpu.log && { echo "suite failed"; exit 1; }
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" >> "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -1 "$OUT/$name.log" | cut -c1-220
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
}
for r in 1 2; do
  run c4 500 python bench.py --workload c4 --skip-cpu --skip-kernel
  AZ_TRUNK4_CHUNKS=0 run c4_nochunk 500 python bench.py --workload c4 --skip-cpu --skip-kernel
done
run arena 600 python bench.py --workload arena --matches 1024
AZ_TRUNK4_CHUNKS=0 run arena_nochunk 600 python bench.py --workload arena --matches 1024
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_eager -o run -- python3 bench.py --skip-cpu --skip-kernel --no-graph --steps 2000 > $OUT/trace_eager.log 2>&1
echo "eager trace rc=$?"; tail -1 $OUT/trace_eager.log | cut -c1-200
exit 0
