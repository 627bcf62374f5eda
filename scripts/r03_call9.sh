#!/bin/bash
# round 3, call 9: deferred moves inside the select launch -- parity tests, the GPU suite,
# bench A/B (configs[2] and [3]), steady-state profile
set -u
mkdir -p gpurun_out/r03i
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03i/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03i/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03i/steps.log
  tail -2 "gpurun_out/r03i/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run defer_tests 600 python -u -m pytest tests/test_defer_gpu.py tests/test_c5_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run gputests 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
run bench_defer 400 python bench.py --skip-cpu --skip-kernel --steps 4000
run bench_nodefer 400 python bench.py --skip-cpu --skip-kernel --steps 4000 --no-defer
run bench_defer2 400 python bench.py --skip-cpu --skip-kernel --steps 4000
run bench_c4_defer 400 python bench.py --workload c4 --skip-cpu --skip-kernel --steps 4000
run bench_c4_nodefer 400 python bench.py --workload c4 --skip-cpu --skip-kernel --steps 4000 --no-defer
run prof_c3 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c3 -o run -- python3 bench.py --skip-cpu --skip-kernel --steps 2000 --warmup 24000
run tail_c3 120 python scripts/trace_tail.py /tmp/prof_c3/run_kernel_trace.csv 2000
cp /tmp/prof_c3/run_kernel_stats.csv gpurun_out/r03i/prof_c3_kernel_stats.csv
exit 0
