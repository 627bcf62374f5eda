#!/bin/bash
# round 3, call 10: the stem inside the select launch -- parity tests, bench A/B (configs[2]
# and [3]), steady-state profile
set -u
mkdir -p gpurun_out/r03j
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03j/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03j/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03j/steps.log
  tail -2 "gpurun_out/r03j/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run stem_tests 600 python -u -m pytest tests/test_engine_stem_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run bench_stem 400 python bench.py --skip-cpu --skip-kernel --steps 4000
run bench_nostem 400 python bench.py --skip-cpu --skip-kernel --steps 4000 --no-engine-stem
run bench_stem2 400 python bench.py --skip-cpu --skip-kernel --steps 4000
run bench_c4_stem 400 python bench.py --workload c4 --skip-cpu --skip-kernel --steps 4000
run bench_c4_nostem 400 python bench.py --workload c4 --skip-cpu --skip-kernel --steps 4000 --no-engine-stem
run prof_c3 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c3 -o run -- python3 bench.py --skip-cpu --skip-kernel --steps 2000 --warmup 24000
run tail_c3 120 python scripts/trace_tail.py /tmp/prof_c3/run_kernel_trace.csv 2000
cp /tmp/prof_c3/run_kernel_stats.csv gpurun_out/r03j/prof_c3_kernel_stats.csv
run gputests 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
exit 0
