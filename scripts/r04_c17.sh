#!/bin/bash
# round 4: full GPU suite (with the pipelined tests), smoke, the configs[1]/[4] lines at their
# new 2-pipeline default, the default bench line with the CPU baseline
set -u
export OUT=gpurun_out/r04q TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
for w in c5 c2; do
  timeout -k 10 500 python bench.py --workload $w --skip-cpu > $OUT/bench_$w.log 2>&1 || exit 1
  echo "$w $(tail -1 $OUT/bench_$w.log | cut -c1-140)"
done
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log | cut -c1-200
exit 0
