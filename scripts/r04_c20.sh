#!/bin/bash
# round 4, final library: full GPU suite, smoke, the default bench line (CPU baseline, step
# kernel roofline), configs[1] / configs[4] lines, and an eager kernel trace of configs[2]
# (its k_step2 average and the step's kernels)
set -u
export OUT=gpurun_out/r04t TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log | cut -c1-200
for w in c5 c2; do
  timeout -k 10 500 python bench.py --workload $w --skip-cpu > $OUT/bench_$w.log 2>&1 || exit 1
  echo "$w $(tail -1 $OUT/bench_$w.log | cut -c1-140)"
done
timeout -k 10 200 python scripts/net_time.py 1024 40 > $OUT/net.jsonl 2> $OUT/net.err || exit 1
cat $OUT/net.jsonl
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_eager -o run -- python3 bench.py --skip-cpu --no-graph --steps 2000 > $OUT/trace_eager.log 2>&1
echo "eager trace rc=$?"; tail -1 $OUT/trace_eager.log | cut -c1-200
exit 0
