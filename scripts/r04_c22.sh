#!/bin/bash
# round 4, final library (tail skip, fill skip, heads in the persistent trunk): full GPU suite,
# smoke, the default bench line, configs[3] / arena lines, eager kernel trace of configs[2]
set -u
export OUT=gpurun_out/r04v TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 500 python bench.py --workload c4 --skip-cpu > $OUT/bench_c4.log 2>&1 || exit 1
echo "c4 $(tail -1 $OUT/bench_c4.log | cut -c1-140)"
timeout -k 10 500 python bench.py --workload arena --matches 1024 > $OUT/bench_arena.log 2>&1 || exit 1
echo "arena $(tail -1 $OUT/bench_arena.log | cut -c1-140)"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_eager -o run -- python3 bench.py --skip-cpu --no-graph --steps 2000 > $OUT/trace_eager.log 2>&1
echo "eager trace rc=$?"
exit 0
