#!/bin/bash
# round 4: AZ_W4_TAIL (the layer's last two chunks skip the look-ahead past the end) -- the
# net and bench-path GPU tests on that build, evaluation time and sums against the tree's
# library, configs[2] bench alternating
set -u
export OUT=gpurun_out/r04s TMPDIR=/tmp
mkdir -p $OUT
T=expbuild/tail/libaz_othello.so
AZ_LIB_PATH=$T timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_bench_path_gpu.py tests/test_c5_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_tail.log 2>&1
rc=$?; tail -3 $OUT/pytest_tail.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python scripts/net_time.py 1024 40 >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
  AZ_LIB_PATH=$T timeout -k 10 200 python scripts/net_time.py 1024 40 >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
done
cat $OUT/net.jsonl
for r in 1 2; do
  timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_base_$r.log 2>&1 || exit 1
  echo "base $(tail -1 $OUT/ab_base_$r.log | cut -c1-110)"
  AZ_LIB_PATH=$T timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_tail_$r.log 2>&1 || exit 1
  echo "tail $(tail -1 $OUT/ab_tail_$r.log | cut -c1-110)"
done
exit 0
