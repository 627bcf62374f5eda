#!/bin/bash
# round 4: pipelined self-play (engine.PipelinedSelfPlay) -- parity tests, then the bench
# with 2 pipelines (the new configs[2] default) against 1, alternating, and the 4,096-slot
# workloads with 2 pipelines against 1
set -u
export OUT=gpurun_out/r04p TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_pipelined_gpu.py tests/test_bench_path_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/c3_p2_$r.log 2>&1 || exit 1
  echo "c3 p2 $(tail -1 $OUT/c3_p2_$r.log | cut -c1-120)"
  timeout -k 10 400 python bench.py --skip-cpu --skip-kernel --pipelines 1 > $OUT/c3_p1_$r.log 2>&1 || exit 1
  echo "c3 p1 $(tail -1 $OUT/c3_p1_$r.log | cut -c1-120)"
done
for w in c4 c5 c2; do
  for p in 2 1; do
    timeout -k 10 500 python bench.py --workload $w --skip-cpu --skip-kernel --pipelines $p > $OUT/${w}_p$p.log 2>&1 || exit 1
    echo "$w p$p $(tail -1 $OUT/${w}_p$p.log | cut -c1-120)"
  done
done
exit 0
