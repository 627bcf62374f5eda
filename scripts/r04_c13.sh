#!/bin/bash
# round 4: where the merged select launch's time goes now (AZ_ENG_STAMP builds: the move
# phase's subtree copy 4 / 8 nodes per thread per round trip); bench A/B of the copy batch;
# configs[1] / configs[4] workload lines; the default bench line with the CPU baseline
set -u
export OUT=gpurun_out/r04m TMPDIR=/tmp
mkdir -p $OUT
AZ_LIB_PATH=expbuild/estamp/libaz_othello.so timeout -k 10 400 python scripts/eng_stamps.py 26000 > $OUT/eng_stamps.json 2> $OUT/eng_stamps.err
echo "stamps rc=$?"
AZ_LIB_PATH=expbuild/estamp8/libaz_othello.so timeout -k 10 400 python scripts/eng_stamps.py 26000 > $OUT/eng_stamps8.json 2> $OUT/eng_stamps8.err
echo "stamps8 rc=$?"
for r in 1 2; do
  timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_kc4_$r.log 2>&1; echo "kc4 $(tail -1 $OUT/ab_kc4_$r.log | cut -c1-120)"
  AZ_LIB_PATH=expbuild/kc8/libaz_othello.so timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_kc8_$r.log 2>&1; echo "kc8 $(tail -1 $OUT/ab_kc8_$r.log | cut -c1-120)"
done
for w in c2 c5; do
  timeout -k 10 500 python bench.py --workload $w --skip-cpu > $OUT/bench_$w.log 2>&1
  echo "$w rc=$?"; tail -1 $OUT/bench_$w.log | cut -c1-200
done
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
echo "bench rc=$?"; tail -1 $OUT/bench.log | cut -c1-200
exit 0
