#!/bin/bash
# round 4: where the merged select launch's time goes now (AZ_ENG_STAMP build); configs[1] /
# configs[4] workload lines; the default bench line with the CPU baseline
set -u
export OUT=gpurun_out/r04m TMPDIR=/tmp
mkdir -p $OUT
AZ_LIB_PATH=expbuild/estamp/libaz_othello.so timeout -k 10 400 python scripts/eng_stamps.py 26000 > $OUT/eng_stamps.json 2> $OUT/eng_stamps.err
echo "stamps rc=$?"
for w in c2 c5; do
  timeout -k 10 500 python bench.py --workload $w --skip-cpu > $OUT/bench_$w.log 2>&1
  echo "$w rc=$?"; tail -1 $OUT/bench_$w.log | cut -c1-200
done
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
echo "bench rc=$?"; tail -1 $OUT/bench.log | cut -c1-200
exit 0
