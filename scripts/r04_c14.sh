#!/bin/bash
# round 4: packed-f32 VALU beside the MFMAs in the trunk conv -- the tree's library against
# conv_wino4.hip built without the packed-fp32 feature (expbuild/nopk: scalar v_add/v_mul/
# v_fma_f32 in the transform and the fold, same IEEE operations): net evaluation time at
# B = 1,024 (sums must agree) and the configs[2] bench, alternating
set -u
export OUT=gpurun_out/r04n TMPDIR=/tmp
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 200 python scripts/net_time.py 1024 40 >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
  AZ_LIB_PATH=expbuild/nopk/libaz_othello.so timeout -k 10 200 python scripts/net_time.py 1024 40 >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
done
cat $OUT/net.jsonl
for r in 1 2; do
  timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_pk_$r.log 2>&1 || exit 1
  echo "pk   $(tail -1 $OUT/ab_pk_$r.log | cut -c1-110)"
  AZ_LIB_PATH=expbuild/nopk/libaz_othello.so timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_nopk_$r.log 2>&1 || exit 1
  echo "nopk $(tail -1 $OUT/ab_nopk_$r.log | cut -c1-110)"
done
exit 0
