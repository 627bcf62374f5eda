#!/bin/bash
# round 4: which change makes the two-board heads exact?  the heads stress tests on the tree
# library and on AZ_HEADS_FIX builds (1: FC weights waited for before use, 2: unpaired f32
# chains, 3: both), each twice
set -u
OUT=gpurun_out/r04g; mkdir -p $OUT; export TMPDIR=/tmp
K="two_board or trunk_heads or fused_heads_bit_identical_to_separate_heads"
for r in 1 2; do
for v in tree hfix1 hfix2 hfix3; do
  if [ $v = tree ]; then L=""; else L="expbuild/$v/libaz_othello.so"; fi
  AZ_LIB_PATH=$L timeout -k 10 200 python -u -m pytest tests/test_nn_gpu.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > $OUT/$v.$r.log 2>&1
  rc=$?; echo "$v run $r rc=$rc $(tail -1 $OUT/$v.$r.log)"
  [ $rc -ge 124 ] && exit $rc
done
done
exit 0
