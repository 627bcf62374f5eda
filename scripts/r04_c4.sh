#!/bin/bash
# round 4, call 4: which two-board heads form gives wrong values?  heads tests on the tree
# library, then on the AZ_HEADS_CHECK build (every differing word of the value path printed)
set -u
export OUT=${OUT:-gpurun_out/r04d} TMPDIR=/tmp
mkdir -p $OUT
K="persistent_trunk or trunk_heads or fused_heads or two_board"
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > $OUT/tree.log 2>&1
echo "tree rc=$?"; grep -E "PASSED|FAILED" $OUT/tree.log | sed 's/.*:://' | head -60
AZ_LIB_PATH=expbuild/hchk/libaz_othello.so timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > $OUT/hchk.log 2>&1
echo "hchk rc=$?"; grep -c HEADS_CHECK $OUT/hchk.log; grep HEADS_CHECK $OUT/hchk.log | head -40
exit 0
