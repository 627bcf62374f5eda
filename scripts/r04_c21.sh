#!/bin/bash
# round 4: heads inside the persistent trunk as the last conv's epilogue body
# (AZ_W4_TRUNK_HEADS_EPI=1 build, AZ_TRUNK_HEADS=1) against the read-back form and the
# default (tower launch + heads-fused conv launch): bit-identity tests, evaluation time, bench
set -u -o pipefail
export OUT=gpurun_out/r04u TMPDIR=/tmp
mkdir -p $OUT
E=expbuild/thepi/libaz_othello.so
AZ_LIB_PATH=$E timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py -k "trunk or heads" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_epi.log 2>&1
rc=$?; tail -3 $OUT/pytest_epi.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python scripts/net_time.py 1024 40 | sed "s/^{/{\"form\": \"default\", /" >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
  AZ_TRUNK_HEADS=1 timeout -k 10 200 python scripts/net_time.py 1024 40 | sed 's/^{/{"form": "readback", /' >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
  AZ_TRUNK_HEADS=1 AZ_LIB_PATH=$E timeout -k 10 200 python scripts/net_time.py 1024 40 | sed 's/^{/{"form": "epi", /' >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
done
cat $OUT/net.jsonl
for r in 1 2; do
  timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_base_$r.log 2>&1 || exit 1
  echo "base $(tail -1 $OUT/ab_base_$r.log | cut -c1-110)"
  AZ_TRUNK_HEADS=1 AZ_LIB_PATH=$E timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_epi_$r.log 2>&1 || exit 1
  echo "epi  $(tail -1 $OUT/ab_epi_$r.log | cut -c1-110)"
done
exit 0
