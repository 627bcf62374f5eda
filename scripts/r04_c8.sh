#!/bin/bash
# round 4: the full GPU suite with the unpaired heads chains, smoke; net-evaluation A/B (heads
# inside the persistent trunk / in the two-board last conv / four-board last conv; co-resident
# stagger builds); default bench
set -u
export OUT=gpurun_out/r04h TMPDIR=/tmp
mkdir -p $OUT
STEPS=pytest,smoke PYTEST_TIMEOUT=900 bash scripts/gpu_check.sh || exit $?
grep -q " failed" $OUT/pytest_gpu.log && { echo "suite failed"; exit 1; }
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" >> "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -1 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
}
for r in 1 2; do
  run net 120 python scripts/net_time.py 1024 40
  AZ_TRUNK_HEADS=0 run net 120 python scripts/net_time.py 1024 40
  AZ_TRUNK_HEADS=0 AZ_W4_HEADS_BOARDS=4 run net 120 python scripts/net_time.py 1024 40
  AZ_LIB_PATH=expbuild/stag1/libaz_othello.so run net 120 python scripts/net_time.py 1024 40
  AZ_LIB_PATH=expbuild/stag2/libaz_othello.so run net 120 python scripts/net_time.py 1024 40
  AZ_LIB_PATH=expbuild/stag4/libaz_othello.so run net 120 python scripts/net_time.py 1024 40
done
run bench 400 python bench.py --skip-cpu
AZ_TRUNK_HEADS=0 AZ_W4_HEADS_BOARDS=4 run bench_r3heads 400 python bench.py --skip-cpu --skip-kernel
run bench2 400 python bench.py --skip-cpu --skip-kernel
exit 0
