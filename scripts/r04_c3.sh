#!/bin/bash
# round 4, call 3: bench-path goldens (K = 4 open batches), trunk / heads tests, then the
# full GPU suite; net-evaluation A/B (heads in the persistent trunk vs its own launch,
# two- vs four-board heads conv, co-resident workgroup stagger builds); default bench
set -u
export OUT=gpurun_out/r04c TMPDIR=/tmp
mkdir -p $OUT
STEPS=pytest PYTEST_TIMEOUT=900 PYTEST_TARGET="tests/test_bench_path_gpu.py tests/test_nn_gpu.py tests/test_vl_gpu.py" bash scripts/gpu_check.sh || exit $?
mv $OUT/pytest_gpu.log $OUT/pytest_first.log
grep -q " failed" $OUT/pytest_first.log && { echo "first tests failed"; exit 1; }
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" >> "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -2 "$OUT/$name.log"
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
AZ_TRUNK_HEADS=0 run bench_noth 400 python bench.py --skip-cpu --skip-kernel
STEPS=pytest,smoke bash scripts/gpu_check.sh
exit 0
