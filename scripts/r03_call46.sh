#!/bin/bash
# round 3, call 46: the engine stem's two channels per lane as one packed fp32 fma
# (AZ_STEM_PK): GPU tests (the engine stem bit-identical to k_conv_stem), smoke, then configs[2]
# against the AZ_STEM_PK=0 build, three alternating rounds
set -u
mkdir -p gpurun_out/r03ar
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ar/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ar/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ar/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ar/$name.log"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run smoke 200 python -c 'import __graft_entry__ as g; g.smoke()'
B="--skip-cpu --skip-kernel"
for r in a b c; do
  run pk_$r 300 python bench.py $B
  AZ_LIB_PATH=expbuild/pk0/libaz_othello.so run pk0_$r 300 python bench.py $B
done
exit 0
