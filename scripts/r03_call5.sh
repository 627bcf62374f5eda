#!/bin/bash
# round 3, call 5: heads fused into the last conv -- parity test, the GPU suite, bench A/B
# (fused vs separate heads), in-step kernel profile of configs[2]
set -u
mkdir -p gpurun_out/r03e
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03e/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03e/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03e/steps.log
  tail -2 "gpurun_out/r03e/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run heads_test 300 python -u -m pytest tests/test_nn_gpu.py -k "fused_heads or inference_copy" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run gputests 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
run bench_fused 400 python bench.py --skip-cpu --steps 4000
run bench_sep 400 env AZ_FUSE_HEADS=0 python bench.py --skip-cpu --skip-kernel --steps 4000
run bench_fused2 400 python bench.py --skip-cpu --skip-kernel --steps 4000
run prof_c3 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03e/prof_c3 -o run -- python3 bench.py --skip-cpu --skip-kernel --steps 2000 --warmup 24000
exit 0
