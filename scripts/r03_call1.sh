#!/bin/bash
# round 3, first GPU call: new c5 / drop-in tests, the whole GPU suite, the conv A/B (diet vs
# round-2 loop), then the configs[4] workload under rocprofv3's kernel tracer (8-step graphs,
# then the 1-step form that crashed in round 2)
set -u
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03/steps.log
  tail -3 "gpurun_out/r03/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run newtests 600 python -u -m pytest tests/test_c5_gpu.py tests/test_callers_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run gputests 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
run convab_new 300 env CONV_AB_ONLY=wino4 python scripts/conv_ab.py 1024 4096
run convab_old 300 env CONV_AB_ONLY=wino4 AZ_LIB_PATH=expbuild/diet0/libaz_othello.so python scripts/conv_ab.py 1024 4096
run convab_new2 300 env CONV_AB_ONLY=wino4 python scripts/conv_ab.py 1024 4096
run bench_new 400 python bench.py --skip-cpu --steps 4000
run bench_old 400 env AZ_LIB_PATH=expbuild/diet0/libaz_othello.so python bench.py --skip-cpu --skip-kernel --steps 4000
run pc5_g8 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03/pc5_g8 -o run -- python3 bench.py --workload c5 --skip-cpu --skip-kernel --steps 2000 --warmup 6000 --warmup-exact
run pc5_g1 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03/pc5_g1 -o run -- python3 bench.py --workload c5 --skip-cpu --skip-kernel --steps 2000 --warmup 6000 --warmup-exact --steps-per-graph 1
exit 0
