#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel-trace summary.
# Stops at the first step that faults, aborts or times out (exit codes >= 124 or signals).
set -u
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping after $name (rc=$rc)"; exit $rc
  fi
  return 0
}
STEPS=${STEPS:-all}
[[ $STEPS == *pytest* || $STEPS == all ]] && run pytest_gpu ${PYTEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_TARGET:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* || $STEPS == all ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* || $STEPS == all ]] && run bench 900 python bench.py ${BENCH_ARGS:-}
[[ $STEPS == *prof* || $STEPS == all ]] && run rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --skip-cpu --steps-per-graph 1 --warmup-exact ${PROF_ARGS:---steps 400 --warmup 2000}
[[ $STEPS == *skb* ]] && run skb 120 python scripts/step_kernel_bench.py
[[ $STEPS == *nnmb* ]] && run nnmb 300 python scripts/nn_microbench.py 1024
[[ $STEPS == *convb* ]] && run convb 300 python scripts/conv_bench.py
[[ $STEPS == *variants* ]] && run variants 300 python scripts/exp/run_step_variants.py
[[ $STEPS == *breakdown* ]] && run breakdown 600 python scripts/step_breakdown.py ${BREAKDOWN_STEPS:-30000}
[[ $STEPS == *pmc* ]] && run pmc 900 bash scripts/pmc_step.sh
[[ $STEPS == *rehearse* ]] && run rehearse 600 env AZ_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 400 --warmup 200 --skip-cpu --skip-kernel
exit 0
