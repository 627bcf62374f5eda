#!/bin/bash
# round 3, call 30: two-rank rehearsal of the distributed bench on one GPU (gloo stats,
# both ranks on cuda:0) with the final library; the engine's terminal-descent cap per step
# (AZ_MAX_DESCENTS 2 / 4 (product) / 8) on configs[2], alternating
set -u
mkdir -p gpurun_out/r03ad
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/r03ad/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ad/$name.json" 2> "gpurun_out/r03ad/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/r03ad/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/r03ad/$name.err"; exit $rc; fi
}
run rehearse 600 env AZ_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 400 --warmup 200 --skip-cpu --skip-kernel
B="--skip-cpu --skip-kernel"
run md4a 300 python bench.py $B
AZ_MAX_DESCENTS=2 run md2a 300 python bench.py $B
AZ_MAX_DESCENTS=8 run md8a 300 python bench.py $B
run md4b 300 python bench.py $B
AZ_MAX_DESCENTS=2 run md2b 300 python bench.py $B
AZ_MAX_DESCENTS=8 run md8b 300 python bench.py $B
exit 0
