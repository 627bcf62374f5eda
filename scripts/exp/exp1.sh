set -u
mkdir -p gpurun_out
timeout -k 10 120 python scripts/step_steady.py 3000 > gpurun_out/steady.log 2>&1 || exit $?
VARIANTS=33,35,33,35 GRIDS=2048,8192 timeout -k 10 200 python scripts/exp/run_step_variants.py > gpurun_out/variants.log 2>&1 || exit $?
