set -u
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-33,28,19,20,33} GRIDS=${GRIDS:-2048,8192} timeout -k 10 300 python scripts/exp/run_step_variants.py > gpurun_out/variants2.log 2>&1 || exit $?
