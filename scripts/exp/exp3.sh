set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_board_gpu.py tests/test_engine_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_board.log 2>&1 || exit $?
timeout -k 10 120 python scripts/step_steady.py 1500 > gpurun_out/steady.log 2>&1 || exit $?
VARIANTS=41,41 GRIDS=8192 timeout -k 10 200 python scripts/exp/run_step_variants.py > gpurun_out/variants2.log 2>&1 || exit $?
timeout -k 10 120 python scripts/step_steady.py 1500 > gpurun_out/steady2.log 2>&1 || exit $?
