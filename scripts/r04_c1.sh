set -u
export OUT=gpurun_out/r04a
STEPS=pytest PYTEST_TARGET=tests/test_bench_path_gpu.py PYTEST_TIMEOUT=600 bash scripts/gpu_check.sh || exit $?
mv $OUT/pytest_gpu.log $OUT/pytest_benchpath.log
STEPS=pytest,smoke,bench bash scripts/gpu_check.sh
