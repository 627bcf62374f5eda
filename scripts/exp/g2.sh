set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_nn_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/nn4.log 2>&1; rc=$?; tail -15 gpurun_out/nn4.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/conv_ab.py 1024 4096 > gpurun_out/conv_ab.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/conv_ab.log; exit $rc
