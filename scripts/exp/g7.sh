# conv kernel iteration: nn parity tests, the wino4 A/B at the bench batch, a c3 bench line
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/nn.log 2>&1; rc=$?; tail -3 gpurun_out/nn.log; [ $rc -ne 0 ] && exit $rc
CONV_AB_ONLY=wino4 timeout -k 10 300 python -u scripts/conv_ab.py 1024 > gpurun_out/ab.log 2>&1; rc=$?; cat gpurun_out/ab.log | grep '^{'; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --workload c3 --skip-cpu --steps 4000 > gpurun_out/bench_c3.log 2>&1; rc=$?; tail -1 gpurun_out/bench_c3.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
exit 0
