set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload c2 > gpurun_out/bench_c2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload c5 > gpurun_out/bench_c5.log 2>&1 || exit $?
