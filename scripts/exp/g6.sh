set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 2000 > gpurun_out/bench_c3.log 2>&1; rc=$?; tail -1 gpurun_out/bench_c3.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
exit 0
