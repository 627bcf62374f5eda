# round 2: caller-compat test, drop-in bench, rocprofv3 kernel trace on 8-step graphs
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_callers_gpu.py -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/callers.log 2>&1; rc=$?; tail -4 gpurun_out/callers.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/dropin_bench.py > gpurun_out/dropin.json 2> gpurun_out/dropin.err; rc=$?; cat gpurun_out/dropin.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/dropin.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof8 -o run -- python bench.py --skip-cpu --steps-per-graph 8 --warmup-exact --steps 400 --warmup 2000 > gpurun_out/prof8.log 2>&1; rc=$?; echo "prof8 rc=$rc"; tail -30 gpurun_out/prof8.log
exit $rc
