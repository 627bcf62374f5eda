#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 200 python -u scripts/dropin_bench.py > gpurun_out/dropin.json 2> gpurun_out/dropin.err && cat gpurun_out/dropin.json && \
timeout -k 10 240 python -u scripts/dropin_pool_bench.py 8 16 > gpurun_out/pool8.json 2> gpurun_out/pool8.err && cat gpurun_out/pool8.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/dprof && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof -o dp --output-format csv -- python3 scripts/dropin_bench.py > gpurun_out/dprof/out.json 2> gpurun_out/dprof/err.log; rc=$?
rm -f gpurun_out/dprof/*kernel_trace.csv gpurun_out/dprof/*agent_info.csv
exit $rc
