#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/dprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof -o dp --output-format csv -- python3 scripts/dropin_bench.py > gpurun_out/dprof/out.json 2> gpurun_out/dprof/err.log
rc=$?
rm -f gpurun_out/dprof/*kernel_trace.csv gpurun_out/dprof/*agent_info.csv
find gpurun_out/dprof -name "*kernel_stats.csv" | head -3
exit $rc
