#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nn_gpu.py > gpurun_out/heads_nn.log 2>&1 || { tail -30 gpurun_out/heads_nn.log; exit 1; }
tail -1 gpurun_out/heads_nn.log
AZ_LIB_PATH=$GRAFT_REPO_ROOT/scripts/exp/_ab/libaz_old.so timeout -k 10 120 python -u scripts/heads_time.py > gpurun_out/heads_time_old.json 2> gpurun_out/heads_time_old.err && cat gpurun_out/heads_time_old.json && \
timeout -k 10 120 python -u scripts/heads_time.py > gpurun_out/heads_time.json 2> gpurun_out/heads_time.err && cat gpurun_out/heads_time.json && \
timeout -k 10 200 python -u scripts/dropin_bench.py > gpurun_out/heads_dropin.json 2> gpurun_out/heads_dropin.err && cut -c1-200 gpurun_out/heads_dropin.json && \
timeout -k 10 500 python -u bench.py --skip-cpu > gpurun_out/heads_bench.json 2> gpurun_out/heads_bench.err && cut -c1-250 gpurun_out/heads_bench.json
