#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u scripts/dropin_bench.py > gpurun_out/dropin.json 2> gpurun_out/dropin.err && cat gpurun_out/dropin.json && \
timeout -k 10 240 python -u scripts/dropin_pool_bench.py 8 16 > gpurun_out/pool8.json 2> gpurun_out/pool8.err && cat gpurun_out/pool8.json
