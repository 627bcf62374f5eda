#!/bin/bash
# split-K conv: numerics tests, per-batch sweep, then drop-in A/B over the split count
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_nn_gpu.py > gpurun_out/splitk_nn.log 2>&1 || { tail -30 gpurun_out/splitk_nn.log; exit 1; }
tail -3 gpurun_out/splitk_nn.log
timeout -k 10 200 python -u scripts/splitk_sweep.py > gpurun_out/splitk_sweep.jsonl 2> gpurun_out/splitk_sweep.err && cat gpurun_out/splitk_sweep.jsonl && \
AZ_SPLITK=16 timeout -k 10 200 python -u scripts/dropin_bench.py > gpurun_out/splitk_ab16.json 2> gpurun_out/splitk_ab16.err && cat gpurun_out/splitk_ab16.json && \
AZ_SPLITK=32 timeout -k 10 200 python -u scripts/dropin_bench.py > gpurun_out/splitk_ab32.json 2> gpurun_out/splitk_ab32.err && cat gpurun_out/splitk_ab32.json
