#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_vl_gpu.py tests/test_callers_gpu.py tests/test_arena_gpu.py > gpurun_out/kmax_tests.log 2>&1 || { tail -30 gpurun_out/kmax_tests.log; exit 1; }
tail -2 gpurun_out/kmax_tests.log
timeout -k 10 200 python -u scripts/dropin_bench.py > gpurun_out/kmax_dropin.json 2> gpurun_out/kmax_dropin.err && cat gpurun_out/kmax_dropin.json && \
timeout -k 10 400 python -u bench.py --games 256 --leaves 4 --steps 4000 --skip-cpu --skip-kernel > gpurun_out/kmax_256x4.json 2> gpurun_out/kmax_256x4.err && cut -c1-300 gpurun_out/kmax_256x4.json
