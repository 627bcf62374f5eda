#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/splitk_sweep.py > gpurun_out/splitk_sweep.jsonl 2> gpurun_out/splitk_sweep.err && cat gpurun_out/splitk_sweep.jsonl && \
for k in 8 16 32 16 8; do
  AZ_SPLITK=$k timeout -k 10 200 python -u scripts/dropin_bench.py > gpurun_out/splitk_ab$k.json 2> gpurun_out/splitk_ab$k.err || exit 1
  echo "splits $k: $(python -c "import json;d=json.load(open('gpurun_out/splitk_ab$k.json'));print(d['num_threads_default_4']['self_play']['games_per_s'], d['num_threads_1']['self_play']['games_per_s'])")"
done
