#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for w in c5 c4; do
  timeout -k 10 500 python -u bench.py --workload $w --skip-cpu > gpurun_out/heads_$w.json 2> gpurun_out/heads_$w.err || exit 1
  cut -c1-200 gpurun_out/heads_$w.json
done
