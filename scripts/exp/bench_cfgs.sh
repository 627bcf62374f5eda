#!/bin/bash
# every bench workload on the current library (one box): configs[1]/[3]/[4] shapes and 256 x 4
set -o pipefail
mkdir -p gpurun_out
for w in c2 c4 c5; do
  timeout -k 10 500 python -u bench.py --workload $w --skip-cpu > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit 1
  cut -c1-200 gpurun_out/bench_$w.json
done
timeout -k 10 500 python -u bench.py --games 256 --leaves 4 --skip-cpu > gpurun_out/bench_256x4.json 2> gpurun_out/bench_256x4.err || exit 1
cut -c1-200 gpurun_out/bench_256x4.json
