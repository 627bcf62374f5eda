#!/bin/bash
# round 4: counters of the shipped trunk forms; steady-state kernel trace of the configs[2]
# step in graph mode; default bench line
set -u
export OUT=gpurun_out/r04i TMPDIR=/tmp
mkdir -p $OUT
OUT=$OUT bash scripts/pmc_trunk.sh 2>&1 | tee $OUT/pmc_steps.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --skip-cpu --skip-kernel --steps 2000 > $OUT/trace_bench.log 2>&1
echo "trace rc=$?"; tail -1 $OUT/trace_bench.log | cut -c1-200
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
echo "bench rc=$?"; tail -1 $OUT/bench.log | cut -c1-300
exit 0
