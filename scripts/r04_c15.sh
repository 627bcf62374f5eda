#!/bin/bash
# round 4: configs[2]'s 1,024 games as 1 / 2 / 4 independent pipelines on their own streams
# (scripts/split_pipeline.py): does a pipeline's select launch hide beside another's trunk?
set -u
export OUT=gpurun_out/r04o TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u scripts/split_pipeline.py 1 2 4 > $OUT/split.jsonl 2> $OUT/split.err
rc=$?; cat $OUT/split.jsonl; tail -3 $OUT/split.err; exit $rc
