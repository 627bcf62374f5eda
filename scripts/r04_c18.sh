#!/bin/bash
# round 4: the persistent trunk's per-layer timeline (AZ_W4_TSTAMP build): prologue, K loop,
# epilogues, layer fence -- is the layer transition worth pipelining?
set -u
export OUT=gpurun_out/r04r TMPDIR=/tmp
mkdir -p $OUT
AZ_LIB_PATH=expbuild/tstamp/libaz_othello.so timeout -k 10 200 python scripts/trunk_stamps.py 1024 > $OUT/tstamps.json 2> $OUT/tstamps.err || { tail -5 $OUT/tstamps.err; exit 1; }
cat $OUT/tstamps.json
timeout -k 10 200 python scripts/net_time.py 1024 40 > $OUT/net.jsonl 2>> $OUT/net.err || exit 1
AZ_LIB_PATH=expbuild/tstamp/libaz_othello.so timeout -k 10 200 python scripts/net_time.py 1024 40 >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
cat $OUT/net.jsonl
exit 0
