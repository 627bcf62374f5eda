#!/bin/bash
# gpurun with retries ONLY when no box was obtained (exit 3: nothing ran, nothing charged)
out=$1; shift; t=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $t -- "$@" > $out 2>&1
  rc=$?
  echo "EXIT $rc (attempt $i)" >> $out
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
