#!/bin/bash
# gpurun with retries ONLY when no box was obtained (exit 3: nothing ran, nothing charged)
out=$1; shift; t=$1; shift
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout $t -- "$@" > $out 2>&1
  rc=$?
  echo "EXIT $rc (attempt $i)" >> $out
  [ $rc -ne 3 ] && exit $rc
  sleep 45
done
