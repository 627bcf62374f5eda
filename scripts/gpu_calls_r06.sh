#!/bin/bash
# Round 6's GPU calls (gpurun), one function per call, in the order they ran; each writes
# under gpurun_out/r06<letter>/ and the summaries that were kept are copied to profiles/.
#     /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_calls_r06.sh c1
set -u
export TMPDIR=/tmp

run() {  # run <name> <timeout> cmd...   (stops the call after a fault / abort / time limit)
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" >> "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
  return $rc
}

pyt() {  # pyt <name> <timeout> <targets...>
  local name=$1 t=$2; shift 2
  run "$name" "$t" python -u -m pytest "$@" -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread
}

c1() {
  # the driver's 20-step window beside long windows: where the short window loses time
  export OUT=gpurun_out/r06a
  mkdir -p $OUT
  run probe_p2 300 python -u scripts/window_probe.py 2 || exit $?
  run probe_p1 300 python -u scripts/window_probe.py 1 || exit $?
  run bench20 300 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu || exit $?
  run bench20_p1 300 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu --skip-kernel --pipelines 1 || exit $?
  run bench8000 300 python bench.py --gpus 1 --steps 8000 --warmup 5 --skip-cpu --skip-kernel || exit $?
  exit 0
}

"$@"
