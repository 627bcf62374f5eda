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



c2() {
  # bench.py's 20-step two-pipeline window with and without the kernel roofline part before
  # the warmup (alternating), and the probe's timeline with the kernel part
  export OUT=gpurun_out/r06b
  mkdir -p $OUT
  for i in 1 2 3; do
    run bench20_k_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu || exit $?
    run bench20_nok_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu --skip-kernel || exit $?
  done
  run probe_p2_kb 300 env PROBE_KB=1 python -u scripts/window_probe.py 2 20 20 20 20 20 || exit $?
  exit 0
}

c3() {
  # FastOthelloNet's 64-channel convs in FP16X2 on the direct kernel: accuracy / bit-identity
  # tests, the reference-net goldens, the drop-in batch order; configs[1] A/B against split3
  export OUT=gpurun_out/r06c
  mkdir -p $OUT
  pyt pytest_fp16x2 600 tests/test_nn_gpu.py -k "direct_fp16x2 or stem_fusion" || exit $?
  pyt pytest_fast 600 tests/test_net_golden_gpu.py tests/test_pipelined_gpu.py tests/test_engine_gpu.py \
    -k "fast or drop_in" || exit $?
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_split3 300 env AZ_CONV64_SPLIT3=1 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c2 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000
  rm -f $OUT/prof_c2/run_kernel_trace.csv
  exit 0
}

c4() {
  # configs[4]'s fp16 trunk and configs[2]'s fp16x2 trunk as four-board workgroups (exp6/tb4:
  # -DAZ_W4_TRUNK_BOARDS=4) against the two-board default; train.py's unchanged pool at the
  # reference's num_self_play = 300 over the job's CPUs
  export OUT=gpurun_out/r06d
  mkdir -p $OUT
  for i in 1 2; do
    run bench_c5 300 python bench.py --workload c5 --skip-cpu --skip-kernel || exit $?
    run bench_c5_tb4 300 env AZ_LIB_PATH=exp6/tb4/libaz_othello.so python bench.py --workload c5 --skip-cpu --skip-kernel || exit $?
  done
  run pool300 600 python scripts/dropin_pool_bench.py 15 300 400 || exit $?
  exit 0
}

c5() {
  # is a slow 20-step window the process or the first window after the warmup?  bench.py's
  # window followed by six more of the same length in the same process (AZ_BENCH_REPEAT)
  export OUT=gpurun_out/r06e
  mkdir -p $OUT
  for i in 1 2 3 4; do
    run bench20_rep_$i 300 env AZ_BENCH_REPEAT=6 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu --skip-kernel || exit $?
  done
  run bench20_rep_p1 300 env AZ_BENCH_REPEAT=6 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu --skip-kernel --pipelines 1 || exit $?
  exit 0
}

c6() {
  # FastOthelloNet's heads GEMM on az_heads_fast_gemm_gpu (fp16x2 MFMA) against torch.bmm;
  # the short window after sustained load with idle pauses (power management?)
  export OUT=gpurun_out/r06f
  mkdir -p $OUT
  pyt pytest_gemm 600 tests/test_nn_gpu.py tests/test_net_golden_gpu.py tests/test_pipelined_gpu.py \
    -k "heads_fast_gemm or fast" || exit $?
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_bmm 300 env AZ_FAST_GEMM=0 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  run power_p2 400 python -u scripts/window_power.py 2 || exit $?
  run power_p1 400 python -u scripts/window_power.py 1 || exit $?
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c2 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000
  rm -f $OUT/prof_c2/run_kernel_trace.csv
  exit 0
}

c7() {
  # bench.py with the settle windows (default 3) and the sustained block: two pipelines x3,
  # one pipeline x2, and the 8000-step window on the same box
  export OUT=gpurun_out/r06g
  mkdir -p $OUT
  for i in 1 2 3; do
    run bench20_p2_$i 300 env AZ_BENCH_REPEAT=3 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu --skip-kernel || exit $?
  done
  for i in 1 2; do
    run bench20_p1_$i 300 env AZ_BENCH_REPEAT=3 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu --skip-kernel --pipelines 1 || exit $?
  done
  run bench8000_p2 300 python bench.py --gpus 1 --steps 8000 --warmup 5 --skip-cpu --skip-kernel --settle 0 || exit $?
  run bench8000_p1 300 python bench.py --gpus 1 --steps 8000 --warmup 5 --skip-cpu --skip-kernel --settle 0 --pipelines 1 || exit $?
  exit 0
}

c8() {
  # conv16 stem weights hoisted (bit-identity and accuracy tests), two-board direct
  # workgroups (AZ_MX_CFG=0) against one for configs[1]; configs[4] with the four-board trunk
  # (exp6/tb4); train.py's unchanged pool at num_self_play = 300
  export OUT=gpurun_out/r06h
  mkdir -p $OUT
  pyt pytest_c16 600 tests/test_nn_gpu.py tests/test_net_golden_gpu.py \
    -k "stem_fusion or direct_fp16x2 or split3_is or fast" || exit $?
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_cfg0 300 env AZ_MX_CFG=0 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  for i in 1 2; do
    run bench_c5 300 python bench.py --workload c5 --skip-cpu --skip-kernel || exit $?
    run bench_c5_tb4 300 env AZ_LIB_PATH=exp6/tb4/libaz_othello.so python bench.py --workload c5 --skip-cpu --skip-kernel || exit $?
  done
  run pool300 600 python scripts/dropin_pool_bench.py 15 300 400 || exit $?
  exit 0
}

c9() {
  # heads GEMM staging by row lane groups (accuracy test, configs[1] bench), configs[1] as
  # four pipelines, and the default bench line (the driver's command)
  export OUT=gpurun_out/r06i
  mkdir -p $OUT
  pyt pytest_gemm 600 tests/test_nn_gpu.py tests/test_net_golden_gpu.py tests/test_pipelined_gpu.py \
    -k "heads_fast_gemm or fast" || exit $?
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_p4 300 python bench.py --workload c2 --skip-cpu --skip-kernel --pipelines 4 || exit $?
  done
  run bench_default 600 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
  exit 0
}

f1() {
  # the whole GPU suite and smoke() on the current tree
  export OUT=gpurun_out/r06j
  mkdir -p $OUT
  run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread || exit $?
  run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
  exit 0
}

f2() {
  # the trunk launch's HBM bytes for this build (profiles/trunk_traffic.json keyed on the build
  # id), then the default bench line (the driver's command) and its rocprofv3 kernel summary
  export OUT=gpurun_out/r06k
  mkdir -p $OUT
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    run hbm_$i 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/hbm_$i -o pmc -- \
      python3 scripts/trunk_heads_one.py 1024 20 || exit $?
  done
  python scripts/trunk_traffic.py $OUT/hbm_1 $OUT/hbm_2 "gpurun_out/r06k: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on scripts/trunk_heads_one.py 1024 20, dispatches 6-20 averaged" > profiles/trunk_traffic.json || exit $?
  cp profiles/trunk_traffic.json $OUT/trunk_traffic.json
  run bench_default 600 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu || exit $?
  rm -f $OUT/prof/run_kernel_trace.csv
  if [ -n "$FIN_C2_PROF" ]; then
    run rocprof_c2 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- \
      python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000 --sustained-steps 0 --settle 0 || exit $?
    rm -f $OUT/prof_c2/run_kernel_trace.csv
  fi
  exit 0
}

f3() {
  # the other workloads' lines on the current tree
  export OUT=gpurun_out/r06l
  mkdir -p $OUT
  run bench_c2 400 python bench.py --workload c2 --skip-cpu || exit $?
  run bench_c4 400 python bench.py --workload c4 --skip-cpu --skip-kernel || exit $?
  run bench_c5 400 python bench.py --workload c5 --skip-cpu --skip-kernel || exit $?
  run bench_arena 400 python bench.py --workload arena || exit $?
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c2 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000
  rm -f $OUT/prof_c2/run_kernel_trace.csv
  exit 0
}

c10() {
  # FastOthelloNet's trunk in one launch (az_fast_trunk_gpu): bit-identity with the three
  # launches, the reference-net goldens, configs[1] A/B and its kernel profile
  export OUT=gpurun_out/r06m
  mkdir -p $OUT
  pyt pytest_ft 600 tests/test_nn_gpu.py tests/test_net_golden_gpu.py tests/test_pipelined_gpu.py \
    -k "fast or stem_fusion" || exit $?
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_3l 300 env AZ_FAST_TRUNK=0 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c2 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000 --sustained-steps 0 --settle 0
  rm -f $OUT/prof_c2/run_kernel_trace.csv
  exit 0
}

c11() {
  # the fused FastOthelloNet trunk with conv2's residual recomputed (six workgroups per CU)
  # against the LDS-copy form (exp6/ftR: four per CU by LDS) and the three launches
  export OUT=gpurun_out/r06n
  mkdir -p $OUT
  pyt pytest_ft 600 tests/test_nn_gpu.py tests/test_net_golden_gpu.py -k "fast or stem_fusion" || exit $?
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_ldsR 300 env AZ_LIB_PATH=exp6/ftR/libaz_othello.so python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_3l 300 env AZ_FAST_TRUNK=0 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c2 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000 --sustained-steps 0 --settle 0
  rm -f $OUT/prof_c2/run_kernel_trace.csv
  exit 0
}

fin() {
  # the final tree: the whole GPU suite, smoke(), the driver's bench command and its kernel
  # summary, the other workloads' lines and configs[1]'s kernel summary
  export OUT=${FIN_OUT:-gpurun_out/r06o}
  mkdir -p $OUT
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread || exit $?
  run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
  run bench_default 600 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
  run bench_c2 400 python bench.py --workload c2 --skip-cpu || exit $?
  run bench_c4 400 python bench.py --workload c4 --skip-cpu --skip-kernel || exit $?
  run bench_c5 400 python bench.py --workload c5 --skip-cpu --skip-kernel || exit $?
  run bench_arena 400 python bench.py --workload arena || exit $?
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu || exit $?
  rm -f $OUT/prof/run_kernel_trace.csv
  if [ -n "$FIN_C2_PROF" ]; then
    run rocprof_c2 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- \
      python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000 --sustained-steps 0 --settle 0 || exit $?
    rm -f $OUT/prof_c2/run_kernel_trace.csv
  fi
  exit 0
}

c12() {
  # the trunk's MFMA shape alone: exp6/m16 (-DAZ_W4_EXP=1024, every 32x32x16 MFMA as two
  # 16x16x32, wrong results, same FLOP and cycles) against the product, alternating
  export OUT=gpurun_out/r06p
  mkdir -p $OUT
  for i in 1 2 3; do
    run net_prod 120 python scripts/net_time.py 1024 40 || exit $?
    run net_m16 120 env AZ_LIB_PATH=exp6/m16/libaz_othello.so python scripts/net_time.py 1024 40 || exit $?
  done
  exit 0
}

c13() {
  # configs[3] / configs[4] as four 1,024-game pipelines (one 1,024-board evaluation each)
  # against the two 2,048-game default
  export OUT=gpurun_out/r06q
  mkdir -p $OUT
  for i in 1 2; do
    run bench_c5 300 python bench.py --workload c5 --skip-cpu --skip-kernel || exit $?
    run bench_c5_p4 300 python bench.py --workload c5 --skip-cpu --skip-kernel --pipelines 4 || exit $?
    run bench_c4 300 python bench.py --workload c4 --skip-cpu --skip-kernel || exit $?
    run bench_c4_p4 300 python bench.py --workload c4 --skip-cpu --skip-kernel --pipelines 4 || exit $?
  done
  exit 0
}

c14() {
  # the driver's command three times on one more box (the window's spread)
  export OUT=gpurun_out/r06r
  mkdir -p $OUT
  for i in 1 2 3; do
    run bench_default_$i 600 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu || exit $?
  done
  run bench_8000 600 python bench.py --gpus 1 --steps 8000 --warmup 5 --skip-cpu --skip-kernel --settle 0 || exit $?
  exit 0
}
c15() {
  # graph length vs the driver's 20-step window: 8 (default, 8 + 8 + four single-step
  # replays per pipeline), 10 and 20 (divide the window), 4; four more windows per run
  export OUT=gpurun_out/r06s
  mkdir -p $OUT
  export AZ_BENCH_REPEAT=4
  for i in 1 2; do
    for k in 8 10 20 4; do
      run bench_spg${k}_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-cpu --skip-kernel --steps-per-graph $k || exit $?
    done
  done
  exit 0
}
c16() {
  # FastOthelloNet's heads: the finish kernel's part loads issued together (product) against
  # one part at a time (exp6/rolled), the GEMM's weight prefetch 6 steps ahead (exp6/pd6);
  # tests, configs[1] A/B, kernel profile
  export OUT=gpurun_out/r06t
  mkdir -p $OUT
  pyt pytest_heads 600 tests/test_nn_gpu.py tests/test_net_golden_gpu.py -k "fast or heads" || exit $?
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_rolled 300 env AZ_LIB_PATH=exp6/rolled/libaz_othello.so python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_pd6 300 env AZ_LIB_PATH=exp6/pd6/libaz_othello.so python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c2 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000 --sustained-steps 0 --settle 0
  rm -f $OUT/prof_c2/run_kernel_trace.csv
  exit 0
}
c17() {
  # c16 again on a consistent tree, plus the GEMM's board tile (AZ_FAST_GEMM_TILE 64 / 128: each
  # weight fragment feeds 2 / 4 row tiles) at 8 / 16 K slices
  export OUT=gpurun_out/r06u
  mkdir -p $OUT
  pyt pytest_heads 600 tests/test_nn_gpu.py tests/test_net_golden_gpu.py -k "fast or heads" || exit $?
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_rolled 300 env AZ_LIB_PATH=exp6/rolled/libaz_othello.so python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_pd6 300 env AZ_LIB_PATH=exp6/pd6/libaz_othello.so python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_t64s8 300 env AZ_FAST_GEMM_TILE=64 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_t64s16 300 env AZ_FAST_GEMM_TILE=64 AZ_FAST_GEMM_SPLITS=16 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_t128s16 300 env AZ_FAST_GEMM_TILE=128 AZ_FAST_GEMM_SPLITS=16 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  for v in t32s8:32:8 t64s16:64:16 t128s16:128:16; do
    IFS=: read n t sp <<< "$v"
    run rocprof_c2_$n 500 env AZ_FAST_GEMM_TILE=$t AZ_FAST_GEMM_SPLITS=$sp rocprofv3 --kernel-trace --stats \
      --output-format csv -d $OUT/prof_c2_$n -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000 --sustained-steps 0 --settle 0 || exit $?
    rm -f $OUT/prof_c2_$n/run_kernel_trace.csv
  done
  exit 0
}
c18() {
  # FastOthelloNet's one-launch trunk at four waves per SIMD (exp6/ft4: amdgpu_waves_per_eu(4),
  # 128 VGPRs, 8 workgroups per CU = one round of 2,048 boards) against three (6 per CU)
  export OUT=gpurun_out/r06v
  mkdir -p $OUT
  run pytest_ft4 300 env AZ_LIB_PATH=exp6/ft4/libaz_othello.so python -u -m pytest tests/test_nn_gpu.py tests/test_net_golden_gpu.py -k "fast" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
  for i in 1 2 3; do
    run net_prod 120 python scripts/net_time.py 2048 40 fast || exit $?
    run net_ft4 120 env AZ_LIB_PATH=exp6/ft4/libaz_othello.so python scripts/net_time.py 2048 40 fast || exit $?
  done
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_ft4 300 env AZ_LIB_PATH=exp6/ft4/libaz_othello.so python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  exit 0
}
c19() {
  # the arena's two engines on their own streams (AZ_ARENA_STREAMS, default on) against one
  # stream: parity tests, then eval.py's matches at configs[2]'s net and sims, alternating
  export OUT=gpurun_out/r06w
  mkdir -p $OUT
  pyt pytest_arena 600 tests/test_arena_gpu.py tests/test_callers_gpu.py || exit $?
  for i in 1 2; do
    run bench_arena 400 python bench.py --workload arena || exit $?
    run bench_arena_1s 400 env AZ_ARENA_STREAMS=0 python bench.py --workload arena || exit $?
  done
  exit 0
}
c20() {
  # unchanged train.py's pool at the reference's num_self_play = 300 over 15 workers: the
  # shared generation (one producer plays all 300 games) against per-worker batches
  # (AZ_DROPIN_SHARED=0), warm workers; then the whole Pool block cold (one generation as
  # train.py pays it, worker start and HIP context included)
  export OUT=gpurun_out/r06y
  mkdir -p $OUT
  run pool_shared 600 python scripts/dropin_pool_bench.py 15 300 400 || exit $?
  run pool_perworker 600 env AZ_DROPIN_SHARED=0 python scripts/dropin_pool_bench.py 15 300 400 || exit $?
  run pool_shared_cold 600 python scripts/dropin_pool_bench.py 15 300 400 cold || exit $?
  exit 0
}
c21() {
  # the shared generation's producer as one pipeline (default) or two (AZ_DROPIN_PIPELINES=2:
  # 2 x 150 slots, each evaluation 600 rows in one trunk launch instead of 1,024 + 176), cold
  export OUT=gpurun_out/r06z
  mkdir -p $OUT
  for i in 1 2; do
    run pool_cold_p1 600 python scripts/dropin_pool_bench.py 15 300 400 cold || exit $?
    run pool_cold_p2 600 env AZ_DROPIN_PIPELINES=2 python scripts/dropin_pool_bench.py 15 300 400 cold || exit $?
  done
  exit 0
}
fin2() {
  # the final tree once more: the GPU suite, smoke(), the driver's command
  export OUT=gpurun_out/r06zz
  mkdir -p $OUT
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread || exit $?
  run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
  run bench_default 600 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
  exit 0
}
c22() {
  # configs[1]'s evaluation by part, each alone (scripts/fast_parts_time.py)
  export OUT=gpurun_out/r06aa
  mkdir -p $OUT
  for i in 1 2; do
    run parts 120 python scripts/fast_parts_time.py 2048 30 || exit $?
  done
  exit 0
}
c23() {
  # bench.py's N > 1 path rehearsed on the one-GPU box with the final bench.py (the driver's
  # torchrun shape, world 2, every rank on cuda:0, gloo collectives; no --skip-cpu: rank 0
  # must leave cpu_baseline out at N > 1), then the driver's N = 1 command
  export OUT=gpurun_out/r06ab
  mkdir -p $OUT
  run rehearse_w2 400 env AZ_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 || exit $?
  run bench_default 600 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
  exit 0
}
c24() {
  # LLVM scheduling strategies for the trunk sources (conv_wino4.hip, conv16.hip): max-ilp,
  # max-memory-clause, iterative-ilp against the default, alternating: configs[2]'s evaluation
  # (net_time 1024) and configs[1]'s by part (fast_parts_time 2048)
  export OUT=gpurun_out/r06ac
  mkdir -p $OUT
  for i in 1 2; do
    for v in prod silp smem sitl; do
      if [ $v = prod ]; then L=""; else L="AZ_LIB_PATH=exp6/$v/libaz_othello.so"; fi
      run net_$v 120 env $L python scripts/net_time.py 1024 40 || exit $?
      run fast_$v 120 env $L python scripts/fast_parts_time.py 2048 30 || exit $?
    done
  done
  exit 0
}
c25() {
  # counters of FastOthelloNet's one-launch trunk (scripts/pmc_fast_trunk.sh)
  export OUT=gpurun_out/r06ad
  mkdir -p $OUT
  bash scripts/pmc_fast_trunk.sh || exit $?
  SQ_KERNEL=k_fast_trunk python scripts/sq_summary.py $OUT/sq_fast > $OUT/sq_fast_summary.txt || exit $?
  exit 0
}
c26() {
  # the fast trunk's epilogue image stores as channel pairs (exp6/pairw) against 16-bit stores:
  # bit-identity tests with the variant, evaluation parts and configs[1] A/B
  export OUT=gpurun_out/r06ae
  mkdir -p $OUT
  run pytest_pairw 300 env AZ_LIB_PATH=exp6/pairw/libaz_othello.so python -u -m pytest tests/test_nn_gpu.py tests/test_net_golden_gpu.py -k "fast" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
  for i in 1 2 3; do
    run fast_prod 120 python scripts/fast_parts_time.py 2048 30 || exit $?
    run fast_pairw 120 env AZ_LIB_PATH=exp6/pairw/libaz_othello.so python scripts/fast_parts_time.py 2048 30 || exit $?
  done
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_pairw 300 env AZ_LIB_PATH=exp6/pairw/libaz_othello.so python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  exit 0
}
c27() {
  # the heads GEMM at 4 K slices (256 workgroups, one per CU) against 8, by part and configs[1]
  export OUT=gpurun_out/r06af
  mkdir -p $OUT
  for i in 1 2 3; do
    run fast_s8 120 python scripts/fast_parts_time.py 2048 30 || exit $?
    run fast_s4 120 env AZ_FAST_GEMM_SPLITS=4 python scripts/fast_parts_time.py 2048 30 || exit $?
  done
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_s4 300 env AZ_FAST_GEMM_SPLITS=4 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  exit 0
}
c28() {
  # non-temporal hints in the resident persistent trunk (AZ_W4_NT: 1 = the residual's LDS-DMA
  # reads, 2 = the output stores, 3 = both) against none, configs[2]'s evaluation, alternating
  export OUT=gpurun_out/r06ag
  mkdir -p $OUT
  for i in 1 2 3; do
    for v in prod nt1 nt2 nt3; do
      if [ $v = prod ]; then L=""; else L="AZ_LIB_PATH=exp6/$v/libaz_othello.so"; fi
      run net_$v 120 env $L python scripts/net_time.py 1024 40 || exit $?
    done
  done
  exit 0
}
c29() {
  # configs[4]'s fp16 persistent trunk: weight prefetch distance (AZ_W4_PD16) 3 / 5 against 7
  export OUT=gpurun_out/r06ah
  mkdir -p $OUT
  for i in 1 2 3; do
    for v in prod pd16_3 pd16_5; do
      if [ $v = prod ]; then L=""; else L="AZ_LIB_PATH=exp6/$v/libaz_othello.so"; fi
      run net16_$v 120 env $L python scripts/net_time.py 1024 40 fp16 || exit $?
    done
  done
  exit 0
}
"$@"
