#!/bin/bash
# Round 4's GPU calls (gpurun), one function per call, in the order they ran; each writes
# under gpurun_out/r04<letter>/ and the summaries that were kept are in profiles/ (DESIGN.md
# cites them).  Run one on the GPU box:
#     /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_calls_r04.sh c22
# Experiment libraries (expbuild/<name>/libaz_othello.so, AZ_LIB_PATH) are built beforehand
# with scripts/build_variants.py; each call names the one it loads.

c1() {
  set -u
  export OUT=gpurun_out/r04a
  STEPS=pytest PYTEST_TARGET=tests/test_bench_path_gpu.py PYTEST_TIMEOUT=600 bash scripts/gpu_check.sh || exit $?
  mv $OUT/pytest_gpu.log $OUT/pytest_benchpath.log
  STEPS=pytest,smoke,bench bash scripts/gpu_check.sh
}

c2() {
  # round 4, call 2: bench-path goldens, heads two-board form, arena graphs; full GPU suite;
  # smoke; a graph-mode rocprofv3 kernel trace of configs[2] (Params by pointer); leaf-row
  # occupancy; arena bench line
  set -u
  export OUT=gpurun_out/r04b TMPDIR=/tmp
  mkdir -p $OUT
  STEPS=pytest PYTEST_TIMEOUT=900 PYTEST_TARGET="tests/test_bench_path_gpu.py tests/test_arena_gpu.py tests/test_nn_gpu.py" bash scripts/gpu_check.sh || exit $?
  mv $OUT/pytest_gpu.log $OUT/pytest_first.log
  STEPS=pytest,smoke bash scripts/gpu_check.sh || exit $?
  run() {
    local name=$1 t=$2; shift 2
    echo "=== $name: $*" | tee -a $OUT/steps.log
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a $OUT/steps.log
    tail -3 "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
  }
  run rocprof_graph 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --skip-cpu --steps 400 --warmup 2000 --warmup-exact
  run occupancy 300 python scripts/row_occupancy.py 2000
  run arena 600 python bench.py --workload arena --matches 1024
  exit 0
}

c3() {
  # round 4, call 3: bench-path goldens (K = 4 open batches), trunk / heads tests, then the
  # full GPU suite; net-evaluation A/B (heads in the persistent trunk vs its own launch,
  # two- vs four-board heads conv, co-resident workgroup stagger builds); default bench
  set -u
  export OUT=gpurun_out/r04c TMPDIR=/tmp
  mkdir -p $OUT
  STEPS=pytest PYTEST_TIMEOUT=900 PYTEST_TARGET="tests/test_bench_path_gpu.py tests/test_nn_gpu.py tests/test_vl_gpu.py" bash scripts/gpu_check.sh || exit $?
  mv $OUT/pytest_gpu.log $OUT/pytest_first.log
  grep -q " failed" $OUT/pytest_first.log && { echo "first tests failed"; exit 1; }
  run() {
    local name=$1 t=$2; shift 2
    echo "=== $name: $*" | tee -a $OUT/steps.log
    timeout -k 10 "$t" "$@" >> "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a $OUT/steps.log
    tail -2 "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
  }
  for r in 1 2; do
    run net 120 python scripts/net_time.py 1024 40
    AZ_TRUNK_HEADS=0 run net 120 python scripts/net_time.py 1024 40
    AZ_TRUNK_HEADS=0 AZ_W4_HEADS_BOARDS=4 run net 120 python scripts/net_time.py 1024 40
    AZ_LIB_PATH=expbuild/stag1/libaz_othello.so run net 120 python scripts/net_time.py 1024 40
    AZ_LIB_PATH=expbuild/stag2/libaz_othello.so run net 120 python scripts/net_time.py 1024 40
    AZ_LIB_PATH=expbuild/stag4/libaz_othello.so run net 120 python scripts/net_time.py 1024 40
  done
  run bench 400 python bench.py --skip-cpu
  AZ_TRUNK_HEADS=0 run bench_noth 400 python bench.py --skip-cpu --skip-kernel
  STEPS=pytest,smoke bash scripts/gpu_check.sh
  exit 0
}

c4() {
  # round 4, call 4: which two-board heads form gives wrong values?  heads tests on the tree
  # library, then on the AZ_HEADS_CHECK build (every differing word of the value path printed)
  set -u
  export OUT=${OUT:-gpurun_out/r04d} TMPDIR=/tmp
  mkdir -p $OUT
  K="persistent_trunk or trunk_heads or fused_heads or two_board"
  timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > $OUT/tree.log 2>&1
  echo "tree rc=$?"; grep -E "PASSED|FAILED" $OUT/tree.log | sed 's/.*:://' | head -60
  AZ_LIB_PATH=expbuild/hchk/libaz_othello.so timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > $OUT/hchk.log 2>&1
  echo "hchk rc=$?"; grep -c HEADS_CHECK $OUT/hchk.log; grep HEADS_CHECK $OUT/hchk.log | head -40
  exit 0
}

c7() {
  # round 4: which change makes the two-board heads exact?  the heads stress tests on the tree
  # library and on AZ_HEADS_FIX builds (1: FC weights waited for before use, 2: unpaired f32
  # chains, 3: both), each twice
  set -u
  OUT=gpurun_out/r04g; mkdir -p $OUT; export TMPDIR=/tmp
  K="two_board or trunk_heads or fused_heads_bit_identical_to_separate_heads"
  for r in 1 2; do
  for v in tree hfix1 hfix2 hfix3; do
    if [ $v = tree ]; then L=""; else L="expbuild/$v/libaz_othello.so"; fi
    AZ_LIB_PATH=$L timeout -k 10 200 python -u -m pytest tests/test_nn_gpu.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > $OUT/$v.$r.log 2>&1
    rc=$?; echo "$v run $r rc=$rc $(tail -1 $OUT/$v.$r.log)"
    [ $rc -ge 124 ] && exit $rc
  done
  done
  exit 0
}

c8() {
  # round 4: the full GPU suite with the unpaired heads chains, smoke; net-evaluation A/B (heads
  # inside the persistent trunk / in the two-board last conv / four-board last conv; co-resident
  # stagger builds); default bench
  set -u
  export OUT=gpurun_out/r04h TMPDIR=/tmp
  mkdir -p $OUT
  STEPS=pytest,smoke PYTEST_TIMEOUT=900 bash scripts/gpu_check.sh || exit $?
  grep -q " failed" $OUT/pytest_gpu.log && { echo "suite failed"; exit 1; }
  run() {
    local name=$1 t=$2; shift 2
    echo "=== $name: $*" | tee -a $OUT/steps.log
    timeout -k 10 "$t" "$@" >> "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a $OUT/steps.log
    tail -1 "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
  }
  for r in 1 2; do
    run net 120 python scripts/net_time.py 1024 40
    AZ_TRUNK_HEADS=0 run net 120 python scripts/net_time.py 1024 40
    AZ_TRUNK_HEADS=0 AZ_W4_HEADS_BOARDS=4 run net 120 python scripts/net_time.py 1024 40
    AZ_LIB_PATH=expbuild/stag1/libaz_othello.so run net 120 python scripts/net_time.py 1024 40
    AZ_LIB_PATH=expbuild/stag2/libaz_othello.so run net 120 python scripts/net_time.py 1024 40
    AZ_LIB_PATH=expbuild/stag4/libaz_othello.so run net 120 python scripts/net_time.py 1024 40
  done
  run bench 400 python bench.py --skip-cpu
  AZ_TRUNK_HEADS=0 AZ_W4_HEADS_BOARDS=4 run bench_r3heads 400 python bench.py --skip-cpu --skip-kernel
  run bench2 400 python bench.py --skip-cpu --skip-kernel
  exit 0
}

c9() {
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
}

c10() {
  # round 4: the persistent trunk without waterfall loops (uniform per-layer pointers): full GPU
  # suite, smoke, net timing, bench; trunk counters; a graph-mode trace with the process map
  # and every thread's stack on a fault
  set -u
  export OUT=gpurun_out/r04j TMPDIR=/tmp
  mkdir -p $OUT
  STEPS=pytest,smoke PYTEST_TIMEOUT=900 bash scripts/gpu_check.sh || exit $?
  grep -q " failed" $OUT/pytest_gpu.log && { echo "suite failed"; exit 1; }
  for r in 1 2; do timeout -k 10 120 python scripts/net_time.py 1024 40 >> $OUT/net.log 2>&1; tail -1 $OUT/net.log; done
  timeout -k 10 600 python bench.py --skip-cpu > $OUT/bench.log 2>&1; echo "bench rc=$?"; tail -1 $OUT/bench.log | cut -c1-200
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
             "GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_TA_BUSY_sum" \
             "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES"; do
    i=$((${i:-0}+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/sq_trunk_$i -o pmc -- python3 scripts/trunk_one.py 1024 20 > $OUT/sq_trunk_$i.log 2>&1
    echo "trunk pass $i rc=$?"
  done
  AZ_DUMP_MAPS=$OUT/maps.txt AZ_FAULTHANDLER=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --skip-cpu --skip-kernel --steps 2000 > $OUT/trace_bench.log 2>&1
  echo "trace rc=$?"; tail -2 $OUT/trace_bench.log | cut -c1-200
  exit 0
}

c11() {
  # round 4: Params back by value (global_* codegen): engine + bench-path tests, smoke; bench A/B
  # of the heads inside the (waterfall-free) trunk; the configs[2] window traced alone in graph
  # mode (--selected-regions); arena bench + its kernel trace
  set -u
  export OUT=gpurun_out/r04k TMPDIR=/tmp
  mkdir -p $OUT
  STEPS=pytest,smoke PYTEST_TIMEOUT=900 bash scripts/gpu_check.sh || exit $?
  grep -q " failed" $OUT/pytest_gpu.log && { echo "suite failed"; exit 1; }
  run() {
    local name=$1 t=$2; shift 2
    echo "=== $name: $*" | tee -a $OUT/steps.log
    timeout -k 10 "$t" "$@" >> "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a $OUT/steps.log
    tail -1 "$OUT/$name.log" | cut -c1-250
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
  }
  for r in 1 2; do
    run net 120 python scripts/net_time.py 1024 40
    AZ_TRUNK_HEADS=1 run net 120 python scripts/net_time.py 1024 40
  done
  run bench 400 python bench.py --skip-cpu
  AZ_TRUNK_HEADS=1 run bench_th 400 python bench.py --skip-cpu --skip-kernel
  run arena 600 python bench.py --workload arena --matches 1024
  AZ_PROF_WINDOW=1 timeout -k 10 600 rocprofv3 --selected-regions --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --skip-cpu --skip-kernel --steps 2000 > $OUT/trace_bench.log 2>&1
  echo "window trace rc=$?"; tail -1 $OUT/trace_bench.log | cut -c1-200
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_arena -o run -- python3 bench.py --workload arena --matches 256 > $OUT/trace_arena.log 2>&1
  echo "arena trace rc=$?"; tail -1 $OUT/trace_arena.log | cut -c1-200
  exit 0
}

c12() {
  # round 4: chunked persistent trunk for batches above the resident capacity (configs[3] 4,096
  # slots, the arena's 2,048-row evaluations): suite + smoke, A/B bench lines; an eager
  # steady-state kernel trace of configs[2]
  set -u
  export OUT=gpurun_out/r04l TMPDIR=/tmp
  mkdir -p $OUT
  STEPS=pytest,smoke PYTEST_TIMEOUT=900 bash scripts/gpu_check.sh || exit $?
  grep -q " failed" $OUT/pytest_gpu.log && { echo "suite failed"; exit 1; }
  run() {
    local name=$1 t=$2; shift 2
    echo "=== $name: $*" | tee -a $OUT/steps.log
    timeout -k 10 "$t" "$@" >> "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a $OUT/steps.log
    tail -1 "$OUT/$name.log" | cut -c1-220
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
  }
  for r in 1 2; do
    run c4 500 python bench.py --workload c4 --skip-cpu --skip-kernel
    AZ_TRUNK4_CHUNKS=0 run c4_nochunk 500 python bench.py --workload c4 --skip-cpu --skip-kernel
  done
  run arena 600 python bench.py --workload arena --matches 1024
  AZ_TRUNK4_CHUNKS=0 run arena_nochunk 600 python bench.py --workload arena --matches 1024
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_eager -o run -- python3 bench.py --skip-cpu --skip-kernel --no-graph --steps 2000 > $OUT/trace_eager.log 2>&1
  echo "eager trace rc=$?"; tail -1 $OUT/trace_eager.log | cut -c1-200
  exit 0
}

c13() {
  # round 4: where the merged select launch's time goes now (AZ_ENG_STAMP builds: the move
  # phase's subtree copy 4 / 8 nodes per thread per round trip); bench A/B of the copy batch;
  # configs[1] / configs[4] workload lines; the default bench line with the CPU baseline
  set -u
  export OUT=gpurun_out/r04m TMPDIR=/tmp
  mkdir -p $OUT
  AZ_LIB_PATH=expbuild/estamp/libaz_othello.so timeout -k 10 400 python scripts/eng_stamps.py 26000 > $OUT/eng_stamps.json 2> $OUT/eng_stamps.err
  echo "stamps rc=$?"
  AZ_LIB_PATH=expbuild/estamp8/libaz_othello.so timeout -k 10 400 python scripts/eng_stamps.py 26000 > $OUT/eng_stamps8.json 2> $OUT/eng_stamps8.err
  echo "stamps8 rc=$?"
  for r in 1 2; do
    timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_kc4_$r.log 2>&1; echo "kc4 $(tail -1 $OUT/ab_kc4_$r.log | cut -c1-120)"
    AZ_LIB_PATH=expbuild/kc8/libaz_othello.so timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_kc8_$r.log 2>&1; echo "kc8 $(tail -1 $OUT/ab_kc8_$r.log | cut -c1-120)"
  done
  for w in c2 c5; do
    timeout -k 10 500 python bench.py --workload $w --skip-cpu > $OUT/bench_$w.log 2>&1
    echo "$w rc=$?"; tail -1 $OUT/bench_$w.log | cut -c1-200
  done
  timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
  echo "bench rc=$?"; tail -1 $OUT/bench.log | cut -c1-200
  exit 0
}

c14() {
  # round 4: packed-f32 VALU beside the MFMAs in the trunk conv -- the tree's library against
  # conv_wino4.hip built without the packed-fp32 feature (expbuild/nopk: scalar v_add/v_mul/
  # v_fma_f32 in the transform and the fold, same IEEE operations): net evaluation time at
  # B = 1,024 (sums must agree) and the configs[2] bench, alternating
  set -u
  export OUT=gpurun_out/r04n TMPDIR=/tmp
  mkdir -p $OUT
  for r in 1 2; do
    timeout -k 10 200 python scripts/net_time.py 1024 40 >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
    AZ_LIB_PATH=expbuild/nopk/libaz_othello.so timeout -k 10 200 python scripts/net_time.py 1024 40 >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
  done
  cat $OUT/net.jsonl
  for r in 1 2; do
    timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_pk_$r.log 2>&1 || exit 1
    echo "pk   $(tail -1 $OUT/ab_pk_$r.log | cut -c1-110)"
    AZ_LIB_PATH=expbuild/nopk/libaz_othello.so timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_nopk_$r.log 2>&1 || exit 1
    echo "nopk $(tail -1 $OUT/ab_nopk_$r.log | cut -c1-110)"
  done
  exit 0
}

c15() {
  # round 4: configs[2]'s 1,024 games as 1 / 2 / 4 independent pipelines on their own streams
  # (scripts/split_pipeline.py): does a pipeline's select launch hide beside another's trunk?
  set -u
  export OUT=gpurun_out/r04o TMPDIR=/tmp
  mkdir -p $OUT
  timeout -k 10 600 python -u scripts/split_pipeline.py 1 2 4 > $OUT/split.jsonl 2> $OUT/split.err
  rc=$?; cat $OUT/split.jsonl; tail -3 $OUT/split.err; exit $rc
}

c16() {
  # round 4: pipelined self-play (engine.PipelinedSelfPlay) -- parity tests, then the bench
  # with 2 pipelines (the new configs[2] default) against 1, alternating, and the 4,096-slot
  # workloads with 2 pipelines against 1
  set -u
  export OUT=gpurun_out/r04p TMPDIR=/tmp
  mkdir -p $OUT
  timeout -k 10 400 python -u -m pytest tests/test_pipelined_gpu.py tests/test_bench_path_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2; do
    timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/c3_p2_$r.log 2>&1 || exit 1
    echo "c3 p2 $(tail -1 $OUT/c3_p2_$r.log | cut -c1-120)"
    timeout -k 10 400 python bench.py --skip-cpu --skip-kernel --pipelines 1 > $OUT/c3_p1_$r.log 2>&1 || exit 1
    echo "c3 p1 $(tail -1 $OUT/c3_p1_$r.log | cut -c1-120)"
  done
  for w in c4 c5 c2; do
    for p in 2 1; do
      timeout -k 10 500 python bench.py --workload $w --skip-cpu --skip-kernel --pipelines $p > $OUT/${w}_p$p.log 2>&1 || exit 1
      echo "$w p$p $(tail -1 $OUT/${w}_p$p.log | cut -c1-120)"
    done
  done
  exit 0
}

c17() {
  # round 4: full GPU suite (with the pipelined tests), smoke, the configs[1]/[4] lines at their
  # new 2-pipeline default, the default bench line with the CPU baseline
  set -u
  export OUT=gpurun_out/r04q TMPDIR=/tmp
  mkdir -p $OUT
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
  tail -1 $OUT/smoke.log
  for w in c5 c2; do
    timeout -k 10 500 python bench.py --workload $w --skip-cpu > $OUT/bench_$w.log 2>&1 || exit 1
    echo "$w $(tail -1 $OUT/bench_$w.log | cut -c1-140)"
  done
  timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit 1
  tail -1 $OUT/bench.log | cut -c1-200
  exit 0
}

c18() {
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
}

c19() {
  # round 4: AZ_W4_TAIL (the layer's last two chunks skip the look-ahead past the end) -- the
  # net and bench-path GPU tests on that build, evaluation time and sums against the tree's
  # library, configs[2] bench alternating
  set -u
  export OUT=gpurun_out/r04s TMPDIR=/tmp
  mkdir -p $OUT
  T=expbuild/tail/libaz_othello.so
  AZ_LIB_PATH=$T timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_bench_path_gpu.py tests/test_c5_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_tail.log 2>&1
  rc=$?; tail -3 $OUT/pytest_tail.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2; do
    timeout -k 10 200 python scripts/net_time.py 1024 40 >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
    AZ_LIB_PATH=$T timeout -k 10 200 python scripts/net_time.py 1024 40 >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
  done
  cat $OUT/net.jsonl
  for r in 1 2; do
    timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_base_$r.log 2>&1 || exit 1
    echo "base $(tail -1 $OUT/ab_base_$r.log | cut -c1-110)"
    AZ_LIB_PATH=$T timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_tail_$r.log 2>&1 || exit 1
    echo "tail $(tail -1 $OUT/ab_tail_$r.log | cut -c1-110)"
  done
  exit 0
}

c20() {
  # round 4, final library: full GPU suite, smoke, the default bench line (CPU baseline, step
  # kernel roofline), configs[1] / configs[4] lines, and an eager kernel trace of configs[2]
  # (its k_step2 average and the step's kernels)
  set -u
  export OUT=gpurun_out/r04t TMPDIR=/tmp
  mkdir -p $OUT
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
  tail -1 $OUT/smoke.log
  timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit 1
  tail -1 $OUT/bench.log | cut -c1-200
  for w in c5 c2; do
    timeout -k 10 500 python bench.py --workload $w --skip-cpu > $OUT/bench_$w.log 2>&1 || exit 1
    echo "$w $(tail -1 $OUT/bench_$w.log | cut -c1-140)"
  done
  timeout -k 10 200 python scripts/net_time.py 1024 40 > $OUT/net.jsonl 2> $OUT/net.err || exit 1
  cat $OUT/net.jsonl
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_eager -o run -- python3 bench.py --skip-cpu --no-graph --steps 2000 > $OUT/trace_eager.log 2>&1
  echo "eager trace rc=$?"; tail -1 $OUT/trace_eager.log | cut -c1-200
  exit 0
}

c21() {
  # round 4: heads inside the persistent trunk as the last conv's epilogue body
  # (AZ_W4_TRUNK_HEADS_EPI=1 build, AZ_TRUNK_HEADS=1) against the read-back form and the
  # default (tower launch + heads-fused conv launch): bit-identity tests, evaluation time, bench
  set -u -o pipefail
  export OUT=gpurun_out/r04u TMPDIR=/tmp
  mkdir -p $OUT
  E=expbuild/thepi/libaz_othello.so
  AZ_LIB_PATH=$E timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py -k "trunk or heads" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_epi.log 2>&1
  rc=$?; tail -3 $OUT/pytest_epi.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2; do
    timeout -k 10 200 python scripts/net_time.py 1024 40 | sed "s/^{/{\"form\": \"default\", /" >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
    AZ_TRUNK_HEADS=1 timeout -k 10 200 python scripts/net_time.py 1024 40 | sed 's/^{/{"form": "readback", /' >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
    AZ_TRUNK_HEADS=1 AZ_LIB_PATH=$E timeout -k 10 200 python scripts/net_time.py 1024 40 | sed 's/^{/{"form": "epi", /' >> $OUT/net.jsonl 2>> $OUT/net.err || exit 1
  done
  cat $OUT/net.jsonl
  for r in 1 2; do
    timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_base_$r.log 2>&1 || exit 1
    echo "base $(tail -1 $OUT/ab_base_$r.log | cut -c1-110)"
    AZ_TRUNK_HEADS=1 AZ_LIB_PATH=$E timeout -k 10 400 python bench.py --skip-cpu --skip-kernel > $OUT/ab_epi_$r.log 2>&1 || exit 1
    echo "epi  $(tail -1 $OUT/ab_epi_$r.log | cut -c1-110)"
  done
  exit 0
}

c22() {
  # round 4, final library (tail skip, fill skip, heads in the persistent trunk): full GPU suite,
  # smoke, the default bench line, configs[3] / arena lines, eager kernel trace of configs[2]
  set -u
  export OUT=gpurun_out/r04v TMPDIR=/tmp
  mkdir -p $OUT
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
  tail -1 $OUT/smoke.log
  timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit 1
  tail -1 $OUT/bench.log | cut -c1-200
  timeout -k 10 500 python bench.py --workload c4 --skip-cpu > $OUT/bench_c4.log 2>&1 || exit 1
  echo "c4 $(tail -1 $OUT/bench_c4.log | cut -c1-140)"
  timeout -k 10 500 python bench.py --workload arena --matches 1024 > $OUT/bench_arena.log 2>&1 || exit 1
  echo "arena $(tail -1 $OUT/bench_arena.log | cut -c1-140)"
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_eager -o run -- python3 bench.py --skip-cpu --no-graph --steps 2000 > $OUT/trace_eager.log 2>&1
  echo "eager trace rc=$?"
  exit 0
}

c23() {
  # round 4, final library: the default bench line twice more and the configs[1] / configs[4]
  # lines (two pipelines), for the spread on one more box
  set -u
  export OUT=gpurun_out/r04w TMPDIR=/tmp
  mkdir -p $OUT
  for r in 1 2; do
    timeout -k 10 400 python bench.py --skip-cpu > $OUT/bench_$r.log 2>&1 || exit 1
    echo "c3 $(tail -1 $OUT/bench_$r.log | cut -c1-120)"
  done
  for w in c5 c2; do
    timeout -k 10 500 python bench.py --workload $w --skip-cpu > $OUT/bench_$w.log 2>&1 || exit 1
    echo "$w $(tail -1 $OUT/bench_$w.log | cut -c1-120)"
  done
  exit 0
}

c24() {
  # round 4, final library: configs[2] with one pipeline against two, alternating three times
  set -u
  export OUT=gpurun_out/r04x TMPDIR=/tmp
  mkdir -p $OUT
  for r in 1 2 3; do
    for p in 1 2; do
      timeout -k 10 400 python bench.py --skip-cpu --skip-kernel --pipelines $p > $OUT/c3_p${p}_$r.log 2>&1 || exit 1
      echo "p$p $(tail -1 $OUT/c3_p${p}_$r.log | cut -c1-110)"
    done
  done
  exit 0
}

c25() {
  # round 4, final library: the trunk conv's prefetch distances again (weight ring 2 / 3 / 4
  # steps ahead, input slices 1 / 2 chunks ahead) -- B = 1,024 evaluation time, alternating
  set -u -o pipefail
  export OUT=gpurun_out/r04y TMPDIR=/tmp
  mkdir -p $OUT
  for r in 1 2; do
    for v in tree pd2 pd4 ipd1; do
      if [ $v = tree ]; then L=""; else L=expbuild/$v/libaz_othello.so; fi
      AZ_LIB_PATH=$L timeout -k 10 200 python scripts/net_time.py 1024 40 | sed "s/^{/{\"variant\": \"$v\", /" >> $OUT/net.jsonl || exit 1
    done
  done
  cat $OUT/net.jsonl
  exit 0
}

c26() {
  # round 4, final: the default bench line with the new roofline_trunk object (the step's
  # dominant launch), and the smoke
  set -u
  export OUT=gpurun_out/r04z TMPDIR=/tmp
  mkdir -p $OUT
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
  tail -1 $OUT/smoke.log
  timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit 1
  tail -1 $OUT/bench.log | cut -c1-200
  exit 0
}

c27() {
  # round 4, last: the full GPU suite on the final tree
  set -u
  export OUT=gpurun_out/r04zz TMPDIR=/tmp
  mkdir -p $OUT
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; exit $rc
}

case "${1:-}" in
  c1|c2|c3|c4|c7|c8|c9|c10|c11|c12|c13|c14|c15|c16|c17|c18|c19|c20|c21|c22|c23|c24|c25|c26|c27) "$1" ;;
  *) echo "usage: $0 {c1|c2|c3|c4|c7|c8|c9|c10|c11|c12|c13|c14|c15|c16|c17|c18|c19|c20|c21|c22|c23|c24|c25|c26|c27}" >&2; exit 2 ;;
esac
