#!/bin/bash
# Round 5's GPU calls (gpurun), one function per call, in the order they ran; each writes
# under gpurun_out/r05<letter>/ and the summaries that were kept are copied to profiles/.
#     /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_calls_r05.sh c1
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
  # the reference-pinned net fixtures, the real-engine world-2 generation, the ADVICE tests,
  # then the default bench line (pattern ceiling + both trunk fractions); the heads probes;
  # the unchanged-pool drop-in rate; a graph-mode kernel trace with graph packet capture off
  export OUT=gpurun_out/r05a
  mkdir -p $OUT
  pyt pytest_new 600 tests/test_net_golden_gpu.py tests/test_dist_gpu.py \
    tests/test_arena_gpu.py tests/test_callers_gpu.py tests/test_engine_gpu.py || exit $?
  run bench 600 python bench.py
  run pk_ds_hazard 120 ./expbuild/pk_ds_hazard 4000
  run heads_paired 300 env AZ_LIB_PATH=expbuild/paired/libaz_othello.so python -u -m pytest \
    tests/test_nn_gpu.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "two_board or trunk_heads or fused_heads_bit_identical_to_separate_heads"
  run dropin_pool 400 python scripts/dropin_pool_bench.py 8 256 400
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_graph 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof -o run -- python3 bench.py --skip-cpu --steps 400 --warmup 2000
  exit 0
}

c2() {
  # the heads hazard with MFMA companions on the same SIMDs; configs[2]'s leaf batch with two
  # 1,024-slot pipelines (2,048 games) against the one-pipeline default, same box
  export OUT=gpurun_out/r05b
  mkdir -p $OUT
  run pk_ds_hazard 300 ./expbuild/pk_ds_hazard 4000
  run bench_1p 300 python bench.py --skip-cpu
  run bench_2x1024 300 python bench.py --skip-cpu --skip-kernel --games 2048 --pipelines 2
  run bench_1p_b 300 python bench.py --skip-cpu --skip-kernel
  run bench_2x1024_b 300 python bench.py --skip-cpu --skip-kernel --games 2048 --pipelines 2
  exit 0
}

c3() {
  # the layer hand-off (AZ_W4_HANDOFF=1) bit for bit against the layer launches and the
  # reference fixtures; then the product, the packed epilogue (AZ_W4_EPI_PK=1) and the
  # hand-off and the packed transform ops (AZ_W4_PK2=1) timed alternately on one box
  export OUT=gpurun_out/r05c
  mkdir -p $OUT
  run hoff_tests 400 env AZ_LIB_PATH=expbuild/hoff/libaz_othello.so python -u -m pytest \
    tests/test_nn_gpu.py tests/test_net_golden_gpu.py -m gpu -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "persistent or trunk_heads or golden or matches" \
    || exit $?
  for i in 1 2; do
    run net_base 120 python scripts/net_time.py 1024 40
    run net_epk 120 env AZ_LIB_PATH=expbuild/epk/libaz_othello.so python scripts/net_time.py 1024 40
    run net_hoff 120 env AZ_LIB_PATH=expbuild/hoff/libaz_othello.so python scripts/net_time.py 1024 40
    run net_pk2 120 env AZ_LIB_PATH=expbuild/pk2/libaz_othello.so python scripts/net_time.py 1024 40
  done
  exit 0
}

c4() {
  # the one-game-per-call drop-in (AZ_DROPIN_BATCH=1) re-measured with this library: one game
  # through the unchanged caller, and train.py's pool of 8 workers
  export OUT=gpurun_out/r05d
  mkdir -p $OUT
  run dropin 400 env AZ_DROPIN_BATCH=1 python scripts/dropin_bench.py
  run dropin_pool_1 400 env AZ_DROPIN_BATCH=1 python scripts/dropin_pool_bench.py 8 16 400
  exit 0
}

c5() {
  # the whole GPU suite and smoke() on the library with the epilogue pairs and the layer
  # hand-off on; the bench line; the unchanged-caller drop-in re-measured (c4's steps)
  export OUT=gpurun_out/r05e
  mkdir -p $OUT
  run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread || exit $?
  run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
  run bench 600 python bench.py
  run net_base0 120 env AZ_LIB_PATH=expbuild/base0/libaz_othello.so python scripts/net_time.py 1024 40
  run net_tree 120 python scripts/net_time.py 1024 40
  run dropin 400 env AZ_DROPIN_BATCH=1 python scripts/dropin_bench.py
  run dropin_pool_1 400 env AZ_DROPIN_BATCH=1 python scripts/dropin_pool_bench.py 8 16 400
  exit 0
}

c6() {
  # the final library: the heads check build's stress (every differing value-path word
  # printed), the persistent trunk's SQ / TA counters (one group per --pmc pass), and a
  # graph-mode kernel trace of the bench (graph packet capture off, r05_tracer_fault_decode)
  export OUT=gpurun_out/r05f
  mkdir -p $OUT
  K="persistent_trunk or trunk_heads or fused_heads or two_board"
  run hchk 400 env AZ_LIB_PATH=expbuild/hchk/libaz_othello.so python -u -m pytest \
    tests/test_nn_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "$K"
  echo "HEADS_CHECK lines: $(grep -c HEADS_CHECK $OUT/hchk.log)" | tee -a $OUT/steps.log
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
             "GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_TA_BUSY_sum" \
             "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    run sq_trunk_$i 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/sq_trunk_$i -o pmc -- \
      python3 scripts/trunk_one.py 1024 20 calib || exit $?
  done
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_graph 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof -o run -- python3 bench.py --skip-cpu --steps 400 --warmup 2000
  exit 0
}

c7() {
  # the N > 1 bench path rehearsed on the one-GPU box (AZ_BENCH_REHEARSE=1: every rank on
  # cuda:0, gloo collectives): torchrun world 2 and world 4, the driver's command shape
  export OUT=gpurun_out/r05g
  mkdir -p $OUT
  run rehearse_w2 400 env AZ_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --skip-cpu
  run rehearse_w4 500 env AZ_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --skip-cpu \
    --steps 2000
  # where the persistent trunk's vector-memory requests are served: L1 accesses and misses
  # (requests to L2), L2 hits and misses
  i=0
  for grp in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
             "TCP_TCC_WRITE_REQ_sum TCC_REQ_sum TCC_EA0_RDREQ_sum"; do
    i=$((i+1))
    run l1l2_trunk_$i 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/l1l2_trunk_$i -o pmc -- \
      python3 scripts/trunk_one.py 1024 20 || exit $?
  done
  exit 0
}

c8() {
  # the next layer's first weight steps requested before the layer fence (AZ_W4_WPRE=1):
  # bit-identity tests, then timed against the product alternately
  export OUT=gpurun_out/r05h
  mkdir -p $OUT
  run wpre_tests 400 env AZ_LIB_PATH=expbuild/wpre/libaz_othello.so python -u -m pytest \
    tests/test_nn_gpu.py tests/test_net_golden_gpu.py -m gpu -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "persistent or trunk_heads or golden or matches" \
    || exit $?
  for i in 1 2 3; do
    run net_tree 120 python scripts/net_time.py 1024 40
    run net_wpre 120 env AZ_LIB_PATH=expbuild/wpre/libaz_othello.so python scripts/net_time.py 1024 40
  done
  exit 0
}

c9() {
  # the round's final tree: the whole GPU suite, smoke() and the default bench line
  export OUT=gpurun_out/r05i
  mkdir -p $OUT
  run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread || exit $?
  run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
  run bench 600 python bench.py
  exit 0
}

c10() {
  # the other workloads on the final library (README quoted round 4's): configs[1] (c2),
  # configs[3] (c4), configs[4] (c5), the arena
  export OUT=gpurun_out/r05j
  mkdir -p $OUT
  run c2 500 python bench.py --workload c2 --skip-cpu --skip-kernel
  run c4 500 python bench.py --workload c4 --skip-cpu --skip-kernel
  run c5 500 python bench.py --workload c5 --skip-cpu --skip-kernel
  run arena 600 python bench.py --workload arena --matches 1024
  exit 0
}

c11() {
  # upper bounds for a layer-resident input (wrong results): no in-loop input-slice loads /
  # LDS stores (EXP 64), no global stores of conv1 outputs (EXP 128), both (EXP 192)
  export OUT=gpurun_out/r05k
  mkdir -p $OUT
  for i in 1 2; do
    run net_tree 120 python scripts/net_time.py 1024 40
    for v in x64 x128 x192; do
      run net_$v 120 env AZ_LIB_PATH=expbuild/$v/libaz_othello.so python scripts/net_time.py 1024 40
    done
  done
  exit 0
}

c12() {
  # the layer input resident in LDS (AZ_W4_RESIDENT=1): the trunk / heads bit-identity tests and
  # the reference fixtures, then timed against the product alternately
  export OUT=gpurun_out/r05l
  mkdir -p $OUT
  run rsd_tests 400 env AZ_LIB_PATH=expbuild/rsd/libaz_othello.so python -u -m pytest \
    tests/test_nn_gpu.py tests/test_net_golden_gpu.py -m gpu -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "persistent or trunk_heads or golden or matches or two_board" \
    || exit $?
  for i in 1 2 3; do
    run net_tree 120 python scripts/net_time.py 1024 40
    run net_rsd 120 env AZ_LIB_PATH=expbuild/rsd/libaz_othello.so python scripts/net_time.py 1024 40
  done
  run bench_tree 300 python bench.py --skip-cpu --skip-kernel
  run bench_rsd 300 env AZ_LIB_PATH=expbuild/rsd/libaz_othello.so python bench.py --skip-cpu --skip-kernel
  exit 0
}

c13() {
  # what the resident trunk still pays (wrong-result builds): the RES epilogues' global residual
  # reads (EXP 256), the X write-out (EXP 512)
  export OUT=gpurun_out/r05m
  mkdir -p $OUT
  for i in 1 2; do
    run net_tree 120 python scripts/net_time.py 1024 40
    for v in x256 x512; do
      run net_$v 120 env AZ_LIB_PATH=expbuild/$v/libaz_othello.so python scripts/net_time.py 1024 40
    done
  done
  exit 0
}

c14() {
  # the resident trunk's residual staged in X's odd rows (AZ_W4_RXS=1): trunk / heads tests,
  # then timed against the product alternately, and the bench
  export OUT=gpurun_out/r05n
  mkdir -p $OUT
  run rxs_tests 400 env AZ_LIB_PATH=expbuild/rxs/libaz_othello.so python -u -m pytest \
    tests/test_nn_gpu.py tests/test_net_golden_gpu.py -m gpu -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "persistent or trunk_heads or golden or matches or two_board" \
    || exit $?
  for i in 1 2 3; do
    run net_tree 120 python scripts/net_time.py 1024 40
    run net_rxs 120 env AZ_LIB_PATH=expbuild/rxs/libaz_othello.so python scripts/net_time.py 1024 40
  done
  run bench_tree 300 python bench.py --skip-cpu --skip-kernel
  run bench_rxs 300 env AZ_LIB_PATH=expbuild/rxs/libaz_othello.so python bench.py --skip-cpu --skip-kernel
  exit 0
}

c15() {
  # the final tree (resident trunk + residual staging): the whole GPU suite, smoke(), the bench
  # line, a graph-mode kernel trace, the trunk's SQ / TA / L2 counters (OUT overridable: r05o
  # was the first final tree, r05v the one after the raw LDS addresses)
  export OUT=${OUT:-gpurun_out/r05o}
  mkdir -p $OUT
  run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread || exit $?
  run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
  run bench 600 python bench.py
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_graph 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof -o run -- python3 bench.py --skip-cpu --steps 400 --warmup 2000
  unset DEBUG_CLR_GRAPH_PACKET_CAPTURE
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
             "GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_TA_BUSY_sum" \
             "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES" \
             "FETCH_SIZE" "WRITE_SIZE" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    run sq_trunk_$i 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/sq_trunk_$i -o pmc -- \
      python3 scripts/trunk_one.py 1024 20 calib || exit $?
  done
  exit 0
}

c16() {
  # what binds the resident trunk now (wrong-result builds): no weight loads (EXP 1), no
  # transform / window work (EXP 2), no MFMAs (EXP 4), no chunk barrier (EXP 8)
  export OUT=gpurun_out/r05p
  mkdir -p $OUT
  for i in 1 2; do
    run net_tree 120 python scripts/net_time.py 1024 40
    for v in e1 e2 e4 e8; do
      run net_$v 120 env AZ_LIB_PATH=expbuild/$v/libaz_othello.so python scripts/net_time.py 1024 40
    done
  done
  exit 0
}

c17() {
  # the resident trunk's sensitivity to the weight prefetch distance (AZ_W4_PD3 = 3 default)
  export OUT=gpurun_out/r05q
  mkdir -p $OUT
  for i in 1 2; do
    run net_tree 120 python scripts/net_time.py 1024 40
    for v in pd2 pd1; do
      run net_$v 120 env AZ_LIB_PATH=expbuild/$v/libaz_othello.so python scripts/net_time.py 1024 40
    done
  done
  exit 0
}

c18() {
  # the resident trunk in four-board eight-wave workgroups, one per CU (AZ_W4_TRUNK_BOARDS=4):
  # trunk / heads tests, then timed against the product alternately, and the bench
  export OUT=gpurun_out/r05r
  mkdir -p $OUT
  run tb4_tests 400 env AZ_LIB_PATH=expbuild/tb4/libaz_othello.so python -u -m pytest \
    tests/test_nn_gpu.py tests/test_net_golden_gpu.py -m gpu -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "persistent or trunk_heads or golden or matches or two_board" \
    || exit $?
  for i in 1 2; do
    run net_tree 120 python scripts/net_time.py 1024 40
    run net_tb4 120 env AZ_LIB_PATH=expbuild/tb4/libaz_othello.so python scripts/net_time.py 1024 40
  done
  run bench_tree 300 python bench.py --skip-cpu --skip-kernel
  run bench_tb4 300 env AZ_LIB_PATH=expbuild/tb4/libaz_othello.so python bench.py --skip-cpu --skip-kernel
  exit 0
}

c19() {
  # the other workloads on the final (resident-trunk) library
  export OUT=gpurun_out/r05s
  mkdir -p $OUT
  run c2 500 python bench.py --workload c2 --skip-cpu --skip-kernel
  run c4 500 python bench.py --workload c4 --skip-cpu --skip-kernel
  run c5 500 python bench.py --workload c5 --skip-cpu --skip-kernel
  run arena 600 python bench.py --workload arena --matches 1024
  exit 0
}

c20() {
  # the select launch's level budget (AZ_SEL_LEVELS, 14 since round 3) re-tuned with the
  # faster trunk: configs[2] bench lines alternated on one box
  export OUT=gpurun_out/r05t
  mkdir -p $OUT
  for i in 1 2; do
    run bench_tree 300 python bench.py --skip-cpu --skip-kernel
    for v in lv10 lv12 lv18; do
      run bench_$v 300 env AZ_LIB_PATH=expbuild/$v/libaz_othello.so python bench.py --skip-cpu --skip-kernel
    done
  done
  exit 0
}

c21() {
  # window reads at raw LDS addresses (no add of the LDS symbol): trunk tests, then timed
  # against the previous build (expbuild/prev) alternately
  export OUT=gpurun_out/r05u
  mkdir -p $OUT
  run tests 400 python -u -m pytest tests/test_nn_gpu.py tests/test_net_golden_gpu.py -m gpu -x -v \
    -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "persistent or trunk_heads or golden or matches or two_board" || exit $?
  for i in 1 2 3; do
    run net_tree 120 python scripts/net_time.py 1024 40
    run net_prev 120 env AZ_LIB_PATH=expbuild/prev/libaz_othello.so python scripts/net_time.py 1024 40
  done
  exit 0
}

c22() {
  # the select launch's terminal backups from registers (AZ_SEL_REGBACKUP=1): the engine and
  # bench-path parity tests on that build, then configs[2] benches alternated
  export OUT=gpurun_out/r05w
  mkdir -p $OUT
  run rb_tests 900 env AZ_LIB_PATH=expbuild/rb/libaz_othello.so python -u -m pytest \
    tests/test_bench_path_gpu.py tests/test_engine_gpu.py tests/test_vl_gpu.py \
    tests/test_callers_gpu.py tests/test_fullwidth_gpu.py -m gpu -x -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread || exit $?
  for i in 1 2; do
    run bench_tree 300 python bench.py --skip-cpu --skip-kernel
    run bench_rb 300 env AZ_LIB_PATH=expbuild/rb/libaz_othello.so python bench.py --skip-cpu --skip-kernel
  done
  exit 0
}

c23() {
  # HBM bytes of the bench's trunk launch (az_trunk_wino4_heads_gpu: stem + convs + heads),
  # for roofline_trunk.traffic: FETCH_SIZE and WRITE_SIZE passes, and a kernel trace of it
  export OUT=gpurun_out/r05x
  mkdir -p $OUT
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    run hbm_$i 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/hbm_$i -o pmc -- \
      python3 scripts/trunk_heads_one.py 1024 20 || exit $?
  done
  run trace 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 scripts/trunk_heads_one.py 1024 20
  exit 0
}

c24() {
  # configs[2] as two 512-slot pipelines on their own streams (one pipeline's select beside the
  # other's trunk) against one pipeline, with the resident-input trunk; alternated
  export OUT=gpurun_out/r05y
  mkdir -p $OUT
  for i in 1 2; do
    run bench_1p 300 python bench.py --skip-cpu --skip-kernel
    run bench_2p 300 python bench.py --skip-cpu --skip-kernel --pipelines 2
  done
  exit 0
}

c25() {
  # configs[2]'s leaf batch of 1,024 with two pipelines: 2,048 games as two 1,024-slot
  # pipelines against one 1,024-slot pipeline, resident-input trunk; alternated
  export OUT=gpurun_out/r05z
  mkdir -p $OUT
  for i in 1 2; do
    run bench_1p 300 python bench.py --skip-cpu --skip-kernel
    run bench_2x1024 300 python bench.py --skip-cpu --skip-kernel --games 2048 --pipelines 2
  done
  exit 0
}

c26() {
  # configs[3]'s 4,096 games per GPU as two 2,048-slot pipelines against one, resident trunk
  export OUT=gpurun_out/r05aa
  mkdir -p $OUT
  for i in 1 2; do
    run c4_1p 500 python bench.py --workload c4 --skip-cpu --skip-kernel --pipelines 1
    run c4_2p 500 python bench.py --workload c4 --skip-cpu --skip-kernel --pipelines 2
  done
  exit 0
}

c27() {
  # configs[2] with three / four 1,024-game pipelines against the two-pipeline default
  export OUT=gpurun_out/r05ac
  mkdir -p $OUT
  for i in 1 2; do
    run bench_2p 300 python bench.py --skip-cpu --skip-kernel
    run bench_3p 400 python bench.py --skip-cpu --skip-kernel --pipelines 3
    run bench_4p 400 python bench.py --skip-cpu --skip-kernel --pipelines 4
  done
  exit 0
}

c28() {
  # one vs two 1,024-game pipelines again, alternated three times on one box
  export OUT=gpurun_out/r05ad
  mkdir -p $OUT
  for i in 1 2 3; do
    run bench_1p 300 python bench.py --skip-cpu --skip-kernel --pipelines 1
    run bench_2p 300 python bench.py --skip-cpu --skip-kernel
  done
  exit 0
}

c29() {
  # round-3 scheduling knobs re-tested on the resident trunk: sched_group_barrier interleave
  # (AZ_W4_SCHED 1 / 2 VALU per MFMA), s_setprio around the MFMA clusters (AZ_W4_PRIO=2)
  export OUT=gpurun_out/r05ae
  mkdir -p $OUT
  for i in 1 2; do
    run net_tree 120 python scripts/net_time.py 1024 40
    for v in s1 s2 p2; do
      run net_$v 120 env AZ_LIB_PATH=expbuild/$v/libaz_othello.so python scripts/net_time.py 1024 40
    done
  done
  exit 0
}

c30() {
  # the merged select + move launch reserves the move phase's 64 KiB of LDS for every select
  # workgroup: beside the other pipeline's trunk it blocks the trunk's second workgroup on
  # a CU.  Moves in their own launch (--no-defer) against the default, two and one pipelines
  export OUT=gpurun_out/r05af
  mkdir -p $OUT
  for i in 1 2; do
    run bench_2p 300 python bench.py --skip-cpu --skip-kernel
    run bench_2p_nodefer 300 python bench.py --skip-cpu --skip-kernel --no-defer
    run bench_1p_nodefer 300 python bench.py --skip-cpu --skip-kernel --no-defer --pipelines 1
  done
  exit 0
}

c31() {
  # the deferred move phase as a forked launch (AZ_SEL_FORK=1: the select launch reserves no
  # LDS): the engine / bench-path / pipelined parity tests with it, then benches
  export OUT=gpurun_out/r05ag
  mkdir -p $OUT
  run fork_tests 900 env AZ_SEL_FORK=1 python -u -m pytest tests/test_bench_path_gpu.py \
    tests/test_engine_gpu.py tests/test_pipelined_gpu.py tests/test_vl_gpu.py -m gpu -x -v \
    -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
  for i in 1 2; do
    run bench_2p 300 python bench.py --skip-cpu --skip-kernel
    run bench_2p_fork 300 env AZ_SEL_FORK=1 python bench.py --skip-cpu --skip-kernel
    run bench_1p 300 python bench.py --skip-cpu --skip-kernel --pipelines 1
    run bench_1p_fork 300 env AZ_SEL_FORK=1 python bench.py --skip-cpu --skip-kernel --pipelines 1
  done
  exit 0
}

c32() {
  # host-side knobs with two pipelines: steps per HIP graph (8 default), the select launch's
  # descent cap (AZ_MAX_DESCENTS, 4 default)
  export OUT=gpurun_out/r05ah
  mkdir -p $OUT
  for i in 1 2; do
    run bench_def 300 python bench.py --skip-cpu --skip-kernel
    run bench_spg16 300 python bench.py --skip-cpu --skip-kernel --steps-per-graph 16
    run bench_md8 300 env AZ_MAX_DESCENTS=8 python bench.py --skip-cpu --skip-kernel
    run bench_md2 300 env AZ_MAX_DESCENTS=2 python bench.py --skip-cpu --skip-kernel
  done
  exit 0
}

c33() {
  # the four-board resident trunk (one workgroup per CU, all 160 KiB) with two pipelines
  export OUT=gpurun_out/r05ai
  mkdir -p $OUT
  for i in 1 2; do
    run bench_2p 300 python bench.py --skip-cpu --skip-kernel
    run bench_2p_tb4 300 env AZ_LIB_PATH=expbuild/tb4/libaz_othello.so python bench.py --skip-cpu --skip-kernel
  done
  exit 0
}

c34() {
  # the pipelined test with bench.py's configs[2] shape (2 x 1,024 games)
  export OUT=gpurun_out/r05aj
  mkdir -p $OUT
  run pytest_pipe 400 python -u -m pytest tests/test_pipelined_gpu.py -m gpu -x -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread || exit $?
  exit 0
}

c35() {
  # configs[4] (fp16 + D4): the direct fp16 conv (default) against the per-layer fp16 Winograd
  # conv (AZ_CONV_ALGO=wino4), speed and the fp16 accuracy tests
  export OUT=gpurun_out/r05ak
  mkdir -p $OUT
  run bench_c5 300 python bench.py --workload c5 --skip-cpu --skip-kernel
  run bench_c5_w4 300 env AZ_CONV_ALGO=wino4 python bench.py --workload c5 --skip-cpu --skip-kernel
  run bench_c5_w 300 env AZ_CONV_ALGO=wino python bench.py --workload c5 --skip-cpu --skip-kernel
  run pytest_w4 400 env AZ_CONV_ALGO=wino4 python -u -m pytest tests/test_c5_gpu.py tests/test_net_golden_gpu.py \
    -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
  exit 0
}

c36() {
  # stream priorities of the two pipelines (AZ_PIPE_PRIO)
  export OUT=gpurun_out/r05am
  mkdir -p $OUT
  run prio_range 60 python -c "import torch; print(torch.cuda.Stream.priority_range())"
  for i in 1 2; do
    run bench_2p 300 python bench.py --skip-cpu --skip-kernel
    run bench_prio_hi_lo 300 env AZ_PIPE_PRIO=-1,0 python bench.py --skip-cpu --skip-kernel
  done
  exit 0
}

c37() {
  # the fp16 persistent trunk (az_trunk_wino4_heads_fp16_gpu): parity, then configs[4] with the
  # fp16 wino4 convs on it against the direct fp16 default
  export OUT=gpurun_out/r05an
  mkdir -p $OUT
  run pytest_fp16trunk 300 python -u -m pytest tests/test_net_golden_gpu.py -m gpu -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread || exit $?
  run pytest_c5_w4 400 env AZ_CONV_ALGO=wino4 python -u -m pytest tests/test_c5_gpu.py tests/test_pipelined_gpu.py \
    -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
  for i in 1 2; do
    run bench_c5 300 python bench.py --workload c5 --skip-cpu --skip-kernel || exit $?
    run bench_c5_w4t 300 env AZ_CONV_ALGO=wino4 python bench.py --workload c5 --skip-cpu --skip-kernel || exit $?
  done
  run net_fp16_direct 120 python scripts/net_time.py 1024 40 fp16
  run net_fp16 120 env AZ_CONV_ALGO=wino4 python scripts/net_time.py 1024 40 fp16
  run net_fp16_w4_layers 120 env AZ_CONV_ALGO=wino4 AZ_TRUNK_FP16=0 python scripts/net_time.py 1024 40 fp16
  exit 0
}

c38() {
  # fp16 at 128 channels defaults to the wino4 convs (the persistent fp16 trunk): the whole GPU
  # suite, smoke(), configs[4] and configs[2] bench lines
  export OUT=gpurun_out/r05ao
  mkdir -p $OUT
  run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread || exit $?
  run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
  run bench_c5 400 python bench.py --workload c5 || exit $?
  run bench 600 python bench.py
  exit 0
}

c39() {
  # configs[4] and configs[3] lines with roofline_trunk (fp16 trunk; chunked evaluations), and
  # configs[4]'s kernel profile
  export OUT=gpurun_out/r05ap
  mkdir -p $OUT
  run bench_c5 400 python bench.py --workload c5 || exit $?
  run bench_c4 400 python bench.py --workload c4 --skip-cpu || exit $?
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c5 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --workload c5 --skip-cpu --skip-kernel --steps 400 --warmup 2000
  exit 0
}

c40() {
  # configs[1] (FastOthelloNet, 4,096 games, 100 sims): kernel profile
  export OUT=gpurun_out/r05ar
  mkdir -p $OUT
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c2 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000
  rm -f $OUT/prof_c2/run_kernel_trace.csv
  exit 0
}

c41() {
  # FastOthelloNet's fused heads (one GEMM + az_heads_fast_finish_gpu): parity, configs[1] A/B
  # and its kernel profile
  export OUT=gpurun_out/r05as
  mkdir -p $OUT
  run pytest_fast 400 python -u -m pytest tests/test_net_golden_gpu.py tests/test_pipelined_gpu.py tests/test_nn_gpu.py \
    -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "fast" || exit $?
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_unfused 300 env AZ_FAST_HEADS=0 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c2 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000
  rm -f $OUT/prof_c2/run_kernel_trace.csv
  exit 0
}

c42() {
  # FastOthelloNet heads GEMM in nn.Linear's weight layout; configs[1] with the Winograd split3
  # convs at 64 channels
  export OUT=gpurun_out/r05at
  mkdir -p $OUT
  run pytest_fast 400 python -u -m pytest tests/test_net_golden_gpu.py -m gpu -x -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "fast" || exit $?
  for i in 1 2; do
    run bench_c2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_wino 300 env AZ_CONV_ALGO=wino python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c2 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000
  rm -f $OUT/prof_c2/run_kernel_trace.csv
  exit 0
}

c43() {
  # FastOthelloNet heads GEMM split over the reduction (AZ_FAST_SPLITK 1 / 4 / 8)
  export OUT=gpurun_out/r05au
  mkdir -p $OUT
  run pytest_fast 400 python -u -m pytest tests/test_net_golden_gpu.py tests/test_pipelined_gpu.py -m gpu -x -v \
    -p no:cacheprovider --timeout 300 --timeout-method thread -k "fast" || exit $?
  for i in 1 2; do
    run bench_c2_s4 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_s1 300 env AZ_FAST_SPLITK=1 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_s8 300 env AZ_FAST_SPLITK=8 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
  done
  export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run rocprof_c2 500 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --skip-cpu --skip-kernel --steps 400 --warmup 2000
  rm -f $OUT/prof_c2/run_kernel_trace.csv
  exit 0
}

c44() {
  # the final tree (fp16 persistent trunk default, FastOthelloNet fused heads): the whole GPU
  # suite, smoke(), the default bench line and the configs[1] line
  export OUT=gpurun_out/r05av
  mkdir -p $OUT
  run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread || exit $?
  run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
  run bench 600 python bench.py || exit $?
  run bench_c2 400 python bench.py --workload c2 || exit $?
  exit 0
}

c45() {
  # configs[1] with the fused fast heads: 1 / 2 / 4 pipelines
  export OUT=gpurun_out/r05aw
  mkdir -p $OUT
  for i in 1 2; do
    run bench_c2_p2 300 python bench.py --workload c2 --skip-cpu --skip-kernel || exit $?
    run bench_c2_p4 300 python bench.py --workload c2 --skip-cpu --skip-kernel --pipelines 4 || exit $?
    run bench_c2_p1 300 python bench.py --workload c2 --skip-cpu --skip-kernel --pipelines 1 || exit $?
  done
  exit 0
}

"$@"
