#!/bin/bash
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
