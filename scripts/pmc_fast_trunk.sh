#!/bin/bash
# rocprofv3 counter passes (one group per pass, --pmc only) on FastOthelloNet's one-launch trunk
# at B = 2,048 (scripts/fast_trunk_one.py): the SQ groups of pmc_trunk.sh + HBM bytes
set -u
export TMPDIR=/tmp
O=${OUT:-gpurun_out}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_TA_BUSY_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/sq_fast_$i -o pmc -- \
    python3 scripts/fast_trunk_one.py 2048 20 > $O/sq_fast_$i.log 2>&1
  rc=$?
  echo "fast trunk pass $i rc=$rc: $grp"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
