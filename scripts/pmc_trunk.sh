#!/bin/bash
# rocprofv3 counter passes (one group per pass, --pmc only) on the shipped trunk forms at
# B = 1,024: the persistent two-board trunk (scripts/trunk_one.py: 10 convs per dispatch) and
# the two-board single conv (scripts/conv_one.py); SQ groups of pmc_conv_sq.sh + HBM bytes
set -u
export TMPDIR=/tmp
O=${OUT:-gpurun_out}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_TA_BUSY_sum" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/sq_trunk_$i -o pmc -- \
    python3 scripts/trunk_one.py 1024 20 calib > $O/sq_trunk_$i.log 2>&1
  echo "trunk pass $i rc=$?: $grp"
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/sq_conv2_$i -o pmc -- \
    python3 scripts/conv_one.py az_conv3x3_wino4_gpu fp16x2 1024 20 calib > $O/sq_conv2_$i.log 2>&1
  echo "conv pass $i rc=$?: $grp"
done
exit 0
