#!/bin/bash
# SQ / TA / GRBM counter passes (one group per pass, --pmc only) on one trunk-conv kernel:
#   bash scripts/pmc_conv_sq.sh az_conv3x3_wino4_gpu split3 1024
# CSVs under gpurun_out/sq_<tag>_<pass>/.  A pass whose counters the tool rejects is
# reported and skipped (each pass is killed after 60 s).
set -u
export TMPDIR=/tmp
K=$1; M=$2; B=$3; TAG=${TAG:-$(echo $K | sed 's/az_conv3x3_//;s/_gpu//')_$M}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_TA_BUSY_sum" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM SQ_ACTIVE_INST_EXP"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/sq_${TAG}_$i -o pmc -- \
    python3 scripts/conv_one.py $K $M $B 20 > gpurun_out/sq_${TAG}_$i.log 2>&1
  echo "pass $i rc=$?: $grp"
done
exit 0
