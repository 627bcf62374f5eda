#!/bin/bash
# rocprofv3 HBM counter passes on the trunk conv in its default form (az_conv3x3_wino4_gpu,
# fp16x2, two boards per workgroup, B = 1,024 x 128 channels, residual + ReLU -- the conv
# bench.py's roofline_conv times), one counter group per pass, no tracing domains beside
# --pmc; CSVs under gpurun_out/pmcc_*/, summarised by scripts/pmc_conv_summary.py.
set -u
export TMPDIR=/tmp
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcc_$grp -o pmc -- \
    python3 scripts/conv_one.py az_conv3x3_wino4_gpu fp16x2 1024 20 calib \
    > gpurun_out/pmcc_$grp.log 2>&1
  rc=$?
  echo "pmc conv $grp rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
