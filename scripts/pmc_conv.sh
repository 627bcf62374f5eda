#!/bin/bash
# rocprofv3 counter passes on the trunk conv (k_conv3x3_wino), one counter group per pass,
# no tracing domains beside --pmc; CSV output under gpurun_out/pmcc_*/.
set -u
export TMPDIR=/tmp
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcc_$grp -o pmc -- \
    python3 scripts/conv_kernel_bench.py 5 > gpurun_out/pmcc_$grp.log 2>&1
  rc=$?
  echo "pmc conv $grp rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
