#!/bin/bash
# rocprofv3 counter passes on the bitboard-step kernel (one counter group per pass, no
# tracing domains beside --pmc), CSV output under gpurun_out/pmc_*/.
set -u
export TMPDIR=/tmp
N=${N:-16777216}
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_$tag -o pmc -- \
    python3 scripts/step_kernel_bench.py $N 5 > gpurun_out/pmc_$tag.log 2>&1
  rc=$?
  echo "pmc $grp rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
