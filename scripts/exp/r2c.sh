set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 1 2 1 2; do
  AZ_W4_NRT=$n timeout -k 10 300 python -u bench.py --skip-cpu --skip-kernel --steps 4000 > gpurun_out/bench_nrt$n.log 2>&1 || exit 1
  echo "nrt=$n $(tail -1 gpurun_out/bench_nrt$n.log | cut -c1-200)"
done
AZ_W4_NRT=1 TAG=wino4_fp16x2_nrt1 bash scripts/pmc_conv_sq.sh az_conv3x3_wino4_gpu fp16x2 1024
python scripts/sq_summary.py gpurun_out/sq_wino4_fp16x2_nrt1
