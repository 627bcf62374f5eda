set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== nrt1"; AZ_W4_NRT=1 CONV_AB_ONLY=wino4 timeout -k 10 120 python -u scripts/conv_ab.py 1024 2>&1 | grep '^{' || exit 1
echo "== nrt2"; CONV_AB_ONLY=wino4 timeout -k 10 120 python -u scripts/conv_ab.py 1024 2>&1 | grep '^{' || exit 1
bash scripts/pmc_conv_sq.sh az_conv3x3_wino4_gpu fp16x2 1024
python scripts/sq_summary.py gpurun_out/sq_wino4_fp16x2
