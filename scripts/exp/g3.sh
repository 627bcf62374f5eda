set -u
mkdir -p gpurun_out
bash scripts/pmc_conv_sq.sh az_conv3x3_wino4_gpu fp16 1024
bash scripts/pmc_conv_sq.sh az_conv3x3_wino4_gpu split3 1024
bash scripts/pmc_conv_sq.sh az_conv3x3_wino_gpu split3 1024
exit 0
