set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/nn.log 2>&1; rc=$?; tail -2 gpurun_out/nn.log; [ $rc -ne 0 ] && exit $rc
bash scripts/exp/conv_exp.sh w4base w4perm w4base w4perm
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU --output-format csv -d gpurun_out/sq_perm_1 -o pmc -- python3 scripts/conv_one.py az_conv3x3_wino4_gpu fp16x2 1024 20 > /dev/null 2>&1
python scripts/sq_summary.py gpurun_out/sq_perm
