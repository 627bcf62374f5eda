# conv_ab (wino4 only, B=1024) on each library given
set -u
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  AZ_LIB_PATH=scripts/exp/_ab/$v.so AZ_W4_NRT=${NRT:-1} CONV_AB_ONLY=wino4 timeout -k 10 120 python -u scripts/conv_ab.py 1024 2>&1 | grep '^{' || exit 1
done
