set -u
mkdir -p gpurun_out
for v in pd3ipd1 pd5ipd1 pd3ipd2; do
  for n in 2 1; do
    AZ_LIB_PATH=expbuild/$v/libaz_othello.so AZ_W4_NRT=$n timeout -k 10 200 python -u scripts/conv_ab.py 1024 > gpurun_out/ab_${v}_$n.log 2>&1 || exit 1
    echo "== $v NRT=$n"; grep wino4 gpurun_out/ab_${v}_$n.log
  done
done
exit 0
