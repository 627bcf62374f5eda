set -u
mkdir -p gpurun_out
for v in stamp proxy2; do
echo "== $v"
AZ_LIB_PATH=expbuild/$v/libaz_othello.so AZ_W4_NRT=2 timeout -k 10 120 python -u scripts/w4_stamps.py split3 1024 2>&1 | grep -v amdgpu.ids || exit 1
done
exit 0
