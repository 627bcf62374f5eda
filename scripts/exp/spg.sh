set -u
mkdir -p gpurun_out
for g in 8 1 2 4 8; do
  timeout -k 10 200 python bench.py --skip-cpu --skip-kernel --steps-per-graph $g > gpurun_out/spg_$g.log 2>&1 || exit $?
  echo "spg $g: $(tail -1 gpurun_out/spg_$g.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
