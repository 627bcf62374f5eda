"""k_step duration over a long back-to-back run (per-launch HIP event pairs): how the
launch time evolves as the chip's clocks settle under sustained load.  Not product code."""
import json, os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import bench

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
kb = bench.StepKernelBench(1 << 24, torch.device("cuda", 0))
nat = kb.nat
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
for e0, e1 in evs:
    e0.record(); nat.lib.oth_step_gpu(*kb.args); e1.record()
torch.cuda.synchronize()
d = np.array([e0.elapsed_time(e1) for e0, e1 in evs])
w = max(1, reps // 30)
out = {"reps": reps, "window_means_ms": [round(float(d[i:i + w].mean()), 4) for i in range(0, reps, w)],
       "first20": [round(float(x), 4) for x in d[:20]],
       "median_last_half": round(float(np.median(d[reps // 2:])), 4),
       "mean_all": round(float(d.mean()), 4)}
print(json.dumps(out))
