"""Steady-state (every slot playing) per-kernel times of one simulation step: after the
bench's staggered warmup (graph replay), eager steps with a HIP event pair around each phase
on the launch stream (select / net / expand / move), averaged over `n` steps, beside the
graph-replay ms/step.  The engine kernels' cost depends on how many slots are active and how
deep their trees are, so an idle-engine profile (a short warmup) under-states them.

    python scripts/phase_times.py [warm_steps] [n] [games] [leaves] > out.json"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import bench  # noqa: E402
from engine import BatchedSelfPlay  # noqa: E402
from Models import AlphaZeroNet  # noqa: E402

warm = int(sys.argv[1]) if len(sys.argv) > 1 else 26000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
games = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
leaves = int(sys.argv[4]) if len(sys.argv) > 4 else 1
torch.manual_seed(0)
sp = BatchedSelfPlay(AlphaZeroNet(8, 65, 5, 128), bench.SELFPLAY_ARGS, games, seed=1,
                     leaves_per_step=leaves)
stagger = (-(-400 // leaves) + 1) * 60
sp.reset(-1, stagger)
done = 0
while done < warm:
    sp.step(2000)
    torch.cuda.synchronize()
    done += 2000
    print(json.dumps({"warm": done}), file=sys.stderr, flush=True)
t0 = time.perf_counter()
sp.step(2000)
torch.cuda.synchronize()
graph_ms = (time.perf_counter() - t0) / 2
e = sp.engine
names = ["select", "net", "expand", "move"]
tot = {k: 0.0 for k in names}
evs = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
with torch.no_grad():
    for _ in range(n):
        evs[0].record()
        e.select()
        evs[1].record()
        sp.net.evaluate_into(e.nn_in, e.priors, e.values)
        evs[2].record()
        e.expand()
        evs[3].record()
        e.play()
        evs[4].record()
        torch.cuda.synchronize()
        for i, k in enumerate(names):
            tot[k] += evs[i].elapsed_time(evs[i + 1])
c = e.counters()
print(json.dumps({"games": games, "leaves_per_step": leaves, "warm_steps": warm,
                  "graph_ms_per_step": round(graph_ms, 4),
                  "eager_phase_us": {k: round(v / n * 1e3, 1) for k, v in tot.items()},
                  "counters": c}), flush=True)
