"""How many of the leaf batch's rows carry a leaf at steady state (configs[2] bench schedule):
rows whose slot sat the step out (its search finished, or every descent of the launch ended
on a terminal node) are evaluated by the net all the same.  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import bench  # noqa: E402
from engine import BatchedSelfPlay  # noqa: E402

G, S = 1024, 400
net = bench.make_net("az5x128")
sp = BatchedSelfPlay(net, dict(bench.SELFPLAY_ARGS, num_simulations=S), G, seed=1234,
                     sample_capacity=G * 130 * 4)
stagger = (S + 1) * 60
sp.reset(start_budget=-1, stagger_steps=stagger)
sp.step(stagger)
live = []
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2000):
    sp.step(1)
    live.append(int((sp.engine.leaf >= 0).sum().item()))
live = np.array(live)
print(json.dumps({"slots": G, "steps": len(live), "mean_live_rows": float(live.mean()),
                  "frac_live": float(live.mean() / G), "min": int(live.min()),
                  "p10": float(np.percentile(live, 10)), "max": int(live.max())}))
