"""Steady-state per-phase step times: after `warm` graph-replayed steps, 200 eager steps
timed phase by phase with HIP events (select / net / expand / move), plus the sustained
ms/step of graph replay in blocks."""
import json, os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "alphazero-othello_amd"))
from engine import BatchedSelfPlay  # noqa: E402
from Models import AlphaZeroNet  # noqa: E402
import bench  # noqa: E402

warm = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
torch.manual_seed(0)
sp = BatchedSelfPlay(AlphaZeroNet(8, 65, 5, 128), bench.SELFPLAY_ARGS, 1024, seed=1)
sp.reset(-1, 401 * 60)
blocks = []
done = 0
while done < warm:
    t0 = time.perf_counter()
    sp.step(2000)
    torch.cuda.synchronize()
    blocks.append(round((time.perf_counter() - t0) / 2, 3))
    done += 2000
e = sp.engine
names = ["select", "net", "expand", "move"]
tot = {k: 0.0 for k in names}
evs = [torch.cuda.Event(True) for _ in range(5)]
with torch.no_grad():
    for _ in range(200):
        evs[0].record(); e.select(); evs[1].record()
        pr, va = sp.net.evaluate_planes(e.nn_in); e.priors.copy_(pr); e.values.copy_(va); evs[2].record()
        e.expand(); evs[3].record(); e.play(); evs[4].record()
        torch.cuda.synchronize()
        for i, k in enumerate(names):
            tot[k] += evs[i].elapsed_time(evs[i + 1])
print(json.dumps({"ms_per_step_by_2000_block": blocks,
                  "steady_phase_ms": {k: round(v / 200, 4) for k, v in tot.items()},
                  "counters": e.counters()}), flush=True)
