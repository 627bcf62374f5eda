"""Experiment: configs[2]'s 1,024 games as P independent BatchedSelfPlay pipelines of 1,024 / P
slots, each replaying its own HIP graphs on its own stream, so one pipeline's select launch
(mostly idle chip: a few slow descents) runs beside another's trunk.  Steady state as in
bench.py (staggered slot starts, warmup of one game length), then a timed window; prints
simulations/s per configuration, interleaving the configurations twice.
    python scripts/split_pipeline.py [P ...]     (default: 1 2)"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import bench  # noqa: E402
from engine import BatchedSelfPlay  # noqa: E402

GAMES, SIMS, STEPS = 1024, 400, int(os.environ.get("SPLIT_STEPS", "6000"))


def build(p):
    net = bench.make_net("az5x128")
    args = dict(bench.SELFPLAY_ARGS, num_simulations=SIMS)
    sps = [BatchedSelfPlay(net, args, GAMES // p, seed=1234 + i, stream_id=i, require_graph=True,
                           sample_capacity=GAMES // p * 130 * 4) for i in range(p)]
    streams = [torch.cuda.Stream() for _ in range(p)]
    stagger = (SIMS + 1) * int(bench.REF_PLIES_PER_GAME)
    for sp in sps:
        sp.reset(start_budget=-1, stagger_steps=stagger)
        sp.step(2)  # capture (parity back to 0 after two single steps)
        if sp._par:
            sp.step(1)
    torch.cuda.synchronize()
    return sps, streams, stagger


def run(sps, streams, n):
    """n steps of every pipeline: multi-step graphs enqueued round-robin over the streams."""
    k = sps[0].steps_per_graph
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)
    for _ in range(n // k):
        for sp, s in zip(sps, streams):
            with torch.cuda.stream(s):
                sp.graph[(k, 0)].replay()
    for s in streams:
        cur.wait_stream(s)


def measure(p):
    sps, streams, stagger = build(p)
    k = sps[0].steps_per_graph
    run(sps, streams, (stagger // k + 1) * k)
    torch.cuda.synchronize()
    c0 = [sp.engine.counters() for sp in sps]
    t0 = time.perf_counter()
    run(sps, streams, STEPS // k * k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    c1 = [sp.engine.counters() for sp in sps]
    sims = sum(b["simulations"] - a["simulations"] for a, b in zip(c0, c1))
    moves = sum(b["moves"] - a["moves"] for a, b in zip(c0, c1))
    out = {"pipelines": p, "slots_each": GAMES // p, "steps": STEPS // k * k,
           "window_s": round(dt, 3), "us_per_step": round(dt / (STEPS // k * k) * 1e6, 2),
           "sims_per_s": round(sims / dt, 1), "moves_per_s": round(moves / dt, 1),
           "games_per_s_at_60_plies": round(sims / dt / SIMS / bench.REF_PLIES_PER_GAME, 3)}
    del sps
    torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    ps = [int(x) for x in sys.argv[1:]] or [1, 2]
    for rep in range(2):
        for p in ps:
            print(json.dumps(dict(measure(p), rep=rep)), flush=True)
