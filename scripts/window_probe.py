"""Where does a short timed window lose time?  bench.py's configs[2] engine (1 or 2 pipelines),
the same steady-state warmup, then a series of timed windows of various lengths, each timed
exactly as bench.py times its window (synchronize, t0, step(n), counters(), synchronize) and,
beside that, with HIP events recorded on every pipeline stream after every graph replay, so
the per-chunk GPU timeline of the window is visible.
    python scripts/window_probe.py <pipelines> [window lengths ...]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import bench  # noqa: E402
from engine import BatchedSelfPlay, PipelinedSelfPlay  # noqa: E402


def build(P, games_per_pipe=1024, spg=8):
    net = bench.make_net("az5x128")
    args = dict(bench.SELFPLAY_ARGS, num_simulations=400)
    G = games_per_pipe * P
    kw = dict(seed=1234, stream_id=0, use_graph=True, require_graph=True,
              device=torch.device("cuda", 0), sample_capacity=games_per_pipe * 130 * 4,
              steps_per_graph=spg, precision="fp16x2")
    sp = PipelinedSelfPlay(net, args, G, pipelines=P, **kw) if P > 1 else \
        BatchedSelfPlay(net, args, G, **kw)
    stagger = 401 * 60
    sp.reset(start_budget=-1, stagger_steps=stagger)
    return sp, stagger


def window(sp, n, events=True):
    """bench.py's window; with events, the step loop is PipelinedSelfPlay.step's with an
    event after every replay on its stream."""
    parts = sp.parts if isinstance(sp, PipelinedSelfPlay) else [sp]
    streams = sp.streams if isinstance(sp, PipelinedSelfPlay) else [torch.cuda.current_stream()]
    torch.cuda.synchronize()
    c0 = sp.counters()
    cur = torch.cuda.current_stream()
    e0 = torch.cuda.Event(enable_timing=True)
    marks = [[] for _ in parts]
    host = []
    t0 = time.perf_counter()
    e0.record(cur)
    if not events:
        sp.step(n)
    else:
        with torch.no_grad():
            for s in streams:
                s.wait_stream(cur)
            k = max(p.steps_per_graph for p in parts)
            left = n
            while left > 0:
                m = min(k, left)
                for i, (p, s) in enumerate(zip(parts, streams)):
                    with torch.cuda.stream(s):
                        p._advance(m)
                        ev = torch.cuda.Event(enable_timing=True)
                        ev.record(s)
                        marks[i].append((f"adv{m}", ev))
                    host.append(round((time.perf_counter() - t0) * 1e3, 3))
                left -= m
            for i, (p, s) in enumerate(zip(parts, streams)):
                with torch.cuda.stream(s):
                    p._flush()
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record(s)
                    marks[i].append(("flush", ev))
            for s in streams:
                cur.wait_stream(s)
    th = (time.perf_counter() - t0) * 1e3
    c1 = sp.counters()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    sims = c1["simulations"] - c0["simulations"]
    out = {"n": n, "ms_per_step": round(dt * 1e3 / n, 4), "window_ms": round(dt * 1e3, 3),
           "host_enqueue_ms": round(th, 3), "sims": sims,
           "sims_per_step": round(sims / n, 1)}
    if events:
        out["host_ms_after_each"] = host
        out["gpu_ms"] = [[(nm, round(e0.elapsed_time(ev), 3)) for nm, ev in mk] for mk in marks]
    return out


def main():
    P = int(sys.argv[1])
    ns = [int(x) for x in sys.argv[2:]] or [20, 20, 20, 8000, 20, 20, 16, 24, 40]
    spg = int(os.environ.get("PROBE_SPG", "8"))
    sp, stagger = build(P, spg=spg)
    if os.environ.get("PROBE_KB") == "1":  # bench.py's kernel roofline first, as bench.py runs it
        kb = bench.StepKernelBench(1 << 24, torch.device("cuda", 0))
        print(json.dumps({"k_step_ms": round(kb.time_ms(), 4), "io_ms": round(kb.time_io_ms(), 4)}),
              flush=True)
    t = time.perf_counter()
    sp.step(stagger)
    torch.cuda.synchronize()
    print(json.dumps({"pipelines": P, "spg": spg, "warmup_steps": stagger,
                      "warmup_ms_per_step": round((time.perf_counter() - t) * 1e3 / stagger, 4)}),
          flush=True)
    for n in ns:
        print(json.dumps(dict(window(sp, n, events=n <= 64), pipelines=P, spg=spg)), flush=True)
    # bench.py's own window without the events
    for n in (20, 20):
        print(json.dumps(dict(window(sp, n, events=False), pipelines=P, spg=spg, plain=True)),
              flush=True)


if __name__ == "__main__":
    main()
