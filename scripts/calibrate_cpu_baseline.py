"""Calibrate bench.py's CPU baseline (the oracle's port of one_self_play) against the
reference itself -- BUILD CONTAINER ONLY (imports /root/reference, which never travels).

Both run on the same host cores with the same configuration: 8 single-threaded worker
processes (the reference's spawn pool, train.py:199-225, one self_play_worker.one_self_play
per task; the port: bench.py --cpu-worker in full-game mode), `--games` complete games per
worker, AlphaZeroNet(8, 65, 5, 128) seed-0 random init, 400 sims, c_puct 2, Dirichlet
alpha 1 / eps 0.3, temperature 1 for 35 plies, lambda 0.98, the reference's default
num_threads=4.  Writes profiles/cpu_calibration.json with both games/s and
ratio_reference_over_port; bench.py scales its sampled port rate by that ratio.

    python scripts/calibrate_cpu_baseline.py [--workers 8] [--games 1]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def _ref_worker_init(seed):
    import sys as _s

    if REF not in _s.path:
        _s.path.insert(0, REF)
    import random

    import numpy as np
    import torch

    pid = os.getpid()
    np.random.seed(seed + pid)
    random.seed(seed + pid)
    torch.manual_seed(seed + pid)
    torch.set_num_threads(1)


def reference_pool(workers, games, sims):
    """The reference's own one_self_play in a spawn pool (train.py:202-223)."""
    sys.path.insert(0, REF)
    from multiprocessing import get_context

    import torch
    from Models import AlphaZeroNet
    from self_play_worker import one_self_play

    torch.manual_seed(0)
    net = AlphaZeroNet(8, 65, 5, 128)
    args = {"c_puct": 2.0, "num_simulations": sims, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    policy = (net.__class__, net.get_config(), net.state_dict())
    items = [(8, args, policy, None) for _ in range(workers * games)]
    ctx = get_context("spawn")
    with ctx.Pool(workers, initializer=_ref_worker_init, initargs=(0,)) as pool:
        t0 = time.perf_counter()
        n = 0
        plies = 0
        for traj in pool.imap_unordered(one_self_play, items, chunksize=1):
            n += 1
            plies += len(traj)
        dt = time.perf_counter() - t0
    return {"games": n, "seconds": dt, "games_per_s": n / dt, "plies_per_game": plies / n}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--games", type=int, default=1)
    ap.add_argument("--sims", type=int, default=400)
    ap.add_argument("--ref-only", action="store_true")
    a = ap.parse_args()
    if a.ref_only:
        print(json.dumps(reference_pool(a.workers, a.games, a.sims)), flush=True)
        return
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", OMP_NUM_THREADS="1")
    out = subprocess.check_output([sys.executable, os.path.abspath(__file__), "--ref-only",
                                   "--workers", str(a.workers), "--games", str(a.games),
                                   "--sims", str(a.sims)], env=env, cwd="/tmp")
    ref = json.loads(out.decode().strip().splitlines()[-1])
    sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
    import bench

    t0 = time.perf_counter()
    outs = bench._cpu_pool("az5x128", a.sims, 0, a.workers, full_games=a.games)
    dt = time.perf_counter() - t0
    port = {"games": sum(o["games"] for o in outs), "seconds": dt,
            "games_per_s": sum(o["games"] for o in outs) / dt,
            "per_worker_games_per_s": [round(o["games_per_s"], 5) for o in outs]}
    res = {"net": "az5x128", "sims": a.sims, "workers": a.workers,
           "games_per_worker": a.games, "cpu_model": bench.cpu_model(),
           "os_cpu_count": os.cpu_count(), "reference": ref, "port": port,
           "ratio_reference_over_port": ref["games_per_s"] / port["games_per_s"],
           "how": "scripts/calibrate_cpu_baseline.py in the build container: the reference's "
                  "one_self_play in a spawn pool vs bench.py's port in full-game mode, same "
                  "cores, same config, one after the other"}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
