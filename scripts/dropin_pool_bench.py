"""Aggregate games/s of the UNCHANGED trainer path: train.py's collect_self_play_games
(train.py:199-225) runs `one_self_play` in a spawn Pool of `num_workers` processes; with this
repo's drop-ins on the path every worker plays its games through the drop-in `MCTS` on the
GPU engine (its own HIP context, one game at a time, the fused HIP net).  Small per-game
kernels from several workers run side by side on the GPU's CUs, so the pool scales with the
worker count until the card is shared out.

    python scripts/dropin_pool_bench.py [workers] [games] [sims] [cold] > out.json

cold: no warm-up -- the timed region is train.py's whole `with Pool(...)` block (worker start,
imports, the HIP context and graph capture of whichever worker plays) as one generation of
train.py pays it.

Each worker plays one short warm-up game in its initializer (HIP context, kernels, graph
capture), then the timed batch of `games` games is streamed through imap_unordered with
chunksize 1, as the reference does.  The reference's own args: no num_threads (4 workers
-> 4 virtual-loss leaves per engine step)."""
import json
import os
import sys
import time
from multiprocessing import get_context

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "alphazero-othello_amd")


def _init():
    sys.path[:0] = [ROOT, PKG]
    import torch

    import self_play_worker
    from Models import AlphaZeroNet

    torch.manual_seed(0)
    net = AlphaZeroNet(8, 65, 5, 128).eval()
    ps = (AlphaZeroNet, {"board_size": 8, "action_size": 65, "n_res_blocks": 5,
                         "channels": 128}, net.state_dict())
    args = {"c_puct": 2.0, "num_simulations": 8, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    self_play_worker.one_self_play((8, args, ps, None))
    torch.cuda.synchronize()


def _play(item):
    import self_play_worker

    return len(self_play_worker.one_self_play(item))


def main():
    workers = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    games = int(sys.argv[2]) if len(sys.argv) > 2 else 2 * workers
    sims = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    sys.path[:0] = [ROOT, PKG]
    import torch

    from Models import AlphaZeroNet

    torch.manual_seed(0)
    net = AlphaZeroNet(8, 65, 5, 128).eval()
    ps = (AlphaZeroNet, {"board_size": 8, "action_size": 65, "n_res_blocks": 5,
                         "channels": 128}, net.state_dict())
    # train.py hands every task its whole args dict, num_self_play / num_workers included
    # (train.py:207-217, 413-420); one_self_play sizes its per-worker batch from them
    args = {"c_puct": 2.0, "num_simulations": sims, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98, "num_self_play": games, "num_workers": workers}
    cold = len(sys.argv) > 4 and sys.argv[4] == "cold"
    ctx = get_context("spawn")
    if cold:
        t0 = time.perf_counter()
        with ctx.Pool(workers) as pool:
            lens = list(pool.imap_unordered(_play, [(8, args, ps, None)] * games, chunksize=1))
        dt = time.perf_counter() - t0
    else:
        with ctx.Pool(workers, initializer=_init) as pool:
            # warm-up tasks (8 sims, without num_self_play: each worker's own batch)
            warm = {k: v for k, v in args.items() if k != "num_self_play"}
            pool.map(_play, [(8, dict(warm, num_simulations=8), ps, None)] * workers)
            t0 = time.perf_counter()
            lens = list(pool.imap_unordered(_play, [(8, args, ps, None)] * games, chunksize=1))
            dt = time.perf_counter() - t0
    plies = sum(lens)
    print(json.dumps({"workers": workers, "games": games, "sims": sims,
                      "games_per_s": round(games / dt, 4), "plies": plies,
                      "mean_plies_returned": round(plies / games, 2),
                      "batch_per_worker": min(int(os.environ.get("AZ_DROPIN_BATCH", "32")),
                                              -(-games // workers)),
                      "window_s": round(dt, 2),
                      "net": "AlphaZeroNet(5,128) random init, fused HIP inference copy",
                      "path": "train.py Pool -> one_self_play (AZ_DROPIN_BATCH games per worker "
                              "batch on the batched engine; 1 = one game per call through the "
                              "drop-in MCTS), 4 leaves/step",
                      "dropin_batch": int(os.environ.get("AZ_DROPIN_BATCH", "32")),
                      "shared_generation": os.environ.get("AZ_DROPIN_SHARED", "1") == "1",
                      "timed": "the whole Pool block (cold)" if cold else
                               "imap_unordered over warm workers"}))


if __name__ == "__main__":
    main()
