"""Statistical pin of the Othello rollout evaluation: outcome distributions of the
REFERENCE's own MCTS._rollout (MCTS_model.py:276-303) from fixed positions.  Build
container only (imports /root/reference read-only); writes tests/golden/rollout_stats.npz.

The reference draws np.random.choice over the legal actions, so the device rollout (a
Philox stream, engine.hip rollout()) can match it only in distribution: the GPU test
(tests/test_rollout_gpu.py) compares win / draw / loss frequencies from the same positions.

Positions: the board corpus's game 1 (a seeded random playout, board_corpus.npz) at the
plies below, each with its side to move; `n` rollouts per position, np.random.seed(ply).

    python tests/golden/make_rollout_goldens.py
"""
import os
import sys

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)

PLIES = [(24, 600), (32, 800), (40, 1500), (44, 2000), (48, 2000), (52, 3000), (55, 3000),
         (57, 3000)]


def main():
    from envs.othello import OthelloGameNew
    from MCTS_model import MCTS

    d = np.load(os.path.join(HERE, "board_corpus.npz"))
    sel = np.nonzero(d["game"] == 1)[0]
    env = OthelloGameNew(8)
    m = MCTS(env, {"c_puct": 2.0, "num_simulations": 1, "num_threads": 1}, None)
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    rows = []
    for ply, n in PLIES:
        i = sel[min(ply, len(sel) - 1)]
        pos, neg, player = int(d["pos"][i]), int(d["neg"][i]), int(d["player"][i])
        state = (((np.uint64(pos) & w) != 0).astype(np.int8)
                 - ((np.uint64(neg) & w) != 0).astype(np.int8)).reshape(8, 8)
        np.random.seed(ply)
        out = np.array([m._rollout(state, player) for _ in range(n)])
        counts = [int((out == v).sum()) for v in (1, 0, -1)]
        rows.append((pos, neg, player, ply, n, *counts))
        print(f"ply {ply}: player {player} win/draw/loss {counts} of {n}", flush=True)
    r = np.array(rows, dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "rollout_stats.npz"),
                        pos=r[:, 0].astype(np.uint64), neg=r[:, 1].astype(np.uint64),
                        player=r[:, 2], ply=r[:, 3], n=r[:, 4], wins=r[:, 5], draws=r[:, 6],
                        losses=r[:, 7])


if __name__ == "__main__":
    main()
