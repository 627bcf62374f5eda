"""Statistical pin of the Othello rollout evaluation: outcome distributions of the
REFERENCE's own MCTS._rollout (MCTS_model.py:276-303) from fixed positions.  Build
container only (imports /root/reference read-only); writes tests/golden/rollout_stats.npz.

The reference draws np.random.choice over the legal actions, so the device rollout (a
Philox stream, engine.hip rollout()) can match it only in distribution: the GPU test
(tests/test_rollout_gpu.py) compares win / draw / loss frequencies from the same positions.

Positions: 8 positions of the board corpus's seeded random playouts (board_corpus.npz) at
plies 12..52 whose outcome under random play is uncertain (win rate of the side to move
between 0.25 and 0.75 in a quick pre-screen on the repo's own CPU step, used only to pick
the positions), so the test has power on every outcome; `n` rollouts each,
np.random.seed(ply).

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

TARGET_PLIES = [12, 18, 24, 30, 36, 42, 48, 52]
N_REF = 1500


def prescreen(pos, neg, player, n=256, seed=0):
    """Win rate of the side to move under uniform random play (the repo's CPU board step,
    vectorised over n playouts) -- only to choose balanced positions."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "alphazero-othello_amd"))
    import az_native as nat

    rng = np.random.default_rng(seed)
    own = np.full(n, pos if player == 1 else neg, np.uint64)
    opp = np.full(n, neg if player == 1 else pos, np.uint64)
    side = np.ones(n, np.int64)  # +1 while the original player is to move
    res = np.full(n, 2, np.int64)
    bitv = np.uint64(1) << np.arange(64, dtype=np.uint64)
    for _ in range(70):
        live = res == 2
        if not live.any():
            break
        lg = nat.legal_cpu(own, opp)
        bits = (lg[:, None] & bitv[None, :]) != 0
        keys = np.where(bits, rng.random(bits.shape), -1.0)
        act = np.where(bits.any(1), keys.argmax(1), 64).astype(np.uint8)
        o, p, _, st = nat.step_cpu(own, opp, act)
        own, opp, side = np.where(live, o, own), np.where(live, p, opp), np.where(live, -side, side)
        term = live & ((st & 1) != 0)
        d = (np.vectorize(lambda x: bin(int(x)).count("1"))(own).astype(np.int64)
             - np.vectorize(lambda x: bin(int(x)).count("1"))(opp).astype(np.int64)) * side
        res = np.where(term, np.sign(d), res)
    return float((res == 1).mean())


def main():
    from envs.othello import OthelloGameNew
    from MCTS_model import MCTS

    d = np.load(os.path.join(HERE, "board_corpus.npz"))
    env = OthelloGameNew(8)
    m = MCTS(env, {"c_puct": 2.0, "num_simulations": 1, "num_threads": 1}, None)
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    rows = []
    games = np.unique(d["game"])
    for ply in TARGET_PLIES:
        for g in games[1:]:
            i = np.nonzero((d["game"] == g) & (d["ply"] == ply))[0]
            if len(i) == 0:
                continue
            i = i[0]
            pos, neg, player = int(d["pos"][i]), int(d["neg"][i]), int(d["player"][i])
            pw = prescreen(pos, neg, player, seed=ply)
            if 0.25 <= pw <= 0.75:
                break
        else:
            raise RuntimeError(f"no balanced position at ply {ply}")
        state = (((np.uint64(pos) & w) != 0).astype(np.int8)
                 - ((np.uint64(neg) & w) != 0).astype(np.int8)).reshape(8, 8)
        np.random.seed(ply)
        out = np.array([m._rollout(state, player) for _ in range(N_REF)])
        counts = [int((out == v).sum()) for v in (1, 0, -1)]
        rows.append((pos, neg, player, ply, N_REF, *counts))
        print(f"game {g} ply {ply}: player {player} prescreen {pw:.2f} win/draw/loss {counts} "
              f"of {N_REF}", flush=True)
    col = lambda k, dt: np.array([r[k] for r in rows], dtype=dt)  # noqa: E731
    np.savez_compressed(os.path.join(HERE, "rollout_stats.npz"),
                        pos=col(0, np.uint64), neg=col(1, np.uint64), player=col(2, np.int64),
                        ply=col(3, np.int64), n=col(4, np.int64), wins=col(5, np.int64),
                        draws=col(6, np.int64), losses=col(7, np.int64))


if __name__ == "__main__":
    main()
