"""Deep self-play goldens for the benchmarked path, made by running the REFERENCE itself.
Build container only (imports /root/reference read-only); writes
tests/golden/selfplay_deep.npz.

selfplay_games.npz (make_goldens.py) holds one 400-simulation game; the bench plays 400
simulations per move, where trees are deep enough to reach the engine's arena compaction of
large subtrees, the K = 1 descent level budget stopping a launch mid-search and the descent
cap.  This file adds complete reference games at the bench's settings:

  K = 1   reference one_self_play (self_play_worker.py:38-88) with args['num_threads'] = 1
          (deterministic), 400 simulations, three seeds;
  K = 4   the same one_self_play with num_threads = 4, its thread pool replaced by the forced
          schedule of make_vl_goldens.py (controlled_simulations: at most K simulations
          blocked in policy.inference, released in start order) -- the interleaving the
          engine's leaves_per_step = 4 implements; 100 and 400 simulations.

The MCTS, Node, env, get_training_data and RNG calls are the reference's own; only the pool
that schedules `_simulate` and the gate inside the mock policy are test scaffolding.  Layout
as selfplay_games.npz plus meta[:, 3] = K:

    python tests/golden/make_deep_goldens.py
"""
import os
import sys
import time

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_goldens import RngRecorder, bb_from_state, encode_log  # noqa: E402
from make_vl_goldens import GatedPolicy, controlled_simulations  # noqa: E402
from mock_policy import MockPolicyNet  # noqa: E402


class _Done:
    def result(self):
        return None


class ControlledPool:
    """Stands in for MCTS.pool (MCTS_model.py:196-197): policy_improve_step submits its
    `num_simulations` _simulate calls (:237-242), and they run under the forced schedule
    when the first result is awaited."""

    def __init__(self, m, K):
        self.m, self.K, self.queued = m, K, 0

    def submit(self, fn, root):
        assert fn == self.m._simulate and root is self.m.root
        self.queued += 1
        pool = self

        class _Fut:
            def result(self_inner):
                if pool.queued:
                    n, pool.queued = pool.queued, 0
                    controlled_simulations(pool.m, pool.m.policy, n, pool.K)
                return None

        return _Fut()

    def shutdown(self, *a, **k):
        return None


class GatedPolicyNet(GatedPolicy):
    """The gated mock constructible the way one_self_play builds its net
    (self_play_worker.py:43-46)."""

    def __init__(self, **cfg):
        super().__init__()

    def load_state_dict(self, sd):
        return None

    def eval(self):
        return self


def play(sims, K, seed):
    import self_play_worker
    from MCTS_model import MCTS

    args = {"c_puct": 2.0, "num_simulations": sims, "num_threads": K,
            "dirichlet_alpha": 1.0, "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0,
            "num_exploratory_moves": 35, "lambda": 0.98}
    policy_cls = MockPolicyNet
    orig = self_play_worker.MCTS
    if K > 1:
        class ControlledMCTS(MCTS):
            def __init__(self, *a, **kw):
                super().__init__(*a, **kw)
                self.pool.shutdown()
                self.pool = ControlledPool(self, K)

        self_play_worker.MCTS = ControlledMCTS
        policy_cls = GatedPolicyNet
    try:
        np.random.seed(seed)
        with RngRecorder() as rec:
            out = self_play_worker.one_self_play((8, args, (policy_cls, {}, {}), None))
    finally:
        self_play_worker.MCTS = orig
    return out, rec.log


def main():
    games = [(400, 1, 7), (400, 1, 8), (400, 1, 9), (100, 4, 21), (100, 4, 22), (400, 4, 23)]
    rows = dict(game=[], ply=[], pos=[], neg=[], pi=[], z=[])
    meta, logs, noises = [], [], []
    for gi, (sims, K, seed) in enumerate(games):
        t0 = time.time()
        out, log = play(sims, K, seed)
        print(f"  game {gi}: sims={sims} K={K} plies={len(out)} {time.time() - t0:.1f}s",
              flush=True)
        for t, (s, pi, z) in enumerate(out):
            p, n = bb_from_state(s)  # canonical (state*player): +1 = side to move
            rows["game"].append(gi)
            rows["ply"].append(t)
            rows["pos"].append(p)
            rows["neg"].append(n)
            rows["pi"].append(np.asarray(pi, np.float32))
            rows["z"].append(float(z))
        k, fa, ib, nz = encode_log(log)
        logs.append((k, fa, ib))
        noises.append(nz)
        meta.append((sims, seed, len(out), K))
    out = {"pos": np.array(rows["pos"], np.uint64), "neg": np.array(rows["neg"], np.uint64),
           "game": np.array(rows["game"], np.int32), "ply": np.array(rows["ply"], np.int32),
           "pi": np.array(rows["pi"], np.float32), "z": np.array(rows["z"], np.float64),
           "meta": np.array(meta, np.int64)}
    offs = [0]
    for k, _, _ in logs:
        offs.append(offs[-1] + len(k))
    out["log_offsets"] = np.array(offs, np.int64)
    out["log_kind"] = np.concatenate([l[0] for l in logs])
    out["log_a"] = np.concatenate([l[1] for l in logs])
    out["log_b"] = np.concatenate([l[2] for l in logs])
    noffs = [0]
    for nz in noises:
        noffs.append(noffs[-1] + len(nz))
    out["noise_offsets"] = np.array(noffs, np.int64)
    out["noise"] = np.concatenate(noises)
    np.savez_compressed(os.path.join(HERE, "selfplay_deep.npz"), **out)
    print("selfplay_deep:", len(games), "games,", len(out["pos"]), "samples")


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"{time.time() - t0:.1f}s")
