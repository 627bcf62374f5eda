"""Statistical pin of the device rollout (engine.hip rollout(), AZ_EVAL_ROLLOUT) against the
reference's own MCTS._rollout (MCTS_model.py:276-303).

The reference draws np.random.choice over the legal actions; the device draws from a Philox
stream, so only the outcome distribution can match.  tests/golden/rollout_stats.npz holds
the reference's win / draw / loss counts (from the side to move's view) at 8 positions of a
seeded random playout; here 4,096 device rollouts per position (one per game slot: the root
expansion of a 1-simulation search evaluates the root by one rollout and backs its value up,
so root W/N is that outcome) are compared category by category with a two-proportion z test.
The device stream is seeded, so the test is deterministic; |z| <= 4.5 rejects any real
difference of a few percent at these sample sizes."""
import math

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from engine import Engine  # noqa: E402

G = 4096


def device_outcomes(own, opp, player, seed):
    e = Engine(G, 1, rollout=True, auto_play=False, seed=seed)
    e.set_roots(np.arange(G), np.full(G, own, np.uint64), np.full(G, opp, np.uint64),
                np.full(G, player, np.int32))
    e.begin_search_slots(np.arange(G), 1)
    e.select()
    e.expand(e.priors, e.values)
    counts, vroot = e.root_stats()
    e.close()
    return vroot


def test_device_rollout_matches_reference_distribution():
    d = load_golden("rollout_stats.npz")
    for i in range(len(d["ply"])):
        player = int(d["player"][i])
        pos, neg = int(d["pos"][i]), int(d["neg"][i])
        own, opp = (pos, neg) if player == 1 else (neg, pos)
        v = device_outcomes(own, opp, player, seed=1000 + i)
        assert set(np.unique(v)) <= {-1.0, 0.0, 1.0}
        n_ref = int(d["n"][i])
        for name, val in (("wins", 1.0), ("draws", 0.0), ("losses", -1.0)):
            p_ref = int(d[name][i]) / n_ref
            p_dev = float((v == val).mean())
            p = (int(d[name][i]) + (v == val).sum()) / (n_ref + G)
            se = math.sqrt(max(p * (1 - p), 1e-12) * (1.0 / n_ref + 1.0 / G))
            z = (p_dev - p_ref) / se
            assert abs(z) <= 4.5, (int(d["ply"][i]), name, p_dev, p_ref, z)
