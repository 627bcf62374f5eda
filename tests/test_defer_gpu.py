"""Deferred moves (az_engine_defer_moves / az_select_move / az_expand_backup_par /
az_move_flush, and with the expansion fused too az_select_move_expand -- BatchedSelfPlay's
default): each step's move phase runs inside the next
step's select launch, beside its descents, instead of after expand.  A slot's games depend only on its own tree, policy and RNG stream -- never on
the step its moves land in -- so every slot must produce exactly the games (training rows)
of the plain move phase (az_play), bit for bit: reference self_play_worker.py:38-88 per
game."""
import numpy as np
import pytest
import torch

from mock_policy import MockNet, mock_eval_torch

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from engine import BatchedSelfPlay  # noqa: E402


def _run(defer, G, sims, steps, use_graph, leaves=1, fuse=True):
    args = {"c_puct": 2.0, "num_simulations": sims, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    sp = BatchedSelfPlay(MockNet(), args, G, seed=5, fold=False, use_graph=use_graph,
                         defer_moves=defer, sample_capacity=G * 400, leaves_per_step=leaves,
                         fuse_expand=fuse)
    assert sp.fuse_expand == (fuse and defer)
    sp.reset(start_budget=-1, stagger_steps=sims * 7)
    sp.step(steps)
    assert (sp.graph is not None) == use_graph and sp.graph_error is None
    c = sp.engine.counters()
    assert c["arena_overflows"] == 0 and c["samples_dropped"] == 0
    s = sp.engine.samples()
    order = np.argsort(s["slot"], kind="stable")  # a slot's games in the order they ended
    return c, {k: v[order] for k, v in s.items()}


@pytest.mark.parametrize("use_graph,leaves,fuse", [(True, 1, True), (False, 1, True),
                                                   (True, 4, True), (True, 1, False),
                                                   (True, 4, False)])
def test_deferred_moves_play_the_same_games(use_graph, leaves, fuse):
    """fuse: the expansion fused into the next step's select launch too
    (az_select_move_expand, BatchedSelfPlay's default)."""
    G, sims = 512, 12
    steps = 2600 if leaves == 1 else 900
    c0, a = _run(False, G, sims, steps, use_graph, leaves)
    c1, b = _run(True, G, sims, steps, use_graph, leaves, fuse)
    assert c0["games_finished"] >= G and c1["games_finished"] >= G
    compared = 0
    for g in range(G):
        ra, rb = np.flatnonzero(a["slot"] == g), np.flatnonzero(b["slot"] == g)
        n = min(len(ra), len(rb))  # the complete games both runs finished (a prefix)
        assert n >= 9, g
        for k in ("own", "opp", "pi", "z", "player"):
            assert np.array_equal(a[k][ra[:n]], b[k][rb[:n]]), (g, k)
        compared += n
    assert compared >= 9 * G


def test_mock_net_matches_mock_policy():
    x = torch.randint(-1, 2, (300, 64), device="cuda").float()
    p0, v0 = MockNet().cuda().evaluate_planes(x)
    p1, v1 = mock_eval_torch(x)
    assert torch.equal(p0, p1) and torch.equal(v0, v1)
