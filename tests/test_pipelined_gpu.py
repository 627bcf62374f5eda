"""engine.PipelinedSelfPlay (bench.py's default for configs[2]): G games as P independent
BatchedSelfPlay pipelines, each replaying its graphs on its own HIP stream.  Streams and the
round-robin enqueue change when launches run, never what they compute: every pipeline must
play exactly the games of a standalone BatchedSelfPlay of G / P slots with the same seed and
Philox stream (rows bit for bit), and play_games must deliver exactly the requested games."""
import numpy as np
import pytest
import torch

from mock_policy import MockNet

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from engine import BatchedSelfPlay, PipelinedSelfPlay  # noqa: E402

ARGS = {"c_puct": 2.0, "num_simulations": 12, "dirichlet_alpha": 1.0, "dirichlet_epsilon": 0.3,
        "mcts_temperature": 1.0, "num_exploratory_moves": 35, "lambda": 0.98}


def _sorted(s):
    order = np.lexsort((np.arange(len(s["slot"])), s["slot"]))  # by slot, in recorded order
    return {k: np.asarray(v)[order] for k, v in s.items()}


def _net(kind):
    if kind == "mock":
        return MockNet(), {"fold": False}
    from Models import AlphaZeroNet, FastOthelloNet

    torch.manual_seed(0)
    if kind == "fast":  # configs[1]'s net (bench --workload c2: 2 pipelines by default)
        return FastOthelloNet(8, 65), {}
    if kind == "c5":  # configs[4]: fused D4 symmetry + fp16 inference (2 pipelines by default)
        return AlphaZeroNet(8, 65, 5, 128), {"d4_augment": True, "dtype": torch.float16}
    return AlphaZeroNet(8, 65, 5, 128), {}  # fp16x2 persistent trunk + heads-fused conv


# G = 2,048: bench.py's configs[2] default shape (two 1,024-game pipelines, each evaluation a
# batch of 1,024 leaves on the persistent trunk, the two trunks on two streams)
@pytest.mark.parametrize("use_graph,kind,G", [(True, "mock", 512), (False, "mock", 512),
                                              (True, "az5x128", 512), (True, "fast", 512),
                                              (True, "c5", 512), (True, "az5x128", 2048)])
def test_pipelines_play_the_standalone_games(use_graph, kind, G):
    P, steps = 2, 1300
    net, extra = _net(kind)
    kw = dict(seed=5, use_graph=use_graph, sample_capacity=G * 400, **extra)
    pp = PipelinedSelfPlay(net, ARGS, G, pipelines=P, **kw)
    pp.reset(start_budget=-1, stagger_steps=12 * 7)
    c0 = pp.counters()
    pp.step(steps)
    c1 = pp.counters()
    assert c1["arena_overflows"] == 0 and c1["samples_dropped"] == 0
    assert c1["games_finished"] >= G // 2
    got = _sorted(pp.samples_since(c0))
    want = []
    for i in range(P):
        sp = BatchedSelfPlay(net, ARGS, G // P, stream_id=i, **kw)
        sp.reset(start_budget=-1, stagger_steps=12 * 7)
        sp.step(steps)
        assert sp.counters()["simulations"] == c1["per_part"][i]["simulations"]
        s = sp.engine.samples()
        s["slot"] = s["slot"] + i * (G // P)
        want.append(s)
    want = _sorted({k: np.concatenate([w[k] for w in want]) for k in want[0]})
    assert len(got["slot"]) == len(want["slot"]) > G
    for k in ("slot", "own", "opp", "pi", "z", "player"):
        assert np.array_equal(got[k], want[k]), k


def test_pipelined_play_games_delivers_every_game():
    pp = PipelinedSelfPlay(MockNet(), ARGS, 64, pipelines=2, seed=3, fold=False,
                           sample_capacity=64 * 400)
    rows = pp.play_games(21, check_every=64)
    c = pp.counters()
    assert c["games_finished"] == 21 and c["games_started"] == 21
    assert len(rows) == c["samples"]
    assert all(r[0].shape == (8, 8) and r[1].shape == (65,) for r in rows)
