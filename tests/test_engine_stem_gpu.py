"""The net's stem inside the select launch (az_engine_set_stem, BatchedSelfPlay's default
for nets whose trunk starts from a stored fp16x2 stem): the wave that packs a row of
player*state planes (reference Models.py:16, MCTS_model.py:15-28 with D4) also runs the
stem on it (Models.py:179-180, :209: conv0 + bn0 folded + relu) into the trunk's first
activation buffer and its per-board range.  Bit-identical to the stem kernel on the packed
planes (az_conv_stem2_gpu, same fmaf chain and tap order), so the evaluation, and every
game, is unchanged.

* Kernel level: after each select of a live engine (active, idle and finished slots, D4
  transforms, K leaves per slot with empty rows, deferred moves on and off, 64 and 128
  channels) y and absmax equal the stem kernel's on nn_in, bit for bit.
* Net level: FusedInferenceNet.evaluate_into(stem_done=True) after such a select gives the
  priors / values of the plain evaluation of nn_in, bit for bit.
* Self-play: BatchedSelfPlay with and without it plays identical games through its graphs.
"""
import numpy as np
import pytest
import torch

from mock_policy import mock_eval_torch

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from engine import BatchedSelfPlay, Engine  # noqa: E402
from Models import AlphaZeroNet  # noqa: E402

ARGS = {"c_puct": 2.0, "num_simulations": 6, "dirichlet_alpha": 1.0,
        "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
        "lambda": 0.98}


def _stem_ref(planes, w9, bias):
    B, C = planes.shape[0], bias.numel()
    y = torch.empty((B, C, 8, 8), dtype=torch.float32, device=planes.device,
                    memory_format=torch.channels_last)
    amax = torch.empty(B, dtype=torch.float32, device=planes.device)
    nat.check(nat.lib.az_conv_stem2_gpu(nat.ptr(planes), nat.ptr(w9), nat.ptr(bias), nat.ptr(y),
                                        B, C, nat.ptr(amax), nat.stream_ptr()), "stem")
    return y, amax


@pytest.mark.parametrize("C,d4,K,defer", [(128, False, 1, True), (128, True, 1, False),
                                          (128, True, 4, True), (64, True, 2, False)])
def test_select_stem_matches_stem_kernel(C, d4, K, defer):
    G = 300  # not a multiple of the 4-slot workgroup
    torch.manual_seed(C + K)
    w9 = (torch.randn(9, C) * 0.7).cuda()
    bias = (torch.randn(C) * 0.3).cuda()  # some channels negative: ReLU zeros
    e = Engine(G, 6, c_puct=2.0, dirichlet_alpha=1.0, dirichlet_epsilon=0.3,
               num_exploratory_moves=35, lambd=0.98, d4_augment=d4, auto_play=True,
               refill=True, seed=11, leaves_per_step=K, sample_capacity=G * 200)
    R = G * K
    y = torch.full((R, C, 8, 8), float("nan"), device="cuda").contiguous(
        memory_format=torch.channels_last)
    amax = torch.full((R,), float("nan"), device="cuda")
    e.set_stem(w9, bias, y, amax)
    if defer:
        e.defer_moves(True)
    e.reset_all(start_budget=G * 3 // 2, stagger_steps=20)  # late starters stay idle a while
    par = 0
    with torch.no_grad():
        for step in range(520):
            if defer:
                e.select_move(par)
            else:
                e.select()
            if step % 13 == 0 or step < 3:
                yr, ar = _stem_ref(e.nn_in, w9, bias)
                assert torch.equal(y, yr), step
                assert torch.equal(amax, ar), step
            pr, va = mock_eval_torch(e.nn_in)
            e.priors.copy_(pr)
            e.values.copy_(va)
            if defer:
                e.expand_par(par)
                par ^= 1
            else:
                e.expand()
                e.play()
    if defer:
        e.move_flush(par ^ 1)
    c = e.counters()
    assert c["moves"] > 0 and c["games_finished"] > 0
    e.set_stem(None, None, None)  # off again: select leaves the buffers alone
    y.fill_(-1.0)
    e.select_move(par) if defer else e.select()
    torch.cuda.synchronize()
    assert (y == -1.0).all()
    e.close()


def _net():
    torch.manual_seed(0)
    return AlphaZeroNet(8, 65, 5, 128)


def test_evaluate_into_with_engine_stem_is_bit_identical(monkeypatch):
    """The stem in the select launch (engine stem), the stem kernel and the stem inside the
    persistent trunk (az_trunk_wino4_gpu with planes) give the same priors and values."""
    from Models import FusedInferenceNet

    monkeypatch.setattr(FusedInferenceNet, "trunk_stem", False)  # the engine stem on
    sp = BatchedSelfPlay(_net(), ARGS, 512, seed=3, use_graph=False, d4_augment=True)
    assert sp.engine_stem and sp.net.precision == "fp16x2"
    sp.reset(start_budget=-1, stagger_steps=30)
    sp.step(40)
    e = sp.engine
    with torch.no_grad():
        e.select_move(sp._par)
        p1 = torch.empty_like(e.priors)
        v1 = torch.empty_like(e.values)
        sp.net.evaluate_into(e.nn_in, p1, v1, stem_done=True)
        p0 = torch.empty_like(e.priors)
        v0 = torch.empty_like(e.values)
        sp.net.evaluate_into(e.nn_in.clone(), p0, v0)
        monkeypatch.setattr(FusedInferenceNet, "trunk_stem", True)
        p2 = torch.empty_like(e.priors)
        v2 = torch.empty_like(e.values)
        sp.net.evaluate_into(e.nn_in.clone(), p2, v2)
    torch.cuda.synchronize()
    assert torch.equal(p0, p1) and torch.equal(v0, v1)
    assert torch.equal(p0, p2) and torch.equal(v0, v2)
    assert torch.isfinite(p1).all() and torch.isfinite(v1).all()


@pytest.mark.parametrize("trunk_stem", [False, True])
def test_selfplay_with_and_without_engine_stem_same_games(trunk_stem, monkeypatch):
    """Self-play with the stem in the select launch against the stem elsewhere (its own
    kernel, or -- trunk_stem -- inside the persistent trunk launch): the same games."""
    from Models import FusedInferenceNet

    runs = []
    for on in (True, False):
        monkeypatch.setattr(FusedInferenceNet, "trunk_stem", trunk_stem and not on)
        sp = BatchedSelfPlay(_net(), ARGS, 512, seed=8, engine_stem=on, require_graph=True,
                             sample_capacity=512 * 200)
        assert sp.engine_stem == on
        sp.reset(start_budget=-1, stagger_steps=60)
        sp.step(720)
        c = sp.engine.counters()
        s = sp.engine.samples()
        order = np.argsort(s["slot"], kind="stable")
        runs.append((c, {k: v[order] for k, v in s.items()}, sp.engine.game_info()))
    (c1, s1, g1), (c0, s0, g0) = runs
    assert c1 == c0 and c1["moves"] > 0 and c1["games_finished"] > 0
    for k in s0:
        assert np.array_equal(s1[k], s0[k]), k
    for k in g0:
        assert np.array_equal(g1[k], g0[k]), k
