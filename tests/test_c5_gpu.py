"""configs[4] as one workload: fused D4 symmetry per leaf + fp16 net inference inside
BatchedSelfPlay at the full per-GPU width (4,096 concurrent games), the path bench.py
--workload c5 runs (reference: MCTS_model.py:15-43, 313-318 for the symmetry; Models.py:9-31
for the inference).

* D4 parity at 4,096 slots: with a D4-EQUIVARIANT policy (the mock policy summed over the
  group: f(x) = 1/8 sum_s unsym_s(mock(sym_s(x))), on the reference's own index tables,
  tests/golden/d4.npz; every term is a multiple of 2^-10, so the sum is exact in any order),
  unsymmetrise(f(random_symmetry(b))) = f(b) for every draw, so the engine with fused D4
  must play exactly the games the engine without it plays -- every training row bit-exact,
  on the same injected Dirichlet / sampling streams.  (The prior-level check of the D4 map
  with a NON-equivariant policy is tests/test_engine_gpu.py.)
* The combined path with the real net: BatchedSelfPlay(AlphaZeroNet(5x128), d4_augment,
  fp16 inference copy) plays 4,096 complete games through its HIP graphs;
  check_complete holds and every sample row is a legal training tuple.
* Graph replay = eager execution, bit for bit, over 600 steps of the bench configuration at
  8 simulations per move with staggered starts (tree reuse, moves, game ends and restarts
  inside).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from mock_policy import mock_eval_torch

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from engine import BatchedSelfPlay, Engine, check_complete  # noqa: E402
from Models import AlphaZeroNet  # noqa: E402

G_FULL = 4096


class EquivariantMock:
    """The mock policy summed over D4 (exact, see the module docstring)."""

    def __init__(self, device):
        d4 = load_golden("d4.npz")
        self.board = torch.as_tensor(d4["sym_board"].astype(np.int64), device=device)
        self.unpi = torch.as_tensor(d4["sym_unpi"].astype(np.int64), device=device)

    def __call__(self, planes):
        P = torch.zeros(planes.shape[0], 65, dtype=torch.float64, device=planes.device)
        V = torch.zeros(planes.shape[0], dtype=torch.float64, device=planes.device)
        for s in range(8):
            p, v = mock_eval_torch(planes[:, self.board[s]])
            P += p.double()[:, self.unpi[s]]
            V += v.double()
        return (P / 8).float(), (V / 8).float()


def test_equivariant_mock_is_equivariant():
    f = EquivariantMock("cuda")
    corpus = load_golden("board_corpus.npz")
    rng = np.random.default_rng(5)
    idx = rng.choice(len(corpus["pos"]), 256, replace=False)
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    x = np.stack([((np.uint64(corpus["pos"][i]) & w) != 0).astype(np.float32)
                  - ((np.uint64(corpus["neg"][i]) & w) != 0).astype(np.float32) for i in idx])
    x = torch.as_tensor(x, device="cuda")
    p0, v0 = f(x)
    for t in range(8):
        pt, vt = f(x[:, f.board[t]])
        assert torch.equal(pt[:, f.unpi[t]], p0), t
        assert torch.equal(vt, v0), t


def _streams(G, NU, seed):
    rng = np.random.default_rng(seed)
    noise = rng.dirichlet(np.ones(65), size=(G, 1))
    return noise, rng.random((G, NU))


def _play(d4, evaluate, G, sims, noise, uni):
    e = Engine(G, sims, c_puct=2.0, dirichlet_alpha=1.0, dirichlet_epsilon=0.3,
               temperature=1.0, num_exploratory_moves=35, lambd=0.98, injected_rng=True,
               d4_augment=d4, auto_play=True, refill=False, inj_noise_slots=1,
               inj_uniform_slots=uni.shape[1], seed=77)
    e.reset_all(start_budget=G)
    e.inject(noise=noise, uniforms=uni)
    with torch.no_grad():
        for _ in range(200):
            for _ in range(100):
                e.select()
                pr, va = evaluate(e.nn_in)
                e.priors.copy_(pr)
                e.values.copy_(va)
                e.expand()
                e.play()
            if e.counters()["games_finished"] == G:
                break
    c = e.counters()
    check_complete(c, G)
    s = e.samples()
    order = np.lexsort((np.arange(len(s["slot"])), s["slot"]))  # by slot, ply order kept
    out = {k: v[order] for k, v in s.items()}
    e.close()
    return c, out


@pytest.mark.timeout(600)
def test_fused_d4_equivariant_policy_plays_the_plain_games_4096_slots():
    f = EquivariantMock("cuda")
    noise, uni = _streams(G_FULL, 256, seed=3)
    c_off, off = _play(False, f, G_FULL, 25, noise, uni)
    c_on, on = _play(True, f, G_FULL, 25, noise, uni)
    assert c_on["games_finished"] == c_off["games_finished"] == G_FULL
    assert c_on["samples"] == c_off["samples"] >= 9 * G_FULL
    for k in ("own", "opp", "pi", "z", "player", "slot"):
        assert np.array_equal(on[k], off[k]), k
    assert c_on["simulations"] == c_off["simulations"]


def _sample_rows_are_training_tuples(s):
    own, opp, pi, z = s["own"], s["opp"], s["pi"], s["z"]
    assert ((own & opp) == 0).all()
    assert np.isfinite(pi).all() and (pi >= 0).all()
    assert np.allclose(pi.sum(1), 1.0, atol=1e-5)
    assert (np.abs(z) <= 1.0).all()
    legal = nat.legal_cpu(own, opp)
    bits = ((legal[:, None] >> np.arange(64, dtype=np.uint64)[None, :]) & np.uint64(1)) != 0
    # pi is zero off the legal moves; the pass (64) only where no placement exists
    assert (pi[:, :64][~bits] == 0).all()
    assert (pi[legal != 0, 64] == 0).all()
    assert (pi[legal == 0, 64] == 1).all()


@pytest.mark.timeout(600)
def test_c5_selfplay_fp16_d4_4096_slots_complete_games():
    torch.manual_seed(0)
    net = AlphaZeroNet(8, 65, 5, 128)
    args = {"c_puct": 2.0, "num_simulations": 16, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    sp = BatchedSelfPlay(net, args, G_FULL, seed=9, d4_augment=True, dtype=torch.float16,
                         precision="fp16", sample_capacity=G_FULL * 130, require_graph=True)
    assert sp.net.precision == "fp16"
    tuples = sp.play_games(G_FULL)  # check_complete inside
    assert sp.graph is not None and sp.graph_error is None
    c = sp.engine.counters()
    assert c["games_finished"] >= G_FULL and c["arena_overflows"] == 0
    s = sp.engine.samples()
    assert len(tuples) == c["samples"] == len(s["z"])
    _sample_rows_are_training_tuples(s)
    # every game's first row is the initial position (black to move, canonical), which no
    # later position of a game can repeat
    init = (s["own"] == np.uint64(0x0000000810000000)) & (s["opp"] == np.uint64(0x0000001008000000))
    assert init.sum() == c["games_finished"]
    assert (np.bincount(s["slot"], minlength=G_FULL) >= 9).all()


@pytest.mark.timeout(600)
def test_c5_graph_replay_equals_eager_bit_exact():
    torch.manual_seed(0)
    net = AlphaZeroNet(8, 65, 5, 128)
    args = {"c_puct": 2.0, "num_simulations": 8, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    kw = dict(seed=21, d4_augment=True, dtype=torch.float16, precision="fp16",
              sample_capacity=G_FULL * 130)
    stagger = 9 * 60  # one game length, as bench.py staggers
    g = BatchedSelfPlay(net, args, G_FULL, use_graph=True, require_graph=True, **kw)
    g.reset(start_budget=-1, stagger_steps=stagger)
    g.step(600)  # 2 warm-up steps run eagerly at capture, then 600 replayed (75 x the 8-step graph)
    e = BatchedSelfPlay(net, args, G_FULL, use_graph=False, **kw)
    e.reset(start_budget=-1, stagger_steps=stagger)
    e.step(602)
    assert g.graph is not None
    cg, ce = g.engine.counters(), e.engine.counters()
    assert cg == ce and cg["moves"] > 0 and cg["games_finished"] > 0
    ng, vg = g.engine.root_stats()
    ne, ve = e.engine.root_stats()
    assert np.array_equal(ng, ne) and np.array_equal(vg, ve)
    ig, ie = g.engine.game_info(), e.engine.game_info()
    for k in ig:
        assert np.array_equal(ig[k], ie[k]), k
    if cg["samples"]:
        # games finishing in the same step reserve their rows in the order their workgroups
        # reach the sample counter; a slot's games reserve in time order, so the rows sorted
        # stably by slot are comparable
        sg, se = g.engine.samples(), e.engine.samples()
        og = np.argsort(sg["slot"], kind="stable")
        oe = np.argsort(se["slot"], kind="stable")
        for k in sg:
            assert np.array_equal(sg[k][og], se[k][oe]), k
