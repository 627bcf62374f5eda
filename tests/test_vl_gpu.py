"""Multi-leaf (virtual-loss) search on the GPU engine: K = leaves_per_step descents per game
per step, the reference's args['num_threads'] = K workers (MCTS_model.py:115-118, :196-197,
:372-395) in the interleaving tests/golden/make_vl_goldens.py forces on the reference.

  * host-driven searches: bit-exact against the reference-generated goldens
    (mcts_vl_cases.npz: K in {2, 4, 8}, 100-400 simulations, Dirichlet noise, tree reuse);
  * auto-play self-play with K = 4: every training tuple bit-exact against the oracle's
    K-leaf self-play (oracle/selfplay.py, pinned by the same goldens on the CPU) with its
    RNG draws injected;
  * K = 1 is the num_threads = 1 engine every other GPU test checks.
"""
import numpy as np
import pytest

from conftest import load_golden
from mock_policy import MockPolicy, mock_eval_torch
from replay_rng import engine_streams

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from engine import Engine  # noqa: E402

from oracle import board as ob  # noqa: E402
from oracle.selfplay import play_game  # noqa: E402


def own_opp(pos, neg, player):
    return (int(pos), int(neg)) if player == 1 else (int(neg), int(pos))


def run_search(e, max_steps=100000):
    for _ in range(max_steps):
        e.select()
        pr, va = mock_eval_torch(e.nn_in)
        e.priors.copy_(pr)
        e.values.copy_(va)
        e.expand()
        e.play()
        if (e.game_info()["status"] != nat.AZ_GAME_ACTIVE).all():
            return
    raise AssertionError("search did not finish")


def _groups():
    d = load_golden("mcts_vl_cases.npz")
    keys = sorted({(int(d["k"][r]), int(d["sims"][r]), float(d["c_puct"][r]), float(d["eps"][r]))
                   for r in range(len(d["k"]))})
    return keys


@pytest.mark.parametrize("group", _groups())
def test_virtual_loss_searches_match_reference(group):
    K, S, cp, eps = group
    d = load_golden("mcts_vl_cases.npz")
    cases = sorted({int(d["log_case"][r]) for r in range(len(d["k"]))
                    if (int(d["k"][r]), int(d["sims"][r]), float(d["c_puct"][r]),
                        float(d["eps"][r])) == group})
    G = len(cases)
    e = Engine(G, S, c_puct=cp, dirichlet_alpha=1.0, dirichlet_epsilon=eps, injected_rng=True,
               auto_play=False, inj_noise_slots=1, leaves_per_step=K)
    assert e.nn_in.shape == (G * K, 64)
    noise = np.zeros((G, 1, 65))
    rows = []
    for s, c in enumerate(cases):
        nlo, nhi = d["noise_offsets"][c], d["noise_offsets"][c + 1]
        if nhi > nlo:
            noise[s, 0] = d["noise"][nlo]
        r = np.nonzero(d["log_case"] == c)[0]
        rows.append(r)
        own, opp = own_opp(d["pos"][r[0]], d["neg"][r[0]], d["player"][r[0]])
        e.set_root(s, own, opp, int(d["player"][r[0]]))
    e.inject(noise=noise)
    for mv in range(max(len(r) for r in rows)):
        live = [s for s in range(G) if mv < len(rows[s])]
        for s in live:
            e.begin_search(s, S)
        run_search(e)
        for s in live:
            r = rows[s][mv]
            pi, counts, vroot = e.root_policy(s, 1.0)
            assert (counts == d["counts"][r]).all(), f"K={K} case {cases[s]} move {mv}"
            assert vroot == d["root_value"][r]
            assert (pi == d["probs"][r]).all()
            assert e.export_tree(s, max_nodes=1)["N"][0] == d["root_n"][r]
            if mv + 1 < len(rows[s]):
                e.make_move(s, int(np.argmax(d["counts"][r])))
    assert e.counters()["arena_overflows"] == 0


class _GenRng:
    """Seeded draws for the oracle, logged in the injected-stream form the engine reads."""

    def __init__(self, seed):
        self.r = np.random.default_rng(seed)
        self.kinds, self.a, self.b, self.noise = [], [], [], []

    def dirichlet(self, alpha, n):
        x = self.r.dirichlet([alpha] * n)
        self.kinds.append(0)
        self.a.append(float(len(self.noise)))
        self.b.append(0)
        self.noise.append(x)
        return x

    def choice_tie(self, best):
        j = int(self.r.random() * len(best))
        self.kinds.append(1)
        self.a.append(float(len(best)))
        self.b.append(j)
        return best[j]

    def choice_p(self, n, p):
        u = float(self.r.random())
        cdf = np.asarray(p, np.float64).cumsum()
        cdf /= cdf[-1]
        r = int(cdf.searchsorted(u, side="right"))
        self.kinds.append(2)
        self.a.append(u)
        self.b.append(r)
        return r


def test_virtual_loss_self_play_matches_oracle():
    K, S, G = 4, 48, 3
    args = {"c_puct": 2.0, "num_simulations": S, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    mp = MockPolicy()

    def evaluate(own, opp, player):
        return mp.inference(ob.to_state(own, opp, player), player)

    games, streams = [], []
    for s in range(G):
        rng = _GenRng(700 + s)
        samples, _ = play_game(args, evaluate, rng=rng, leaves_per_step=K)
        games.append(samples)
        streams.append(engine_streams(rng.kinds, rng.a, rng.b,
                                      np.array(rng.noise).reshape(-1, 65)))
    NU = max(len(u) for _, u in streams)
    noise = np.zeros((G, 1, 65))
    uni = np.zeros((G, NU))
    for s, (nz, u) in enumerate(streams):
        noise[s, 0] = nz[0]
        uni[s, :len(u)] = u
    e = Engine(G, S, c_puct=2.0, dirichlet_alpha=1.0, dirichlet_epsilon=0.3, temperature=1.0,
               num_exploratory_moves=35, lambd=0.98, injected_rng=True, auto_play=True,
               refill=False, inj_noise_slots=1, inj_uniform_slots=NU, leaves_per_step=K)
    e.reset_all(start_budget=G)
    e.inject(noise=noise, uniforms=uni)
    for _ in range(200):
        for _ in range(50):
            e.select()
            pr, va = mock_eval_torch(e.nn_in)
            e.priors.copy_(pr)
            e.values.copy_(va)
            e.expand()
            e.play()
        if e.counters()["games_finished"] == G:
            break
    c = e.counters()
    assert c["games_finished"] == G and c["arena_overflows"] == 0
    smp = e.samples()
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    for s in range(G):
        mine = smp["slot"] == s
        assert mine.sum() == len(games[s])
        for t, (board, pi, z) in enumerate(games[s]):
            flat = board.reshape(-1)
            assert smp["own"][mine][t] == np.bitwise_or.reduce(np.where(flat == 1, w, np.uint64(0)))
            assert smp["opp"][mine][t] == np.bitwise_or.reduce(np.where(flat == -1, w, np.uint64(0)))
            assert (smp["pi"][mine][t] == np.asarray(pi, np.float32)).all(), f"slot {s} ply {t}"
            assert smp["z"][mine][t] == z


def test_leaves_per_step_bounds():
    with pytest.raises(RuntimeError, match="leaves_per_step"):
        Engine(1, 4, auto_play=False, leaves_per_step=9)


def test_virtual_loss_with_fused_d4_and_equivariant_policy_is_invisible():
    """K = 4 leaves per step with the fused per-leaf D4 transform (config #5): a D4-equivariant
    policy must give the same searches with and without it (each row's own transform is
    inverted on its own priors)."""
    import torch

    def eq_eval(planes):
        pr = torch.cat([planes * 0.25 + 1.0, torch.ones_like(planes[:, :1])], 1)
        return pr.contiguous(), (planes.sum(1) / 64.0).contiguous()

    res = []
    for d4 in (False, True):
        e = Engine(4, 60, d4_augment=d4, auto_play=False, seed=5, leaves_per_step=4)
        for s in range(4):
            e.set_root(s, 0x0000000810000000, 0x0000001008000000, 1)
        e.begin_search(-1, 60)
        for _ in range(500):
            e.select()
            pr, va = eq_eval(e.nn_in)
            e.priors.copy_(pr)
            e.values.copy_(va)
            e.expand()
            e.play()
            if (e.game_info()["status"] != nat.AZ_GAME_ACTIVE).all():
                break
        res.append([e.root_policy(s, 1.0)[1] for s in range(4)])
    for a, b in zip(*res):
        assert (a == b).all() and a.sum() == 60


def test_virtual_loss_rollout_mode_counts():
    """Rollout evaluation (policy None) with K = 4: every search completes its simulations."""
    e = Engine(8, 32, rollout=True, auto_play=False, leaves_per_step=4)
    for s in range(8):
        e.set_root(s, 0x0000000810000000, 0x0000001008000000, 1)
    e.begin_search(-1, 32)
    for _ in range(200):
        e.select()
        e.expand(e.priors, e.values)
        e.play()
        if (e.game_info()["status"] != nat.AZ_GAME_ACTIVE).all():
            break
    for s in range(8):
        _, counts, _ = e.root_policy(s, 1.0)
        assert counts.sum() == 32
    c = e.counters()
    assert c["arena_overflows"] == 0
    assert c["simulations"] == 8 * 32  # per-slot counts summed by az_counters


def test_batched_selfplay_with_virtual_loss_properties():
    """BatchedSelfPlay with a random-init net, device RNG and K = 4 leaves per game per step:
    every finished game yields well-formed training tuples."""
    import torch

    from engine import BatchedSelfPlay
    from Models import FastOthelloNet

    torch.manual_seed(0)
    args = {"c_puct": 2.0, "num_simulations": 16, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    sp = BatchedSelfPlay(FastOthelloNet(8, 65), args, 32, seed=1, use_graph=True,
                         leaves_per_step=4)
    assert sp.engine.nn_in.shape == (128, 64)
    tuples = sp.play_games(48)
    c = sp.engine.counters()
    assert c["games_finished"] == 48 and c["arena_overflows"] == 0
    smp = sp.engine.samples()
    assert len(tuples) == c["samples"] >= 9 * 48
    assert ((smp["own"] & smp["opp"]) == 0).all()
    assert np.allclose(smp["pi"].sum(1), 1.0, atol=1e-5)
    assert (np.abs(smp["z"]) <= 1.0).all()


@pytest.mark.parametrize("threads,pipelines", [(None, 1), (1, 1), (1, 2)])
def test_collect_self_play_games_drop_in(threads, pipelines):
    """self_play_worker.collect_self_play_games (the batched replacement of train.py's pool)
    at the reference's default worker count (4 leaves per step) and at num_threads = 1:
    the reference's training tuples, one list per call."""
    import torch

    from Models import FastOthelloNet
    from self_play_worker import collect_self_play_games

    torch.manual_seed(0)
    args = {"c_puct": 2.0, "num_simulations": 12, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    if threads is not None:
        args["num_threads"] = threads
    out = collect_self_play_games(FastOthelloNet(8, 65), args, 20, pipelines=pipelines)
    assert len(out) >= 9 * 20
    for s, pi, z in out:
        assert s.shape == (8, 8) and s.dtype == np.int8
        assert pi.shape == (65,) and abs(float(pi.sum()) - 1.0) < 1e-5
        assert -1.0 <= z <= 1.0
