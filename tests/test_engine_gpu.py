"""Parity of the GPU MCTS engine (select / expand+backup / move kernels) with the
reference, on golden vectors recorded by running the reference itself with
args['num_threads'] = 1 and the deterministic mock policy (tests/golden/make_goldens.py).
Bit-exact: visit counts, root values, pi, canonical boards and TD(lambda) targets."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from mock_policy import MockPolicyNet, mock_eval_torch
from replay_rng import ReplayNpRandom, case_log, engine_streams

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from engine import Engine  # noqa: E402

INIT_OWN, INIT_OPP = 0x0000000810000000, 0x0000001008000000


def own_opp(pos, neg, player):
    return (int(pos), int(neg)) if player == 1 else (int(neg), int(pos))


def run_search(e, max_steps=100000):
    """Host-driven engine: step until every active slot's search is done."""
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


@pytest.mark.parametrize("group", [(2.0, 0.0), (1.0, 0.3), (2.0, 0.3)])
def test_mcts_cases_match_reference(group):
    d = load_golden("mcts_cases.npz")
    n_cases = int(d["n_cases"])
    cases = [c for c in range(n_cases)
             if (float(d["c_puct"][d["log_case"] == c][0]),
                 float(d["eps"][d["log_case"] == c][0])) == group]
    G = len(cases)
    e = Engine(G, 1, c_puct=group[0], dirichlet_alpha=1.0, dirichlet_epsilon=group[1],
               injected_rng=True, auto_play=False, inj_noise_slots=2, inj_uniform_slots=4)
    noise = np.zeros((G, 2, 65))
    rows = []
    ties = []
    for s, c in enumerate(cases):
        kinds, a, b, nz = case_log(d, c)
        if len(nz):
            noise[s, :len(nz)] = nz
        ties.append([(int(x), int(y)) for k, x, y in zip(kinds, a, b) if k == 1])
        r = np.nonzero(d["log_case"] == c)[0]
        rows.append(r)
        own, opp = own_opp(d["pos"][r[0]], d["neg"][r[0]], d["player"][r[0]])
        e.set_root(s, own, opp, int(d["player"][r[0]]))
    e.inject(noise=noise)
    max_moves = max(len(r) for r in rows)
    for mv in range(max_moves):
        live = [s for s in range(G) if mv < len(rows[s])]
        for s in live:
            e.begin_search(s, int(d["sims"][rows[s][mv]]))
        run_search(e)
        for s in live:
            r = rows[s][mv]
            temp = float(d["temp"][r])
            u_tie = 0.0
            if abs(temp) < 0.1:
                k, j = ties[s].pop(0)
                u_tie = (j + 0.5) / k
            pi, counts, vroot = e.root_policy(s, temp, u_tie)
            assert (counts == d["counts"][r]).all(), f"case {cases[s]} move {mv}"
            assert vroot == d["root_value"][r]
            assert (pi == d["probs"][r]).all()
            t = e.export_tree(s, max_nodes=1)
            assert t["N"][0] == d["root_n"][r]
            if mv + 1 < len(rows[s]):
                e.make_move(s, int(np.argmax(d["counts"][r])))


def test_make_move_on_non_child_raises_keyerror():
    e = Engine(1, 4, auto_play=False)
    e.set_root(0, INIT_OWN, INIT_OPP, 1)
    e.begin_search(0, 4)
    run_search(e)
    with pytest.raises(KeyError):
        e.make_move(0, 0)  # corner: not a legal opening move
    e.make_move(0, 19)


def test_selfplay_games_match_reference_on_device():
    """The auto-play engine plays the six golden games concurrently (one slot each) with the
    recorded Dirichlet vectors and uniforms injected; every training tuple must match."""
    d = load_golden("selfplay_games.npz")
    n_games = len(d["meta"])
    sims = [int(m[0]) for m in d["meta"]]
    # slots of one engine share num_simulations: one engine per sims value
    for S in sorted(set(sims)):
        games = [g for g in range(n_games) if sims[g] == S]
        G = len(games)
        streams = [engine_streams(*case_log(d, g)) for g in games]
        NU = max(len(u) for _, u in streams)
        noise = np.zeros((G, 1, 65))
        uni = np.zeros((G, NU))
        for s, (nz, u) in enumerate(streams):
            noise[s, 0] = nz[0]
            uni[s, :len(u)] = u
        e = Engine(G, S, c_puct=2.0, dirichlet_alpha=1.0, dirichlet_epsilon=0.3,
                   temperature=1.0, num_exploratory_moves=35, lambd=0.98, injected_rng=True,
                   auto_play=True, refill=False, inj_noise_slots=1, inj_uniform_slots=NU)
        e.reset_all(start_budget=G)
        e.inject(noise=noise, uniforms=uni)
        for _ in range(1000):
            for _ in range(100):
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
        # every move is exactly S simulations (per-slot counts summed by az_counters)
        assert c["simulations"] == S * len(smp["z"]) and c["moves"] == len(smp["z"])
        for s, g in enumerate(games):
            sel = d["game"] == g
            mine = smp["slot"] == s
            assert mine.sum() == sel.sum()
            # canonical boards: own stones = +1 (state*player)
            assert (smp["own"][mine] == d["pos"][sel]).all()
            assert (smp["opp"][mine] == d["neg"][sel]).all()
            assert (smp["pi"][mine] == d["pi"][sel]).all()
            assert (smp["z"][mine] == d["z"][sel]).all()


def test_drop_in_one_self_play_matches_reference(monkeypatch):
    """self_play_worker.one_self_play -> MCTS drop-in (GPU engine, host-driven) with the
    recorded np.random draws replayed: identical training tuples (the one-game-per-call path,
    AZ_DROPIN_BATCH=1)."""
    import self_play_worker

    monkeypatch.setenv("AZ_DROPIN_BATCH", "1")

    d = load_golden("selfplay_games.npz")
    for g in (0, 3):
        sims = int(d["meta"][g][0])
        args = {"c_puct": 2.0, "num_simulations": sims, "num_threads": 1,
                "dirichlet_alpha": 1.0, "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0,
                "num_exploratory_moves": 35, "lambda": 0.98}
        with ReplayNpRandom(*case_log(d, g)) as rr:
            out = self_play_worker.one_self_play((8, args, (MockPolicyNet, {}, {}), None))
        assert rr.i == len(rr.kinds)
        sel = d["game"] == g
        assert len(out) == sel.sum()
        w = np.uint64(1) << np.arange(64, dtype=np.uint64)
        for t, (s, pi, z) in enumerate(out):
            flat = s.reshape(-1)
            pos = np.bitwise_or.reduce(np.where(flat == 1, w, np.uint64(0)))
            neg = np.bitwise_or.reduce(np.where(flat == -1, w, np.uint64(0)))
            assert pos == d["pos"][sel][t] and neg == d["neg"][sel][t]
            assert (np.asarray(pi, np.float32) == d["pi"][sel][t]).all()
            assert z == d["z"][sel][t]


def test_rollout_mode_and_counts():
    e = Engine(8, 32, rollout=True, auto_play=False)
    for s in range(8):
        e.set_root(s, INIT_OWN, INIT_OPP, 1)
    e.begin_search(-1, 32)
    for _ in range(200):
        e.select()
        e.expand(e.priors, e.values)
        e.play()
        if (e.game_info()["status"] != nat.AZ_GAME_ACTIVE).all():
            break
    for s in range(8):
        pi, counts, v = e.root_policy(s, 1.0)
        assert counts.sum() == 32 and abs(pi.sum() - 1) < 1e-6 and -1 <= v <= 1


def test_d4_augment_with_equivariant_policy_is_invisible():
    """A policy that depends on each cell only is D4-equivariant, so the fused random
    transform + inverse prior map must leave every search result unchanged."""

    def eq_eval(planes):
        pr = torch.cat([planes * 0.25 + 1.0, torch.ones_like(planes[:, :1])], 1)
        return pr.contiguous(), (planes.sum(1) / 64.0).contiguous()

    res = []
    for d4 in (False, True):
        e = Engine(4, 40, d4_augment=d4, auto_play=False, seed=5)
        for s in range(4):
            e.set_root(s, INIT_OWN, INIT_OPP, 1)
        e.begin_search(-1, 40)
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
        assert (a == b).all()


def test_batched_selfplay_properties():
    """Random-init FastOthelloNet, device RNG, slot refill: every finished game yields
    well-formed training tuples (property checks at scale)."""
    from engine import BatchedSelfPlay
    from Models import FastOthelloNet

    torch.manual_seed(0)
    args = {"c_puct": 2.0, "num_simulations": 8, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    sp = BatchedSelfPlay(FastOthelloNet(8, 65), args, 64, seed=1, use_graph=True)
    tuples = sp.play_games(96)
    c = sp.engine.counters()
    assert c["games_finished"] == 96 and c["arena_overflows"] == 0
    assert len(tuples) == c["samples"]
    smp = sp.engine.samples()
    assert ((smp["own"] & smp["opp"]) == 0).all()
    assert np.allclose(smp["pi"].sum(1), 1.0, atol=1e-5)
    assert (np.abs(smp["z"]) <= 1.0).all()
    assert len(tuples) >= 9 * 96  # the shortest possible Othello game has 9 plies
    s0, pi0, z0 = tuples[0]
    assert s0.dtype == np.int8 and s0.shape == (8, 8) and pi0.shape == (65,)


def test_d4_augment_priors_match_reference_unsymmetrise():
    """Fused D4 (config #5) with a NON-equivariant policy: every slot's random transform is
    recovered from the packed leaf (an asymmetric position has 8 distinct images), and the
    expanded children's priors must equal, bit for bit, the reference's path
    unsymmetrise_pi(policy(random_symmetry(state))) (MCTS_model.py:15-43, :313-318)
    followed by the mask and renormalisation of :345-349 -- restated in NumPy on the
    reference's own (k, flip) index tables (tests/golden/d4.npz)."""
    from mock_policy import mock_eval

    d4 = load_golden("d4.npz")
    corpus = load_golden("board_corpus.npz")
    i = np.nonzero((corpus["game"] == 1) & (corpus["ply"] == 11))[0][0]
    player = int(corpus["player"][i])
    pos, neg = int(corpus["pos"][i]), int(corpus["neg"][i])
    own, opp = own_opp(pos, neg, player)
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    canon = (((np.uint64(own) & w) != 0).astype(np.int64)
             - ((np.uint64(opp) & w) != 0).astype(np.int64))  # player * state, flat
    images = np.stack([canon[d4["sym_board"][s]] for s in range(8)])
    assert len({tuple(x) for x in images}) == 8  # asymmetric: the transform is identifiable
    G = 64
    e = Engine(G, 1, d4_augment=True, auto_play=False, seed=11)
    for s in range(G):
        e.set_root(s, own, opp, player)
    e.begin_search(-1, 1)
    e.select()
    planes = np.rint(e.nn_in.cpu().numpy()).astype(np.int64)
    syms = [int(np.nonzero((images == planes[g]).all(1))[0][0]) for g in range(G)]
    assert len(set(syms)) == 8  # every D4 element drawn somewhere
    pr, va = mock_eval_torch(e.nn_in)  # position-dependent: not D4-equivariant
    e.priors.copy_(pr)
    e.values.copy_(va)
    e.expand()
    valid = np.zeros(65, np.uint8)
    legal = nat.legal_cpu(np.array([own], np.uint64), np.array([opp], np.uint64))[0]
    valid[:64] = ((np.uint64(legal) >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(np.uint8)
    if legal == 0:
        valid[64] = 1
    for g in range(G):
        p_sym, _ = mock_eval(images[syms[g]])  # the policy on the transformed board
        # unsymmetrise_pi of arange(65) (float64 in the fixture) is the gather index map
        priors = p_sym[d4["sym_unpi"][syms[g]].astype(np.int64)]
        priors = priors * valid  # float32 * uint8 -> float32 (NEP 50)
        tot = priors.sum()
        if tot > 1e-12:
            priors = priors / tot
        t = e.export_tree(g)
        fc, nc = int(t["first"][0]), int(t["nchild"][0])
        acts = t["action"][fc:fc + nc].astype(np.int64)
        assert (acts == np.nonzero(valid)[0]).all()
        assert (t["prior"][fc:fc + nc].astype(np.float32) == priors[acts]).all(), g


def test_drop_in_one_self_play_batched(monkeypatch):
    """one_self_play's default per-process batch (AZ_DROPIN_BATCH games on the batched engine
    at the first call, one returned per call): the games are exactly the engine's games for
    the seed the first call draws from np.random; a batch is reused only for the same
    weights and args; every game is a complete reference-format trajectory."""
    import self_play_worker as spw
    from Models import FastOthelloNet

    monkeypatch.setenv("AZ_DROPIN_BATCH", "4")
    spw._BATCH.update(key=None, games=[])
    torch.manual_seed(0)
    net = FastOthelloNet(8, 65)
    ps = (FastOthelloNet, net.get_config(), net.state_dict())
    args = {"c_puct": 2.0, "num_simulations": 6, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    np.random.seed(123)
    got = [spw.one_self_play((8, args, ps, None)) for _ in range(4)]
    assert not spw._BATCH["games"]
    np.random.seed(123)
    seed = int(np.random.randint(0, 2**31 - 1))
    want = spw._games_from_rows(spw._local_rows(net, args, 4, None, seed, 0, False,
                                                torch.float32))
    assert len(want) == 4
    # handed out in slot order (_games_from_rows), exactly the engine's games

    for g, w in zip(got, want):
        assert len(g) == len(w) >= 10
        s0 = g[0][0]
        assert (s0 != 0).sum() == 4 and s0[3, 4] == 1 and s0[3, 3] == -1
        for (s, pi, z), (ws, wpi, wz) in zip(g, w):
            assert s.dtype == np.int8 and s.shape == (8, 8) and pi.shape == (65,)
            assert np.array_equal(s, ws) and np.array_equal(pi, wpi) and z == wz
            assert abs(float(pi.sum()) - 1.0) < 1e-5 and -1.0 <= z <= 1.0
    # the next call starts a new batch; other weights or args never reuse it
    spw.one_self_play((8, args, ps, None))
    assert len(spw._BATCH["games"]) == 3
    key = spw._BATCH["key"]
    torch.manual_seed(1)
    ps2 = (FastOthelloNet, net.get_config(), FastOthelloNet(8, 65).state_dict())
    spw.one_self_play((8, args, ps2, None))
    assert spw._BATCH["key"] != key and len(spw._BATCH["games"]) == 3
    spw.one_self_play((8, dict(args, num_simulations=7), ps2, None))
    assert len(spw._BATCH["games"]) == 3


def test_drop_in_batch_hands_out_slot_order(monkeypatch):
    """AZ_DROPIN_BATCH = 8: the first k games one_self_play returns are exactly slots
    0..k-1's games of the batch (not the k that finished first: the sample ring is in
    completion order, i.e. shortest first), so a worker returning only part of its batch
    returns games whose lengths do not depend on the handout."""
    import self_play_worker as spw
    from Models import FastOthelloNet

    monkeypatch.setenv("AZ_DROPIN_BATCH", "8")
    spw._BATCH.update(key=None, games=[])
    torch.manual_seed(0)
    net = FastOthelloNet(8, 65)
    ps = (FastOthelloNet, net.get_config(), net.state_dict())
    args = {"c_puct": 2.0, "num_simulations": 6, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    np.random.seed(7)
    got = [spw.one_self_play((8, args, ps, None)) for _ in range(3)]
    np.random.seed(7)
    seed = int(np.random.randint(0, 2**31 - 1))
    rows = spw._local_rows(net, args, 8, None, seed, 0, False, torch.float32)
    slot = np.asarray(rows["slot"])
    tuples = spw._rows_to_tuples(rows)
    per_slot = [[tuples[i] for i in np.flatnonzero(slot == s)] for s in range(8)]
    assert sorted(len(g) for g in per_slot) == sorted(len(g) for g in spw._games_from_rows(rows))
    for k, g in enumerate(got):
        w = per_slot[k]
        assert len(g) == len(w)
        for (s, pi, z), (ws, wpi, wz) in zip(g, w):
            assert np.array_equal(s, ws) and np.array_equal(pi, wpi) and z == wz
    # the ring's completion order differs from slot order for this seed (else the test
    # would not tell them apart)
    ring_first = [int(x) for x in slot[np.r_[0, np.flatnonzero(np.diff(slot)) + 1]]]
    assert ring_first != list(range(8))
    spw._BATCH.update(key=None, games=[])
