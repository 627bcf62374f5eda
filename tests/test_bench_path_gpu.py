"""The benchmarked self-play path, pinned to complete reference games.

bench.py plays through BatchedSelfPlay's default step: deferred moves and the fused
expansion in one select launch per step (az_select_move_expand), the K = 1 descent level
budget, slot refill, staggered starts and HIP graphs of 8 steps.  Here that exact path replays
the reference's own self-play games (self_play_worker.py:38-88 with MCTS_model.py:217-395,
recorded by tests/golden/make_goldens.py and make_deep_goldens.py: 25 / 100 / 400
simulations) with the recorded Dirichlet vectors and sampling uniforms injected, 1,024 slots
at once (the bench's slot count), each slot playing two games back to back (the refill path,
its RNG cursors running on from one game to the next), with the deterministic mock policy
as the net.  Every canonical board, pi and TD(lambda) target must be bit-identical to the
reference's, in graph and in eager execution.

K = 4 leaves per step (virtual loss, the reference's num_threads = 4) runs the same path at
256 slots x 4 rows.  The reference games there were recorded under the forced thread
schedule of make_vl_goldens.py; the engine's auto-play mode caps a step at 4 K descents,
another legal interleaving of the reference's workers, which the oracle's K-leaf self-play
models (oracle/selfplay.py, max_descents) -- so the K = 4 games are checked against the oracle
replaying the same recorded draws, and the oracle itself against the reference games without
the cap (tests/test_oracle_golden.py).
"""
import numpy as np
import pytest

from conftest import load_golden
from mock_policy import MockNet, MockPolicy
from replay_rng import case_log, engine_streams

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from engine import BatchedSelfPlay  # noqa: E402

ARGS = {"c_puct": 2.0, "dirichlet_alpha": 1.0, "dirichlet_epsilon": 0.3,
        "mcts_temperature": 1.0, "num_exploratory_moves": 35, "lambda": 0.98}


def _games(K, S):
    """(fixture, game index) of every recorded reference game with K leaves and S sims."""
    out = []
    for name in ("selfplay_games.npz", "selfplay_deep.npz"):
        d = load_golden(name)
        for g, m in enumerate(d["meta"]):
            k = int(m[3]) if len(m) > 3 else 1
            if k == K and int(m[0]) == S:
                out.append((d, g))
    return out


def _expected_rows(d, g):
    sel = d["game"] == g
    return {"own": d["pos"][sel], "opp": d["neg"][sel], "pi": d["pi"][sel], "z": d["z"][sel]}


def _oracle_rows(d, g, K):
    """The oracle's K-leaf self-play (the engine's auto-play cap of 4 K descents per step) on
    the reference game's recorded draws."""
    from oracle import board as ob
    from oracle.mcts import LogRng
    from oracle.selfplay import play_game

    kinds, a, b, noise = case_log(d, g)
    mp = MockPolicy()

    def evaluate(own, opp, player):
        return mp.inference(ob.to_state(own, opp, player), player)

    args = dict(ARGS, num_simulations=int(d["meta"][g][0]))
    samples, _ = play_game(args, evaluate, rng=LogRng(kinds, a, b, noise), leaves_per_step=K,
                           max_descents=4 * K)
    own, opp = zip(*[ob.to_bitboards(s, 1) for s, _, _ in samples])
    return {"own": np.array(own, np.uint64), "opp": np.array(opp, np.uint64),
            "pi": np.array([p for _, p, _ in samples], np.float32),
            "z": np.array([z for _, _, z in samples], np.float64)}


def _play(games, expected, S, K, G, use_graph):
    """Slot s plays games[s % n] then games[(s + 1) % n] through BatchedSelfPlay's default
    path; returns the slot-ordered sample rows and, per slot, the expected rows."""
    n = len(games)
    pairs = [(s % n, (s + 1) % n) for s in range(G)]
    streams = [engine_streams(*case_log(d, g)) for d, g in games]
    NU = max(len(streams[i][1]) + len(streams[j][1]) for i, j in pairs)
    noise = np.zeros((G, 2, 65))
    uni = np.zeros((G, NU))
    for s, (i, j) in enumerate(pairs):
        (ni, ui), (nj, uj) = streams[i], streams[j]
        assert len(ni) == len(nj) == 1  # one Dirichlet vector per game: the ply-0 root
        noise[s, 0], noise[s, 1] = ni[0], nj[0]
        uni[s, :len(ui)] = ui
        uni[s, len(ui):len(ui) + len(uj)] = uj
    sp = BatchedSelfPlay(MockNet(), dict(ARGS, num_simulations=S), G, fold=False,
                         use_graph=use_graph, require_graph=use_graph, leaves_per_step=K,
                         injected_rng=True, inj_noise_slots=2, inj_uniform_slots=NU,
                         sample_capacity=G * 2 * 70)
    assert sp.defer_moves and sp.fuse_expand  # the bench's default step
    # bench.py's schedule: starts staggered over one game length, every slot refilled once
    sp.reset(start_budget=2 * G, stagger_steps=(S + 1) * 60 // K)
    sp.inject(noise=noise, uniforms=uni)
    e = sp.engine
    for _ in range(4000):
        sp.step(256)
        if e.counters()["games_finished"] >= 2 * G:
            break
    c = e.counters()
    assert (sp.graph is not None) == use_graph and sp.graph_error is None
    assert c["games_finished"] == 2 * G and c["games_started"] == 2 * G
    assert c["arena_overflows"] == 0 and c["samples_dropped"] == 0
    smp = e.samples()
    order = np.argsort(smp["slot"], kind="stable")  # a slot's rows in the order its games ended
    smp = {k: v[order] for k, v in smp.items()}
    want = [{k: np.concatenate([expected[i][k], expected[j][k]]) for k in expected[i]}
            for i, j in pairs]
    assert c["moves"] == len(smp["z"]) == sum(len(w["z"]) for w in want)
    return smp, want


def _check(smp, want):
    bounds = np.searchsorted(smp["slot"], np.arange(len(want) + 1))
    for s, w in enumerate(want):
        lo, hi = bounds[s], bounds[s + 1]
        assert hi - lo == len(w["z"]), f"slot {s}: {hi - lo} rows, expected {len(w['z'])}"
        for k in ("own", "opp", "pi", "z"):
            assert np.array_equal(smp[k][lo:hi], w[k]), (s, k)


@pytest.mark.parametrize("S,use_graph", [(25, True), (100, True), (400, True), (400, False)])
def test_bench_path_plays_the_reference_games(S, use_graph):
    games = _games(1, S)
    assert games, S
    if S == 400:
        assert len(games) == 4  # selfplay_games.npz game 5 + selfplay_deep.npz games 0-2
    expected = [_expected_rows(d, g) for d, g in games]
    smp, want = _play(games, expected, S, 1, 1024, use_graph)
    _check(smp, want)


@pytest.mark.parametrize("S", [100, 400])
def test_bench_path_virtual_loss_games(S):
    games = _games(4, S)
    assert games, S
    expected = [_oracle_rows(d, g, 4) for d, g in games]
    for (d, g), x in zip(games, expected):
        # the first move of every game is the reference's own (no end-game cap reached there)
        ref = _expected_rows(d, g)
        assert x["own"][0] == ref["own"][0] and np.array_equal(x["pi"][0], ref["pi"][0])
    smp, want = _play(games, expected, S, 4, 256, True)
    _check(smp, want)
