"""The benchmarked self-play path, pinned to complete reference games.

bench.py plays through BatchedSelfPlay's default step: deferred moves and the fused
expansion in one select launch per step (az_select_move_expand), the K = 1 descent level
budget, slot refill, staggered starts and HIP graphs of 8 steps.  Here that exact path replays
the reference's own self-play games (self_play_worker.py:38-88 with MCTS_model.py:217-395,
recorded by tests/golden/make_goldens.py and make_deep_goldens.py: 25 / 100 / 400
simulations) with the recorded Dirichlet vectors and sampling uniforms injected, 1,024 slots
at once (the bench's slot count), each slot playing its queue of games back to back (the
refill path, its RNG cursors running on from one game to the next) until every slot has
completed at least two, with the deterministic mock policy
as the net.  Every canonical board, pi and TD(lambda) target must be bit-identical to the
reference's, in graph and in eager execution.

K = 4 leaves per step (virtual loss, the reference's num_threads = 4) runs the same path at
256 slots x 4 rows against reference games recorded under the forced thread schedule of
make_vl_goldens.py (simulations started until K wait on the net): a select launch that reaches
its descent cap leaves the batch open and the next launch continues it, so the engine's
batches are the reference's wherever the launches split them.
"""
import numpy as np
import pytest

from conftest import load_golden
from mock_policy import MockNet
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


NG = 4  # reference games queued per slot (its injected streams, back to back)


def _play(games, expected, S, K, G, use_graph):
    """Slot s plays games[(s + i) % n], i = 0, 1, ... through BatchedSelfPlay's default path
    with unlimited refill and bench.py's staggered starts, until every slot has completed at
    least two games; returns per slot its sample rows and the expected rows of its queue."""
    n = len(games)
    queues = [[(s + i) % n for i in range(NG)] for s in range(G)]
    streams = [engine_streams(*case_log(d, g)) for d, g in games]
    NU = max(sum(len(streams[i][1]) for i in q) for q in queues)
    noise = np.zeros((G, NG, 65))
    uni = np.zeros((G, NU))
    for s, q in enumerate(queues):
        u = 0
        for i, gi in enumerate(q):
            nz, us = streams[gi]
            assert len(nz) == 1  # one Dirichlet vector per game: the ply-0 root
            noise[s, i] = nz[0]
            uni[s, u:u + len(us)] = us
            u += len(us)
    sp = BatchedSelfPlay(MockNet(), dict(ARGS, num_simulations=S), G, fold=False,
                         use_graph=use_graph, require_graph=use_graph, leaves_per_step=K,
                         injected_rng=True, inj_noise_slots=NG, inj_uniform_slots=NU,
                         sample_capacity=G * NG * 70)
    assert sp.defer_moves and sp.fuse_expand  # the bench's default step
    # bench.py's schedule: starts staggered over one game length, slots refilled as their
    # games end; stepped until the last-started slot has completed two games (a game is at
    # most 64 plies of ceil(S / K) + 1 steps, + 1 per ply sitting out) -- then no slot is
    # past the NG games queued for it
    per_game = 64 * (-(-S // K) + 2)
    stagger = (-(-S // K) + 1) * 60
    sp.reset(start_budget=-1, stagger_steps=stagger)
    sp.inject(noise=noise, uniforms=uni)
    total = stagger + 2 * per_game + 64
    done = 0
    while done < total:
        sp.step(min(1024, total - done))
        done += min(1024, total - done)
    e = sp.engine
    c = e.counters()
    assert (sp.graph is not None) == use_graph and sp.graph_error is None
    assert c["arena_overflows"] == 0 and c["samples_dropped"] == 0
    smp = e.samples()
    order = np.argsort(smp["slot"], kind="stable")  # a slot's rows in the order its games ended
    smp = {k: v[order] for k, v in smp.items()}
    want = [[expected[gi] for gi in q] for q in queues]
    return smp, want


def _check(smp, want):
    """Every slot's rows are its queue's first m >= 2 games, bit for bit."""
    bounds = np.searchsorted(smp["slot"], np.arange(len(want) + 1))
    games_checked = 0
    for s, q in enumerate(want):
        lo, hi = bounds[s], bounds[s + 1]
        m, rows = 0, 0
        while m < len(q) and rows + len(q[m]["z"]) <= hi - lo:
            rows += len(q[m]["z"])
            m += 1
        assert rows == hi - lo and 2 <= m < len(q), f"slot {s}: {hi - lo} rows, {m} games"
        for k in ("own", "opp", "pi", "z"):
            w = np.concatenate([g[k] for g in q[:m]])
            assert np.array_equal(smp[k][lo:hi], w), (s, k)
        games_checked += m
    return games_checked


@pytest.mark.parametrize("S,use_graph", [(25, True), (100, True), (400, True), (400, False)])
def test_bench_path_plays_the_reference_games(S, use_graph):
    games = _games(1, S)
    assert games, S
    if S == 400:
        assert len(games) == 4  # selfplay_games.npz game 5 + selfplay_deep.npz games 0-2
    expected = [_expected_rows(d, g) for d, g in games]
    smp, want = _play(games, expected, S, 1, 1024, use_graph)
    assert _check(smp, want) >= 2 * 1024


@pytest.mark.parametrize("S", [100, 400])
def test_bench_path_virtual_loss_games(S):
    games = _games(4, S)
    assert games, S
    expected = [_expected_rows(d, g) for d, g in games]
    smp, want = _play(games, expected, S, 4, 256, True)
    assert _check(smp, want) >= 2 * 256
