"""configs[3] / configs[4] at full per-GPU width (4,096 concurrent games, BASELINE.json):

* the auto-play engine with all 4,096 slots (the 7.5 GB node arena of one GPU's share of
  the 32,768-game node) replays the 100-sim golden self-play games of the reference
  (tests/golden/selfplay_games.npz, recorded Dirichlet vectors and uniforms injected per
  slot): every slot's training tuples are bit-exact;
* the per-generation replay exchange (dist_replay.allgather_samples, train.py:220-223's
  replacement) over the RCCL ("nccl") backend on device rows taken from a real engine, at
  world_size 1: bit-exact against the input rows.
"""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import load_golden
from mock_policy import mock_eval_torch
from replay_rng import case_log, engine_streams

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from engine import Engine  # noqa: E402

G_FULL = 4096


def _replicated_golden_engine(games, G, sample_capacity=0):
    """An auto-play engine whose slot s plays golden game games[s % len(games)] with its
    recorded random draws injected."""
    d = load_golden("selfplay_games.npz")
    S = int(d["meta"][games[0]][0])
    assert all(int(d["meta"][g][0]) == S for g in games)
    streams = [engine_streams(*case_log(d, g)) for g in games]
    NU = max(len(u) for _, u in streams)
    noise = np.zeros((G, 1, 65))
    uni = np.zeros((G, NU))
    for s in range(G):
        nz, u = streams[s % len(games)]
        noise[s, 0] = nz[0]
        uni[s, :len(u)] = u
    e = Engine(G, S, c_puct=2.0, dirichlet_alpha=1.0, dirichlet_epsilon=0.3,
               temperature=1.0, num_exploratory_moves=35, lambd=0.98, injected_rng=True,
               auto_play=True, refill=False, inj_noise_slots=1, inj_uniform_slots=NU,
               sample_capacity=sample_capacity)
    e.reset_all(start_budget=G)
    e.inject(noise=noise, uniforms=uni)
    return d, e


def _drive(e, G, chunk=200, max_chunks=400):
    for _ in range(max_chunks):
        for _ in range(chunk):
            e.select()
            pr, va = mock_eval_torch(e.nn_in)
            e.priors.copy_(pr)
            e.values.copy_(va)
            e.expand()
            e.play()
        if e.counters()["games_finished"] == G:
            return
    raise AssertionError("games did not finish")


@pytest.mark.timeout(900)
def test_4096_slots_replay_golden_games_bit_exact():
    games = [3, 4]  # the two 100-sim reference games
    d, e = _replicated_golden_engine(games, G_FULL)
    assert e.G == G_FULL
    _drive(e, G_FULL)
    c = e.counters()
    assert c["games_finished"] == G_FULL
    assert c["arena_overflows"] == 0 and c["samples_dropped"] == 0
    smp = e.samples()
    order = np.argsort(smp["slot"], kind="stable")  # rows of one slot stay in ply order
    slot = smp["slot"][order]
    for gi, g in enumerate(games):
        sel = d["game"] == g
        n = int(sel.sum())
        slots = np.arange(gi, G_FULL, len(games))
        rows = np.isin(slot, slots)
        assert rows.sum() == n * len(slots)
        own = smp["own"][order][rows].reshape(len(slots), n)
        opp = smp["opp"][order][rows].reshape(len(slots), n)
        pi = smp["pi"][order][rows].reshape(len(slots), n, 65)
        z = smp["z"][order][rows].reshape(len(slots), n)
        assert (own == d["pos"][sel][None]).all()
        assert (opp == d["neg"][sel][None]).all()
        assert (pi == d["pi"][sel][None]).all()
        assert (z == d["z"][sel][None]).all()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_allgather_of_engine_rows_world1():
    import torch.distributed as dist

    from dist_replay import allgather_samples

    d, e = _replicated_golden_engine([0, 1, 2], 6)
    _drive(e, 6, chunk=100)
    n = e.counters()["samples"]
    rows = e.samples(0, n, device=True)
    assert rows["own"].is_cuda and n == 6 * 60
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        got, counts = allgather_samples(rows, torch.device("cuda", 0))
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    assert counts == [n]
    for k in ("own", "opp", "pi", "z", "player"):
        assert got[k].is_cuda
        a = got[k].cpu().numpy()
        b = rows[k].cpu().numpy()
        assert a.dtype.itemsize == b.dtype.itemsize
        assert np.array_equal(a.view(np.uint8), b.reshape(a.shape).view(np.uint8)), k


def test_sample_buffer_overflow_keeps_committed_rows_intact():
    """More finished games than the sample buffer holds: a game whose rows do not fit is
    rejected whole (samples_dropped), the counter never passes the capacity, and every row
    that was kept is its game's reference row (no reservation is overwritten)."""
    games = [0, 1, 2]
    cap = 200  # three 60-ply games fit, the other three are dropped
    d, e = _replicated_golden_engine(games, 6, sample_capacity=cap)
    _drive(e, 6, chunk=100)
    c = e.counters()
    assert c["games_finished"] == 6
    assert c["samples"] == 180 and c["samples_dropped"] == 180
    smp = e.samples(0, c["samples"])
    for s in np.unique(smp["slot"]):
        g = games[s % len(games)]
        sel = d["game"] == g
        mine = smp["slot"] == s
        assert mine.sum() == sel.sum()
        assert (smp["own"][mine] == d["pos"][sel]).all()
        assert (smp["pi"][mine] == d["pi"][sel]).all()
        assert (smp["z"][mine] == d["z"][sel]).all()
    with pytest.raises(RuntimeError):
        from engine import check_complete
        check_complete(c, 6)
