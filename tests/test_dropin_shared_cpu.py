"""one_self_play's shared generation (self_play_worker._shared_game): train.py's spawn-pool
workers (train.py:199-225) share ONE batch of num_self_play games -- the first worker plays it,
every call claims the next game -- on synthetic sample rows (no GPU): every game is handed out
exactly once across processes, in slot order within a process, one producer, the directory
removed after the last read, a dead producer's directory retired, a failed one reported."""
import multiprocessing as mp
import os
import pathlib
import shutil
import sys
import uuid

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import self_play_worker as spw  # noqa: E402


@pytest.fixture
def scratch():
    """A fresh directory under tests/_scratch/ (inside the checkout), removed afterwards."""
    d = os.path.join(ROOT, "tests", "_scratch", uuid.uuid4().hex)
    os.makedirs(d)
    yield pathlib.Path(d)
    shutil.rmtree(d, ignore_errors=True)


INIT_OWN, INIT_OPP = 0x0000000810000000, 0x0000001008000000


def _fake_rows(total):
    """total games in slot order, game g: 3 + g % 4 plies; its first row the initial position
    and every pi row tagged with g (so a returned game names its index)."""
    own, opp, pi, z, player, slot = [], [], [], [], [], []
    for g in range(total):
        for t in range(3 + g % 4):
            own.append(INIT_OWN | (1 << (40 + t)) if t else INIT_OWN)
            opp.append(INIT_OPP)
            row = np.zeros(65, np.float32)
            row[g % 65] = 1.0
            row[64] = g
            pi.append(row)
            z.append(0.5)
            player.append(1)
            slot.append(g)
    # the ring holds games in completion order, not slot order: reverse it
    order = np.argsort(-np.asarray(slot), kind="stable")
    return {"own": np.asarray(own, np.uint64)[order].view(np.int64),
            "opp": np.asarray(opp, np.uint64)[order].view(np.int64),
            "pi": np.asarray(pi, np.float32)[order], "z": np.asarray(z)[order],
            "player": np.asarray(player, np.int8)[order], "slot": np.asarray(slot, np.int32)[order]}


def _produce(total):
    with open(os.path.join(os.environ["AZ_DROPIN_DIR"], "..", "produced"), "a") as f:
        f.write(f"{os.getpid()}\n")
    return _fake_rows(total)


def _game_index(game):
    return int(game[0][1][64])


def _worker(d, key, total, calls, q):
    os.environ["AZ_DROPIN_DIR"] = d
    got = []
    for _ in range(calls):
        g = spw._shared_game(key, total, _produce)
        if g is None:
            break
        got.append(_game_index(g))
    q.put((os.getpid(), got))


def test_shared_generation_hands_out_every_game_once(scratch):
    d = str(scratch / "gen")
    total, procs, key = 24, 4, "k" * 40  # exactly `total` calls, as train.py makes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(d, key, total, total // procs, q))
          for _ in range(procs)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(procs)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    got = [i for _, g in res for i in g]
    assert sorted(got) == list(range(total))
    for _, g in res:
        assert g == sorted(g)  # each process claims upward
    with open(scratch / "produced") as f:
        assert len(f.read().split()) == 1  # one producer
    assert not os.path.exists(os.path.join(d, key))  # the last reader removed it


def test_shared_generation_game_contents(scratch, monkeypatch):
    monkeypatch.setenv("AZ_DROPIN_DIR", str(scratch / "gen"))
    rows = _fake_rows(5)
    want = spw._games_from_rows(rows)
    got = [spw._shared_game("c" * 40, 5, lambda n: _fake_rows(n)) for _ in range(5)]
    for a, b in zip(got, want):
        assert len(a) == len(b)
        for (s1, p1, z1), (s2, p2, z2) in zip(a, b):
            assert np.array_equal(s1, s2) and np.array_equal(p1, p2) and z1 == z2
    assert [len(g) for g in got] == [3 + g % 4 for g in range(5)]


def test_dead_producer_is_retired(scratch, monkeypatch):
    monkeypatch.setenv("AZ_DROPIN_DIR", str(scratch / "gen"))
    p = mp.get_context("spawn").Process(target=int)
    p.start()
    p.join()
    d = scratch / "gen" / ("d" * 40)
    d.mkdir(parents=True)
    (d / "producer").write_text(str(p.pid))  # exited without publishing
    g = spw._shared_game("d" * 40, 3, lambda n: _fake_rows(n), poll_s=0.001)
    assert _game_index(g) == 0
    assert any(n.startswith("d" * 40 + ".dead.") for n in os.listdir(scratch / "gen"))


def test_failed_producer_is_reported(scratch, monkeypatch):
    """The producer's error propagates from its call; a waiter that sees `failed` raises it; a
    later call produces anew."""
    monkeypatch.setenv("AZ_DROPIN_DIR", str(scratch / "gen"))

    def boom(n):
        raise ValueError("no GPU")

    with pytest.raises(ValueError):
        spw._shared_game("f" * 40, 3, boom)
    assert any(".failed." in n for n in os.listdir(scratch / "gen"))
    assert _game_index(spw._shared_game("f" * 40, 3, lambda n: _fake_rows(n))) == 0
    d = scratch / "gen" / ("e" * 40)  # a live producer (this process) that failed
    d.mkdir()
    (d / "producer").write_text(str(os.getpid()))
    (d / "failed").write_text("ValueError('no GPU')")
    with pytest.raises(RuntimeError, match="no GPU"):
        spw._shared_game("e" * 40, 3, lambda n: _fake_rows(n))


def test_stale_generations_are_retired_but_not_live_producers(scratch):
    root = scratch / "gen"
    old_done, old_dead, old_live = (root / n for n in ("a" * 40, "b" * 40, "c" * 40))
    for d in (old_done, old_dead, old_live):
        d.mkdir(parents=True)
    (old_done / "done").write_text("x")
    p = mp.get_context("spawn").Process(target=int)
    p.start()
    p.join()
    (old_dead / "producer").write_text(str(p.pid))
    (old_live / "producer").write_text(str(os.getpid()))  # still playing
    for d in (old_done, old_dead, old_live):
        os.utime(d, (0, 0))
    spw._retire_stale(str(root), "z" * 40)
    assert not old_done.exists() and not old_dead.exists() and old_live.exists()


def test_shared_total_from_args(monkeypatch):
    assert spw._shared_total({"num_self_play": 300, "num_workers": 15}) == 300
    assert spw._shared_total({"num_workers": 15}) is None
    assert spw._shared_total(None) is None
    monkeypatch.setenv("AZ_DROPIN_SHARED", "0")
    assert spw._shared_total({"num_self_play": 300}) is None
