"""The N>1 path on CPU: world_size-2 gloo process group running the per-generation replay
all-gather (dist_replay.allgather_samples) and the best-net broadcast, bit-exact."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows(rank, n):
    rng = np.random.default_rng(rank)
    return {"own": rng.integers(0, 2**63, n, dtype=np.int64).astype(np.uint64) | np.uint64(1 << 63),
            "opp": rng.integers(0, 2**63, n, dtype=np.int64).astype(np.uint64),
            "pi": rng.random((n, 65)).astype(np.float32),
            "z": rng.standard_normal(n),
            "player": rng.choice([-1, 1], n).astype(np.int8)}


def _worker(rank, world, port, q, counts=(5, 0, 3)):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "alphazero-othello_amd"))
    from dist_replay import allgather_samples, broadcast_state_dict
    from Models import FastOthelloNet

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    counts = list(counts)[:world]
    got, cnts = allgather_samples(_rows(rank, counts[rank]), "cpu")
    torch.manual_seed(rank)
    net = FastOthelloNet(8, 65)
    broadcast_state_dict(net, src=0)
    w = float(net.fc_value2.weight.sum())
    q.put((rank, cnts, {k: v.numpy() for k, v in got.items()}, w))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, counts=(5, 0, 3)):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, counts)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def test_replay_allgather_world2_bit_exact():
    res = _run(2)
    want = [_rows(0, 5), _rows(1, 0)]
    for rank, cnts, got, w in res:
        assert cnts == [5, 0]
        for k in ("own", "opp", "pi", "z", "player"):
            exp = np.concatenate([want[0][k], want[1][k]])
            g = got[k]
            if k in ("own", "opp"):
                g = g.view(np.uint64)
            assert np.array_equal(g, exp), k
    assert res[0][3] == res[1][3]  # broadcast weights identical on every rank


def test_replay_allgather_world2_no_rows_anywhere():
    """A window in which no rank finished a move: counts [0, 0], no rows collective, empty
    pooled rows on every rank."""
    res = _run(2, counts=(0, 0))
    for rank, cnts, got, w in res:
        assert cnts == [0, 0]
        assert all(len(got[k]) == 0 for k in ("own", "opp", "pi", "z", "player"))


def test_pack_unpack_rows_edge_counts():
    """0 and 1 rows (a generation in which no / one game finished) round-trip too."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "alphazero-othello_amd"))
    from dist_replay import pack_rows, unpack_rows

    for n in (0, 1, 2):
        s = _rows(3, n)
        got = unpack_rows(pack_rows(s, "cpu"))
        assert (got["own"].numpy().view(np.uint64) == s["own"]).all()
        assert (got["opp"].numpy().view(np.uint64) == s["opp"]).all()
        assert np.array_equal(got["pi"].numpy(), s["pi"])
        assert np.array_equal(got["z"].numpy(), s["z"])
        assert np.array_equal(got["player"].numpy(), s["player"])


def _bench_stats_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # [moves, games_done, sims, plies_total, games_total, window_s] of this rank
    mine = [[10, 1, 4000, 600, 10, 2.0], [12, 2, 4800, 1260, 20, 2.5]][rank]
    allst = bench.gather_stats(torch.tensor(mine, dtype=torch.float64), dist, world)
    agg = bench.aggregate_stats(allst, 400)
    q.put((rank, agg, dist.get_backend(), dist.get_world_size()))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_stats_aggregation_world2():
    """bench.py's whole-job value over a world-2 gloo group: counts summed over ranks, the
    slowest rank's window, plies per game over every rank's completed games."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bench_stats_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    want_ppg = (600 + 1260) / (10 + 20)
    want = (4000 + 4800) / 400 / want_ppg / 2.5
    for rank, agg, backend, world in res:
        assert backend == "gloo" and world == 2
        assert agg["sims"] == 8800 and agg["moves"] == 22 and agg["window_s"] == 2.5
        assert agg["plies_per_game"] == want_ppg
        assert abs(agg["value"] - want) < 1e-12
        assert [r["sims"] for r in agg["per_rank"]] == [4000, 4800]
        assert [r["window_s"] for r in agg["per_rank"]] == [2.0, 2.5]


def test_bench_stats_fallback_plies_and_cpu_calibration_gate():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    # fewer than 16 completed games: the reference's 60 plies per game
    agg = bench.aggregate_stats(np.array([[5, 0, 1000, 100, 2, 1.0]]), 100)
    assert agg["plies_per_game"] == bench.REF_PLIES_PER_GAME
    assert abs(agg["value"] - 1000 / 100 / 60 / 1.0) < 1e-12
    cal = {"net": "az5x128", "sims": 400, "cpu_model": "X", "os_cpu_count": 8,
           "ratio_reference_over_port": 0.5}
    assert bench.calibration_for(cal, "az5x128", 400, "X", 8) == 0.5
    assert bench.calibration_for(cal, "az5x128", 400, "Y", 8) is None   # other CPU model
    assert bench.calibration_for(cal, "az5x128", 400, "X", 256) is None  # other CPU count
    assert bench.calibration_for(cal, "fast", 400, "X", 8) is None
    assert 1 <= bench.host_cpu_share() <= (os.cpu_count() or 1)


def _collect_worker(rank, world, port, q, num_games):
    """self_play_worker.collect_self_play_games under a world-`world` gloo group, the GPU
    games replaced by synthetic engine rows (7 rows per game, tagged by rank and stream)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "alphazero-othello_amd"))
    import self_play_worker as spw
    from Models import FastOthelloNet

    calls = []

    def fake_local_rows(policy, args, n, n_slots, seed, stream_id, d4, dtype, pipelines=1):
        calls.append((n, stream_id, float(policy.fc_value2.weight.sum())))
        return _rows(100 * rank + stream_id, 7 * n)

    spw._local_rows = fake_local_rows
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(rank)  # different weights per rank until the broadcast
    out = spw.collect_self_play_games(FastOthelloNet(8, 65), {"num_simulations": 4}, num_games,
                                      stream_id=10)
    q.put((rank, calls, [(s.copy(), pi.copy(), z) for s, pi, z in out]))
    dist.barrier()
    dist.destroy_process_group()


def test_collect_self_play_games_world2():
    """One generation over two ranks: games split 3 / 2, stream_id + rank, rank 0's weights on
    both ranks, and every rank returning the same pooled tuples in rank order (SURVEY.md
    8(e); reference train.py:199-225)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "alphazero-othello_amd"))
    from self_play_worker import _rows_to_tuples

    world, num_games = 2, 5
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_collect_worker, args=(r, world, port, q, num_games))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    (_, c0, out0), (_, c1, out1) = res
    assert [c[:2] for c in c0] == [(3, 10)] and [c[:2] for c in c1] == [(2, 11)]
    assert c0[0][2] == c1[0][2]  # the broadcast best net on both ranks
    want = _rows_to_tuples({k: np.concatenate([_rows(10, 21)[k], _rows(111, 14)[k]])
                            for k in ("own", "opp", "pi", "z")})
    assert len(out0) == len(out1) == len(want) == 35
    for a, b, w in zip(out0, out1, want):
        for x, y, v in zip(a, b, w):
            assert np.array_equal(x, v) and np.array_equal(y, v)
