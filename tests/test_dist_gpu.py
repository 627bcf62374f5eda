"""One self-play generation over two ranks with REAL engines (reference train.py:199-225,
SURVEY.md 8(e)): `collect_self_play_games` under a world-2 gloo group, both ranks' engines
on cuda:0.  Everything of the N > 1 path runs except RCCL itself: the best net's weights
broadcast from rank 0 (each rank starts from different weights), rank r's share of the
games on Philox stream stream_id + r, and one all-gather of the finished rows.

Bar: every rank returns the same pooled tuples, and they are exactly two standalone
single-process generations (stream 0's games, then stream 1's) on rank 0's net -- rows bit
for bit (compared as multisets within a rank: the engine's sample ring records finishing
slots in completion order)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ARGS = {"c_puct": 2.0, "num_simulations": 8, "num_threads": 4, "dirichlet_alpha": 1.0,
        "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
        "lambda": 0.98}
GAMES = 7  # rank 0 plays 4, rank 1 plays 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _key(t):
    s, pi, z = t
    return s.astype(np.int8).tobytes() + pi.astype(np.float32).tobytes() + np.float64(z).tobytes()


def _worker(rank, world, port, q):
    import sys
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "alphazero-othello_amd"))
    import self_play_worker as spw
    from Models import FastOthelloNet

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(rank)  # rank 1 starts from other weights: the broadcast must fix it
        net = FastOthelloNet(8, 65).cuda().eval()
        out = spw.collect_self_play_games(net, ARGS, GAMES, stream_id=0)
        q.put((rank, [(s.copy(), pi.copy(), float(z)) for s, pi, z in out], None))
        dist.barrier()
    except Exception as ex:  # report instead of hanging the parent's queue
        q.put((rank, None, repr(ex)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_collect_self_play_games_world2_real_engines():
    import self_play_worker as spw
    from Models import FastOthelloNet

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=500) for _ in range(2)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
    errs = [e for _, _, e in res if e]
    assert not errs, errs
    assert all(p.exitcode == 0 for p in ps)
    out0, out1 = res[0][1], res[1][1]

    # the same generation as two standalone single-process runs on rank 0's net
    torch.manual_seed(0)
    net = FastOthelloNet(8, 65).cuda().eval()
    want = []
    for r in range(2):
        n = GAMES // 2 + (1 if r < GAMES % 2 else 0)
        rows = spw._local_rows(net, ARGS, n, None, 0, r, False, torch.float32)
        want.append(spw._rows_to_tuples(rows))
    n0 = len(want[0])
    assert len(out0) == len(out1) == n0 + len(want[1])
    for a, b in zip(out0, out1):  # every rank holds the same pooled list
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x), np.asarray(y))
    for got, w in ((out0[:n0], want[0]), (out0[n0:], want[1])):  # rank 0's games first
        assert sorted(map(_key, got)) == sorted(map(_key, w))
    assert sorted(map(_key, want[0])) != sorted(map(_key, want[1]))  # distinct streams
