"""one_self_play's shared generation through a real spawn pool (train.py:199-225's shape):
three workers, num_self_play = 6 in the args; one worker plays the six games on the GPU
engine, every call returns one of them, each exactly once, equal to the engine's games for
the seed the producer draws from np.random (every worker seeded alike here)."""
import os
import pathlib
import shutil
import sys
import uuid
from multiprocessing import get_context

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]

pytestmark = pytest.mark.gpu


@pytest.fixture
def scratch():
    """A fresh directory under tests/_scratch/ (inside the checkout), removed afterwards."""
    d = os.path.join(ROOT, "tests", "_scratch", uuid.uuid4().hex)
    os.makedirs(d)
    yield pathlib.Path(d)
    shutil.rmtree(d, ignore_errors=True)


ARGS = {"c_puct": 2.0, "num_simulations": 6, "dirichlet_alpha": 1.0, "dirichlet_epsilon": 0.3,
        "mcts_temperature": 1.0, "num_exploratory_moves": 35, "lambda": 0.98,
        "num_self_play": 6, "num_workers": 3}


def _seed_worker():
    np.random.seed(99)


def _net():
    from Models import FastOthelloNet

    torch.manual_seed(0)
    return FastOthelloNet(8, 65)


def test_shared_generation_through_spawn_pool(scratch, monkeypatch):
    import self_play_worker as spw
    from Models import FastOthelloNet

    monkeypatch.setenv("AZ_DROPIN_DIR", str(scratch / "gen"))
    net = _net()
    ps = (FastOthelloNet, net.get_config(), net.state_dict())
    items = [(8, ARGS, ps, None)] * ARGS["num_self_play"]
    with get_context("spawn").Pool(3, initializer=_seed_worker) as pool:
        got = list(pool.imap_unordered(spw.one_self_play, items, chunksize=1))
    np.random.seed(99)
    seed = int(np.random.randint(0, 2**31 - 1))
    want = spw._games_from_rows(spw._local_rows(net, ARGS, 6, None, seed, 0, False,
                                                torch.float32))
    assert len(got) == len(want) == 6

    def sig(g):
        return tuple((s.tobytes(), pi.tobytes(), z) for s, pi, z in g)

    assert sorted(map(sig, got)) == sorted(map(sig, want))  # each game exactly once
    for g in got:
        s0 = g[0][0]
        assert (s0 != 0).sum() == 4 and len(g) >= 10
    assert not os.path.exists(scratch / "gen" / spw._batch_key(8, ARGS, ps)[:40])
