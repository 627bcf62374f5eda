"""Replay-buffer aggregation on the GPU (csrc/replay.hip) against the reference's
Trainer._aggregate_duplicates: the reference-generated fixture bit for bit (order included),
larger synthetic buffers against the oracle restatement (oracle/replay.py), edge sizes."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import replay as oracle_replay

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
import replay  # noqa: E402

W = np.uint64(1) << np.arange(64, dtype=np.uint64)


def boards(pos, neg):
    b = np.zeros((len(pos), 64), np.int8)
    b[(pos[:, None] & W) != 0] = 1
    b[(neg[:, None] & W) != 0] = -1
    return b.reshape(-1, 8, 8)


def test_aggregate_duplicates_matches_reference_fixture():
    d = load_golden("replay_aggregate.npz")
    buf = [(s, p, float(v), int(ver)) for s, p, v, ver in
           zip(boards(d["in_pos"], d["in_neg"]), d["in_pi"], d["in_v"], d["in_ver"])]
    states, pis, vs = replay.aggregate_duplicates(buf)
    assert len(states) == len(d["out_pos"])
    ref_states = boards(d["out_pos"], d["out_neg"])
    for i in range(len(states)):
        assert np.array_equal(states[i], ref_states[i])
    assert np.array_equal(np.stack(pis), d["out_pi"])
    assert np.array_equal(np.array(vs, np.float32), d["out_v"])
    assert all(isinstance(x, np.float32) for x in vs)


@pytest.mark.parametrize("n,pool,versions", [(0, 1, 1), (1, 1, 1), (7, 1, 1), (50000, 500, 3),
                                             (200000, 20000, 2)])
def test_aggregate_rows_matches_oracle(n, pool, versions):
    rng = np.random.default_rng(n + pool)
    keys_own = rng.integers(0, 2**63, pool, dtype=np.int64).astype(np.uint64)
    keys_opp = rng.integers(0, 2**63, pool, dtype=np.int64).astype(np.uint64) & ~keys_own
    k = (rng.zipf(1.5, n) - 1) % pool if n else np.zeros(0, np.int64)
    own, opp = keys_own[k], keys_opp[k]
    ver = rng.integers(0, versions, n).astype(np.int32)
    pi = rng.random((n, 65)).astype(np.float32)
    pi /= pi.sum(1, keepdims=True)
    v = rng.uniform(-1, 1, n)
    dev = torch.device("cuda")
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(device=dev, dtype=dt)  # noqa: E731
    got = replay.aggregate_rows(t(own.view(np.int64), torch.int64), t(opp.view(np.int64), torch.int64),
                                t(ver, torch.int32), t(pi, torch.float32), t(v, torch.float64))
    r_own, r_opp, r_ver, r_pi, r_v, r_cnt = oracle_replay.aggregate(own, opp, ver, pi, v)
    assert (got["own"].cpu().numpy().view(np.uint64) == r_own).all()
    assert (got["opp"].cpu().numpy().view(np.uint64) == r_opp).all()
    assert (got["ver"].cpu().numpy() == r_ver).all()
    assert np.array_equal(got["pi"].cpu().numpy(), r_pi)
    assert np.array_equal(got["v"].cpu().numpy(), r_v)
    assert (got["count"].cpu().numpy() == r_cnt).all()
