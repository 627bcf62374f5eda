"""Training-side GPU path (train_gpu.py): the D4 augmentation against the reference's
get_random_symmetry fixture (bit-exact for the drawn (k, flip)), the device loader's batch
contract, and one train_iters pass of AlphaZeroNet on device batches."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
import train_gpu  # noqa: E402
from Models import AlphaZeroNet  # noqa: E402


def test_augment_matches_reference_fixture():
    d = load_golden("augment.npz")
    dev = torch.device("cuda")
    own = torch.from_numpy(d["pos"].view(np.int64)).to(dev)
    opp = torch.from_numpy(d["neg"].view(np.int64)).to(dev)
    sym = torch.from_numpy((d["k"] + 4 * d["flip"]).astype(np.int64)).to(dev)
    s, p = train_gpu.augment(own, opp, torch.from_numpy(d["pi"]).to(dev), sym)
    assert np.array_equal(s.cpu().numpy(), d["out_state"])
    assert np.array_equal(p.cpu().numpy(), d["out_pi"])


def test_loader_and_train_iters():
    rng = np.random.default_rng(0)
    d = load_golden("augment.npz")
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    states = [(((d["pos"][i] & w) != 0).astype(np.float32) - ((d["neg"][i] & w) != 0)).reshape(8, 8)
              for i in range(len(d["pos"]))]
    values = rng.uniform(-1, 1, len(states)).astype(np.float32)
    loader = train_gpu.DeviceReplayLoader(states, list(d["pi"]), values, batch_size=96, seed=3)
    seen = 0
    for s, p, v in loader:
        assert s.shape[1:] == (1, 8, 8) and p.shape[1] == 65 and v.shape[1] == 1
        assert torch.allclose(p.sum(1), torch.ones_like(p[:, 0]), atol=1e-5)
        assert ((s == 0) | (s == 1) | (s == -1)).all()
        seen += s.shape[0]
    assert seen == len(states) and len(loader) == (len(states) + 95) // 96
    torch.manual_seed(0)
    net = AlphaZeroNet(8, 65, 2, 32).cuda()
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    first = train_gpu.train_iters(net, opt, loader, 0.01)
    for _ in range(5):
        last = train_gpu.train_iters(net, opt, loader, 0.01)
    assert all(np.isfinite(first)) and last[0] + last[1] < first[0] + first[1]
