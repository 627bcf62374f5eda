"""This repo's Models.py against the REFERENCE's nets (tests/golden/net_outputs.npz, made by
tests/golden/make_net_goldens.py from /root/reference/Models.py): the state_dict loads
strictly (same keys and shapes), the same seed builds the same parameters (same module
construction order), and the plain-PyTorch forward and batch-1 `Inference.inference`
reproduce the reference's outputs on CPU.  The HIP inference path is held to the same
fixture in tests/test_net_golden_gpu.py."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from Models import AlphaZeroNet, FastOthelloNet

NETS = {"az": (lambda: AlphaZeroNet(8, 65, 5, 128), 5), "fast": (lambda: FastOthelloNet(8, 65), 6)}


def golden_net(kind, fx):
    make, _ = NETS[kind]
    net = make()
    pre = f"{kind}/sd/"
    sd = {k[len(pre):]: torch.from_numpy(v) for k, v in fx.items() if k.startswith(pre)}
    net.load_state_dict(sd, strict=True)
    return net.eval()


@pytest.fixture(scope="module")
def fx():
    return load_golden("net_outputs.npz")


@pytest.mark.parametrize("kind", ["az", "fast"])
def test_state_dict_keys_and_init_match_reference(kind, fx):
    make, seed = NETS[kind]
    torch.manual_seed(seed)
    net = make()
    pre = f"{kind}/sd/"
    ref_keys = sorted(k[len(pre):] for k in fx if k.startswith(pre))
    assert sorted(net.state_dict().keys()) == ref_keys
    # conv / linear parameters come out of the same seeded init (BatchNorm tensors were
    # randomised after construction in the generator)
    for k, v in net.state_dict().items():
        ref = fx[pre + k]
        assert tuple(v.shape) == ref.shape, k
        if "bn" not in k and not k.startswith(("initial_conv.1", "conv_add.1")):
            assert np.array_equal(v.numpy(), ref), k


@pytest.mark.parametrize("kind", ["az", "fast"])
def test_module_forward_matches_reference(kind, fx):
    torch.set_num_threads(min(8, torch.get_num_threads()))
    net = golden_net(kind, fx)
    x = torch.from_numpy(fx["canon"].astype(np.float32)).unsqueeze(1)
    with torch.no_grad():
        logits, v = net(x)
    np.testing.assert_allclose(torch.softmax(logits, -1).numpy(), fx[f"{kind}/priors"],
                               atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(v.reshape(-1).numpy(), fx[f"{kind}/values"], atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("kind", ["az", "fast"])
def test_batch1_inference_matches_reference(kind, fx):
    net = golden_net(kind, fx)
    for s, p, pol, val in zip(fx["inf_states"], fx["inf_players"], fx[f"{kind}/inf_policy"],
                              fx[f"{kind}/inf_value"]):
        pi, v = net.inference(s, int(p))
        assert pi.dtype == np.float32 and pi.shape == (65,)
        assert isinstance(v, float)
        np.testing.assert_allclose(pi, pol, atol=1e-6, rtol=1e-5)
        assert abs(v - val) <= 1e-6 + 1e-5 * abs(val)
