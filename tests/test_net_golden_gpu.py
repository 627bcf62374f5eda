"""The HIP leaf-evaluation path against the REFERENCE's nets (tests/golden/net_outputs.npz,
from /root/reference/Models.py via tests/golden/make_net_goldens.py).

The reference's state_dicts load strictly into this repo's modules; `inference_copy`'s
default path (fp16x2 Winograd trunk: the persistent trunk with the heads fused at up to
4 x CUs boards, chunked above) and FastOthelloNet's trunk then reproduce the reference's
softmax priors and tanh values on the fixture's 1,024 canonical boards.

Tolerance (fp32 with a different summation order): atol 1e-5, rtol 1e-4 -- the bar the
repo's own module is held to.  configs[4]'s fp16 trunk (fp16 operands, fp32 accumulation):
atol 2e-3, rtol 2e-2."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from Models import AlphaZeroNet, FastOthelloNet, FusedInferenceNet, inference_copy  # noqa: E402

NETS = {"az": lambda: AlphaZeroNet(8, 65, 5, 128), "fast": lambda: FastOthelloNet(8, 65)}


@pytest.fixture(scope="module")
def fx():
    return load_golden("net_outputs.npz")


def golden_net(kind, fx):
    net = NETS[kind]()
    pre = f"{kind}/sd/"
    sd = {k[len(pre):]: torch.from_numpy(v) for k, v in fx.items() if k.startswith(pre)}
    net.load_state_dict(sd, strict=True)
    return net.cuda().eval()


def _run(fused, canon, B):
    reps = -(-B // len(canon))
    x = torch.from_numpy(np.tile(canon.reshape(-1, 64), (reps, 1))[:B].astype(np.float32)).cuda()
    pr = torch.full((B, 65), float("nan"), device="cuda")
    va = torch.full((B,), float("nan"), device="cuda")
    with torch.no_grad():
        fused.evaluate_into(x, pr, va)
    torch.cuda.synchronize()
    return pr.cpu().numpy(), va.cpu().numpy()


def _want(fx, kind, B):
    reps = -(-B // 1024)
    return (np.tile(fx[f"{kind}/priors"], (reps, 1))[:B], np.tile(fx[f"{kind}/values"], reps)[:B])


@pytest.mark.parametrize("B", [257, 1024, 4096])
def test_az_default_path_matches_reference(B, fx):
    fused = inference_copy(golden_net("az", fx), "cuda")
    assert fused.precision == "fp16x2"
    if B <= 1024:  # the persistent trunk with the heads in its last conv (the bench's path)
        assert fused.fuse_trunk4 and fused.trunk_heads
    p, v = _run(fused, fx["canon"], B)
    wp, wv = _want(fx, "az", B)
    np.testing.assert_allclose(p, wp, atol=1e-5, rtol=1e-4)
    np.testing.assert_allclose(v, wv, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("B", [1, 8, 33])
def test_az_split_conv_path_matches_reference(B, fx):
    """The drop-in MCTS's batch sizes (1-8 leaves): the channel-split conv forms."""
    fused = inference_copy(golden_net("az", fx), "cuda")
    assert FusedInferenceNet.splitk_for(B) > 0
    p, v = _run(fused, fx["canon"], B)
    wp, wv = _want(fx, "az", B)
    np.testing.assert_allclose(p, wp, atol=1e-5, rtol=1e-4)
    np.testing.assert_allclose(v, wv, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("B", [257, 1024, 4096])
def test_fast_default_path_matches_reference(B, fx):
    fused = inference_copy(golden_net("fast", fx), "cuda")
    p, v = _run(fused, fx["canon"], B)
    wp, wv = _want(fx, "fast", B)
    np.testing.assert_allclose(p, wp, atol=1e-5, rtol=1e-4)
    np.testing.assert_allclose(v, wv, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("kind", ["az", "fast"])
def test_fp16_trunk_matches_reference(kind, fx):
    """configs[4]'s fp16 net inference (stated looser bound: atol 2e-3, rtol 2e-2)."""
    fused = inference_copy(golden_net(kind, fx), "cuda", dtype=torch.float16)
    assert fused.precision == "fp16"
    p, v = _run(fused, fx["canon"], 1024)
    wp, wv = _want(fx, kind, 1024)
    np.testing.assert_allclose(p, wp, atol=2e-3, rtol=2e-2)
    np.testing.assert_allclose(v, wv, atol=2e-3, rtol=2e-2)


@pytest.mark.parametrize("kind", ["az", "fast"])
def test_fused_batch1_inference_matches_reference(kind, fx):
    """`Inference.inference(state, player)` (reference Models.py:9-31) on the HIP copy."""
    fused = inference_copy(golden_net(kind, fx), "cuda")
    for s, p, pol, val in zip(fx["inf_states"], fx["inf_players"], fx[f"{kind}/inf_policy"],
                              fx[f"{kind}/inf_value"]):
        pi, v = fused.inference(s, int(p))
        np.testing.assert_allclose(pi, pol, atol=1e-5, rtol=1e-4)
        assert abs(v - val) <= 1e-5 + 1e-4 * abs(val)


@pytest.mark.parametrize("B", [257, 1024, 4096])
def test_fp16_persistent_trunk(B, fx, monkeypatch):
    """configs[4]'s fp16 net on the fp16 wino4 convs (conv_algo="wino4"): the stem, tower and
    heads as one persistent launch per resident chunk (az_trunk_wino4_heads_fp16_gpu) against
    the per-layer fp16 wino4 launches + the separate heads kernel, bit for bit (repeated
    launches), and against the reference's nets at configs[4]'s stated bound."""
    fused = inference_copy(golden_net("az", fx), "cuda", dtype=torch.float16, conv_algo="wino4")
    assert fused.precision == "fp16" and all(c.algo == "wino4" for c in fused.c1)
    assert fused._trunk4_fp16_ready(list(fused.c1), list(fused.c2))
    monkeypatch.setattr(FusedInferenceNet, "trunk_fp16", False)
    lp, lv = _run(fused, fx["canon"], B)
    monkeypatch.setattr(FusedInferenceNet, "trunk_fp16", True)
    for _ in range(3):
        p, v = _run(fused, fx["canon"], B)
        assert np.array_equal(p, lp) and np.array_equal(v, lv)
    wp, wv = _want(fx, "az", B)
    np.testing.assert_allclose(p, wp, atol=2e-3, rtol=2e-2)
    np.testing.assert_allclose(v, wv, atol=2e-3, rtol=2e-2)


@pytest.mark.parametrize("B", [1, 33, 4096])
def test_fast_fused_heads(B, fx, monkeypatch):
    """FastOthelloNet's heads as one GEMM on the NHWC tail output + az_heads_fast_finish_gpu
    (bench --workload c2's path) against the module's own heads (flattening copy, three
    GEMMs, softmax / ReLU / tanh) and the reference's nets."""
    fused = inference_copy(golden_net("fast", fx), "cuda")
    assert fused._fast_heads_ready()
    monkeypatch.setattr(FusedInferenceNet, "fuse_fast_heads", False)
    up, uv = _run(fused, fx["canon"], B)
    monkeypatch.setattr(FusedInferenceNet, "fuse_fast_heads", True)
    p, v = _run(fused, fx["canon"], B)
    assert np.isfinite(p).all() and np.isfinite(v).all()
    np.testing.assert_allclose(p, up, atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(v, uv, atol=1e-6, rtol=1e-5)
    wp, wv = _want(fx, "fast", B)
    np.testing.assert_allclose(p, wp, atol=1e-5, rtol=1e-4)
    np.testing.assert_allclose(v, wv, atol=1e-5, rtol=1e-4)
