"""The leaf-evaluation net's device kernels against a plain PyTorch fp32 reference of the
same op: the fused MFMA 3x3 conv (bias / residual / ReLU epilogue), the stem, the conv
epilogue kernel, and the whole inference copy against the reference-layout module
(Models.py).  Tolerance: fp32 with a different summation order, |d| <= 2e-5 + 2e-5 |ref|."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from Models import AlphaZeroNet, FastOthelloNet, inference_copy  # noqa: E402

TOL = dict(atol=2e-5, rtol=2e-5)


@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("B", [1, 3, 64])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_conv3x3_kernel_matches_torch(C, B, res, relu):
    g = torch.Generator().manual_seed(C * 7 + B)
    x = torch.randn(B, C, 8, 8, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).cuda()
    b = torch.randn(C, generator=g).cuda()
    r = torch.randn(B, C, 8, 8, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    ref = F.conv2d(x.contiguous(), w, b, padding=1)
    if res:
        ref = ref + r
    if relu:
        ref = F.relu(ref)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    y = torch.empty_like(x, memory_format=torch.channels_last)
    nat.check(nat.lib.az_conv3x3_gpu(nat.ptr(x), nat.ptr(w9), nat.ptr(b),
                                     nat.ptr(r) if res else None, nat.ptr(y), B, C, int(relu),
                                     nat.stream_ptr()), "az_conv3x3_gpu")
    torch.cuda.synchronize()
    torch.testing.assert_close(y, ref, **TOL)


@pytest.mark.parametrize("C", [64, 128])
def test_stem_kernel_matches_torch(C):
    g = torch.Generator().manual_seed(C)
    planes = torch.randint(-1, 2, (37, 64), generator=g).float().cuda()
    w = torch.randn(C, 1, 3, 3, generator=g).cuda()
    b = torch.randn(C, generator=g).cuda()
    ref = F.relu(F.conv2d(planes.view(-1, 1, 8, 8), w, b, padding=1))
    y = torch.empty(37, C, 8, 8, device="cuda", memory_format=torch.channels_last)
    w9 = w.reshape(C, 9).t().contiguous()
    nat.check(nat.lib.az_conv_stem_gpu(nat.ptr(planes), nat.ptr(w9), nat.ptr(b), nat.ptr(y), 37,
                                       C, nat.stream_ptr()), "az_conv_stem_gpu")
    torch.cuda.synchronize()
    torch.testing.assert_close(y, ref, **TOL)


def test_bias_act_kernel_matches_torch():
    y0 = torch.randn(5, 64, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(y0).contiguous(memory_format=torch.channels_last)
    b = torch.randn(64, device="cuda")
    for res in (None, r):
        y = y0.clone()
        nat.check(nat.lib.az_bias_act_gpu(nat.ptr(y), nat.ptr(b), None if res is None else nat.ptr(res),
                                          y.numel(), 64, 1, nat.stream_ptr()), "az_bias_act_gpu")
        ref = F.relu(y0 + b.view(1, -1, 1, 1) + (0 if res is None else res))
        torch.cuda.synchronize()
        assert torch.equal(y, ref)


@pytest.mark.parametrize("kind", ["az", "fast"])
@pytest.mark.parametrize("conv", ["hip", "miopen"])
def test_inference_copy_matches_module(kind, conv):
    torch.manual_seed(0)
    net = AlphaZeroNet(8, 65, 5, 128) if kind == "az" else FastOthelloNet(8, 65)
    # non-trivial BatchNorm statistics so the folding is exercised
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.5, 0.5)
            m.running_var.uniform_(0.5, 2.0)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    net = net.cuda().eval()
    fused = inference_copy(net, "cuda", conv=conv)
    x = torch.randint(-1, 2, (257, 64), device="cuda").float()
    with torch.no_grad():
        logits, v = net(x.view(-1, 1, 8, 8))
        p_ref = torch.softmax(logits, -1)
        p, val = fused.evaluate_planes(x)
    torch.testing.assert_close(p, p_ref, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(val, v.reshape(-1), atol=1e-5, rtol=1e-4)
