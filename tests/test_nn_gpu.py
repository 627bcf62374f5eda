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
    # the absmax-fused entry: same output bit for bit, plus each board's exact max |y|
    y2 = torch.empty_like(y, memory_format=torch.channels_last)
    amax = torch.full((37,), -1.0, device="cuda")
    nat.check(nat.lib.az_conv_stem2_gpu(nat.ptr(planes), nat.ptr(w9), nat.ptr(b), nat.ptr(y2), 37,
                                        C, nat.ptr(amax), nat.stream_ptr()), "az_conv_stem2_gpu")
    torch.cuda.synchronize()
    assert torch.equal(y2, y)
    assert torch.equal(amax, y.abs().amax(dim=(1, 2, 3)))


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
@pytest.mark.parametrize("conv,precision,algo", [("hip", "split3", "wino"), ("hip", "split3", "wino4"),
                                                 ("hip", "fp16x2", None),
                                                 ("hip", "split3", "direct"),
                                                 ("hip", "fp32", None), ("miopen", None, None)])
def test_inference_copy_matches_module(kind, conv, precision, algo):
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
    fused = inference_copy(net, "cuda", conv=conv, precision=precision, conv_algo=algo)
    if algo is not None:
        want = "wino" if algo == "wino4" and kind == "fast" else algo  # wino4: 128 channels
        assert all(c.algo == want for c in list(fused.c1) + list(fused.c2))
    x = torch.randint(-1, 2, (257, 64), device="cuda").float()
    with torch.no_grad():
        logits, v = net(x.view(-1, 1, 8, 8))
        p_ref = torch.softmax(logits, -1)
        p, val = fused.evaluate_planes(x)
    torch.testing.assert_close(p, p_ref, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(val, v.reshape(-1), atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("B", [1, 4, 9, 33, 257])
def test_inference_copy_fp16x2_small_batches(B):
    """The default fp32 inference copy (fp16x2 trunk) at a search's batch sizes: up to 8 boards
    the trunk runs the 16-way split conv (channels x transform rows), up to 32 the 8-way
    channel split, up to 256 the 4-way one, above it the one-pass kernel; all match the
    module at the fp32 tolerance."""
    from Models import FusedInferenceNet

    torch.manual_seed(1)
    net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
    fused = inference_copy(net, "cuda")
    assert fused.precision == "fp16x2"
    x = torch.randint(-1, 2, (B, 64), device="cuda").float()
    with torch.no_grad():
        logits, v = net(x.view(-1, 1, 8, 8))
        p, val = fused.evaluate_planes(x)
    splits = FusedInferenceNet.splitk_for(B)
    assert splits == (16 if B <= 8 else 8 if B <= 32 else 4 if B <= 256 else 0)
    part = fused._trunk_scratch[(x.device, B)].get("part")
    assert (part is not None) == bool(splits)
    if splits:
        assert part.numel() == splits * B * 64 * 128
    # another batch size gets its own scratch: a graph captured at B keeps valid pointers
    with torch.no_grad():
        fused.evaluate_planes(torch.zeros(B + 3, 64, device="cuda"))
    assert fused._trunk_scratch[(x.device, B)].get("part") is part
    torch.testing.assert_close(p, torch.softmax(logits, -1), atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(val, v.reshape(-1), atol=1e-5, rtol=1e-4)


def _mx_conv(x, w, b, r, relu, mode):
    C = x.shape[1]
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    wq = torch.empty(nat.lib.az_conv3x3_mx_prep_bytes(C, mode) // 2, dtype=torch.int16,
                     device="cuda")
    nat.check(nat.lib.az_conv3x3_mx_prep_gpu(nat.ptr(w9), nat.ptr(wq), C, mode, nat.stream_ptr()),
              "az_conv3x3_mx_prep_gpu")
    y = torch.empty_like(x, memory_format=torch.channels_last)
    nat.check(nat.lib.az_conv3x3_mx_gpu(nat.ptr(x), nat.ptr(wq), nat.ptr(b),
                                        None if r is None else nat.ptr(r), nat.ptr(y), x.shape[0],
                                        C, int(relu), mode, nat.stream_ptr()), "az_conv3x3_mx_gpu")
    torch.cuda.synchronize()
    return y


def _wino_conv(x, w, b, r, relu, mode, fn="az_conv3x3_wino_gpu", out_absmax=None, splits=0,
               in_absmax=None):
    C = x.shape[1]
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    wq = torch.empty(nat.lib.az_conv3x3_wino_prep_bytes(C, mode) // 2, dtype=torch.int16,
                     device="cuda")
    nat.check(nat.lib.az_conv3x3_wino_prep_gpu(nat.ptr(w9), nat.ptr(wq), C, mode,
                                               nat.stream_ptr()), "az_conv3x3_wino_prep_gpu")
    y = torch.empty_like(x, memory_format=torch.channels_last)
    args = [nat.ptr(x), nat.ptr(wq), nat.ptr(b), None if r is None else nat.ptr(r), nat.ptr(y),
            x.shape[0], C, int(relu), mode]
    if fn == "az_conv3x3_wino4_gpu":
        from Models import board_absmax

        if in_absmax is None:
            in_absmax = board_absmax(x)
        args += [nat.ptr(in_absmax), nat.ptr(out_absmax)]
        if splits:
            fn = "az_conv3x3_wino4_splitk_gpu"
            part = torch.full((splits * x.numel(),), float("nan"), device="cuda")
            args += [nat.ptr(part), splits]
    nat.check(getattr(nat.lib, fn)(*args, nat.stream_ptr()), fn)
    torch.cuda.synchronize()
    return y


def _case(C, B, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, C, 8, 8, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)
    b = torch.randn(C, generator=g)
    r = torch.randn(B, C, 8, 8, generator=g)
    cl = lambda t: t.cuda().contiguous(memory_format=torch.channels_last)
    ref64 = F.conv2d(x.double(), w.double(), b.double(), padding=1)
    return cl(x), w.cuda(), b.cuda(), cl(r), ref64


@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("B", [1, 3, 130])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_conv3x3_split3_is_fp32_accurate(C, B, res, relu):
    """The bf16x3-split MFMA conv against an fp64 reference: its error must stay at the fp32
    MFMA kernel's level (max |err| <= 2x the fp32 kernel's + 1e-6, mean <= 2x), and within
    the fp32 tolerance of this file against torch fp32."""
    x, w, b, r, ref64 = _case(C, B, C * 13 + B)
    rr = r if res else None
    y = _mx_conv(x, w, b, rr, relu, nat.AZ_CONV_SPLIT3)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    y32 = torch.empty_like(x, memory_format=torch.channels_last)
    nat.check(nat.lib.az_conv3x3_gpu(nat.ptr(x), nat.ptr(w9), nat.ptr(b), None if rr is None else nat.ptr(rr),
                                     nat.ptr(y32), B, C, int(relu), nat.stream_ptr()), "az_conv3x3_gpu")
    torch.cuda.synchronize()
    ref = ref64 + (r.cpu().double() if res else 0)
    if relu:
        ref = F.relu(ref)
    e_mx = (y.cpu().double() - ref).abs()
    e_32 = (y32.cpu().double() - ref).abs()
    assert e_mx.max() <= 2 * e_32.max() + 1e-6, (e_mx.max(), e_32.max())
    assert e_mx.mean() <= 2 * e_32.mean() + 1e-8, (e_mx.mean(), e_32.mean())
    torch.testing.assert_close(y, ref.float().cuda(), **TOL)


@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("B", [1, 3, 130])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_conv3x3_direct_fp16x2_is_fp32_accurate(C, B, res, relu):
    """The direct kernel's FP16X2 mode (csrc/conv16.hip: fp16 hi + lo operand pairs after
    exact power-of-two scaling -- the weights per layer, each board by the max |x| its
    workgroup stages -- three products; FastOthelloNet's 64-channel convs) against fp64: the
    fp32-accuracy bar of the split3 kernels (max |err| <= 2x the fp32 MFMA kernel's + 1e-6,
    mean <= 2x), boards from 1e-3 to 1e3 in one batch."""
    x, w, b, r, ref64 = _case(C, B, C * 29 + B)
    if B > 1:  # per-board ranges from 1e-3 to 1e3
        s = torch.logspace(-3, 3, B, device="cuda").view(B, 1, 1, 1)
        x = (x * s).contiguous(memory_format=torch.channels_last)
        ref64 = F.conv2d(x.cpu().double(), w.cpu().double(), b.cpu().double(), padding=1)
    rr = r if res else None
    y = _mx_conv(x, w, b, rr, relu, nat.AZ_CONV_FP16X2)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    y32 = torch.empty_like(x, memory_format=torch.channels_last)
    nat.check(nat.lib.az_conv3x3_gpu(nat.ptr(x), nat.ptr(w9), nat.ptr(b), None if rr is None else nat.ptr(rr),
                                     nat.ptr(y32), B, C, int(relu), nat.stream_ptr()), "az_conv3x3_gpu")
    torch.cuda.synchronize()
    ref = ref64 + (r.cpu().double() if res else 0)
    if relu:
        ref = F.relu(ref)
    e_h = (y.cpu().double() - ref).abs()
    e_32 = (y32.cpu().double() - ref).abs()
    assert torch.isfinite(y).all()
    assert e_h.max() <= 2 * e_32.max() + 1e-6, (e_h.max(), e_32.max())
    assert e_h.mean() <= 2 * e_32.mean() + 1e-8, (e_h.mean(), e_32.mean())
    # per board too (the global bar is set by the 1e3 boards): a board scaled by another
    # board's range would lose the lo words of its small values -- ~1e-5 on a 1e-3 board
    for bi in range(B):
        assert e_h[bi].max() <= 4 * e_32[bi].max() + 1e-7, (bi, e_h[bi].max(), e_32[bi].max())


@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("B", [1, 3, 130])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_conv3x3_winograd_is_fp32_accurate(C, B, res, relu):
    """Winograd F(2x2,3x3) with split3 operands against fp64: the same bar as the direct
    split3 kernel (max |err| <= 2x the fp32 kernel's + 1e-6, mean <= 2x), odd board counts
    included (a workgroup holds two boards), and the fp32 tolerance against torch."""
    x, w, b, r, ref64 = _case(C, B, C * 17 + B)
    rr = r if res else None
    y = _wino_conv(x, w, b, rr, relu, nat.AZ_CONV_SPLIT3)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    y32 = torch.empty_like(x, memory_format=torch.channels_last)
    nat.check(nat.lib.az_conv3x3_gpu(nat.ptr(x), nat.ptr(w9), nat.ptr(b), None if rr is None else nat.ptr(rr),
                                     nat.ptr(y32), B, C, int(relu), nat.stream_ptr()), "az_conv3x3_gpu")
    torch.cuda.synchronize()
    ref = ref64 + (r.cpu().double() if res else 0)
    if relu:
        ref = F.relu(ref)
    e_w = (y.cpu().double() - ref).abs()
    e_32 = (y32.cpu().double() - ref).abs()
    assert e_w.max() <= 2 * e_32.max() + 1e-6, (e_w.max(), e_32.max())
    assert e_w.mean() <= 2 * e_32.mean() + 1e-8, (e_w.mean(), e_32.mean())
    torch.testing.assert_close(y, ref.float().cuda(), **TOL)


@pytest.mark.parametrize("B", [1, 3, 4, 5, 130, 1024])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_conv3x3_winograd4_is_fp32_accurate(B, res, relu):
    """The four-board Winograd form (output transform folded per transform-grid row,
    csrc/conv_wino4.hip) against fp64: the fp32-accuracy bar of the other split3 kernels,
    board counts that leave 1-3 boards in the last workgroup included."""
    C = 128
    x, w, b, r, ref64 = _case(C, B, C * 19 + B)
    rr = r if res else None
    y = _wino_conv(x, w, b, rr, relu, nat.AZ_CONV_SPLIT3, fn="az_conv3x3_wino4_gpu")
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    y32 = torch.empty_like(x, memory_format=torch.channels_last)
    nat.check(nat.lib.az_conv3x3_gpu(nat.ptr(x), nat.ptr(w9), nat.ptr(b), None if rr is None else nat.ptr(rr),
                                     nat.ptr(y32), B, C, int(relu), nat.stream_ptr()), "az_conv3x3_gpu")
    torch.cuda.synchronize()
    ref = ref64 + (r.cpu().double() if res else 0)
    if relu:
        ref = F.relu(ref)
    e_w = (y.cpu().double() - ref).abs()
    e_32 = (y32.cpu().double() - ref).abs()
    assert e_w.max() <= 2 * e_32.max() + 1e-6, (e_w.max(), e_32.max())
    assert e_w.mean() <= 2 * e_32.mean() + 1e-8, (e_w.mean(), e_32.mean())
    torch.testing.assert_close(y, ref.float().cuda(), **TOL)


@pytest.mark.parametrize("splits", [0, 2, 4, 8, 16, 32])
@pytest.mark.parametrize("B", [1, 3, 5, 130, 1024])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_conv3x3_winograd4_fp16x2_is_fp32_accurate(B, res, relu, splits):
    """FP16X2 (fp16 hi + lo operand pairs after exact power-of-two scaling, three products)
    against fp64: the same fp32-accuracy bar as split3 (max |err| <= 2x the fp32 MFMA
    kernel's + 1e-6, mean <= 2x), boards of very different magnitude in one batch included
    (the input scale is per board), and the per-board max |y| output exact.  splits = 2 / 4 /
    8 (channel chunks) or 16 / 32 (also the transform rows): the channel-split small-batch form
    (az_conv3x3_wino4_splitk_gpu), which also consumes in_absmax (reset to 0)."""
    C = 128
    x, w, b, r, ref64 = _case(C, B, C * 23 + B)
    if B > 1:  # per-board ranges from 1e-3 to 1e3
        s = torch.logspace(-3, 3, B, device="cuda").view(B, 1, 1, 1)
        x = (x * s).contiguous(memory_format=torch.channels_last)
        ref64 = F.conv2d(x.cpu().double(), w.cpu().double(), b.cpu().double(), padding=1)
    rr = r if res else None
    amax = torch.zeros(B, dtype=torch.float32, device="cuda")
    from Models import board_absmax

    in_amax = board_absmax(x)
    y = _wino_conv(x, w, b, rr, relu, nat.AZ_CONV_FP16X2, fn="az_conv3x3_wino4_gpu",
                   out_absmax=amax, splits=splits, in_absmax=in_amax)
    assert (in_amax == 0).all()
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    y32 = torch.empty_like(x, memory_format=torch.channels_last)
    nat.check(nat.lib.az_conv3x3_gpu(nat.ptr(x), nat.ptr(w9), nat.ptr(b), None if rr is None else nat.ptr(rr),
                                     nat.ptr(y32), B, C, int(relu), nat.stream_ptr()), "az_conv3x3_gpu")
    torch.cuda.synchronize()
    ref = ref64 + (r.cpu().double() if res else 0)
    if relu:
        ref = F.relu(ref)
    # the error bar is relative to each board's magnitude: normalise per board
    scale = ref.abs().amax(dim=(1, 2, 3), keepdim=True).clamp_min(1e-30)
    e_w = ((y.cpu().double() - ref).abs() / scale)
    e_32 = ((y32.cpu().double() - ref).abs() / scale)
    assert e_w.max() <= 2 * e_32.max() + 1e-7, (e_w.max(), e_32.max())
    assert e_w.mean() <= 2 * e_32.mean() + 1e-9, (e_w.mean(), e_32.mean())
    assert torch.equal(amax.cpu(), y.abs().amax(dim=(1, 2, 3)).cpu())


@pytest.mark.parametrize("splits", [4, 16])
def test_conv3x3_winograd4_splitk_is_deterministic(splits):
    """The split form adds its partials in a fixed order (no atomics on the data): two runs
    on the same inputs are bit-identical, per-board max |y| included."""
    from Models import board_absmax

    x, w, b, r, _ = _case(128, 6, 128 * 31 + splits)
    outs = []
    for _ in range(2):
        amax = torch.zeros(6, dtype=torch.float32, device="cuda")
        y = _wino_conv(x, w, b, r, True, nat.AZ_CONV_FP16X2, fn="az_conv3x3_wino4_gpu",
                       out_absmax=amax, splits=splits, in_absmax=board_absmax(x))
        outs.append((y, amax))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("mode", ["fp16x2", "fp16"])
@pytest.mark.parametrize("B", [1, 3, 130, 1030])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True)])
def test_conv3x3_winograd4_two_board_form_is_bit_identical(mode, B, res, relu, monkeypatch):
    """The default two-board workgroups (two per CU) and the four-board form
    (AZ_W4_BOARDS=4) run the same tiles with the same arithmetic: outputs and the per-board
    max |y| bit for bit, ragged last workgroups included."""
    from Models import board_absmax

    m = {"fp16x2": nat.AZ_CONV_FP16X2, "fp16": nat.AZ_CONV_FP16}[mode]
    x, w, b, r, _ = _case(128, B, 128 * 41 + B)
    if B > 1:
        s = torch.logspace(-2, 2, B, device="cuda").view(B, 1, 1, 1)
        x = (x * s).contiguous(memory_format=torch.channels_last)
    out = {}
    for boards in ("2", "4"):
        monkeypatch.setenv("AZ_W4_BOARDS", boards)
        amax = torch.zeros(B, dtype=torch.float32, device="cuda")
        y = _wino_conv(x, w, b, r if res else None, relu, m, fn="az_conv3x3_wino4_gpu",
                       out_absmax=amax, in_absmax=board_absmax(x))
        out[boards] = (y, amax)
    assert torch.equal(out["2"][0], out["4"][0])
    assert torch.equal(out["2"][1], out["4"][1])


def test_conv3x3_winograd4_fp16_mode():
    x, w, b, r, ref64 = _case(128, 37, 128 + 11)
    y = _wino_conv(x, w, b, r, True, nat.AZ_CONV_FP16, fn="az_conv3x3_wino4_gpu")
    ref = F.relu(ref64 + r.cpu().double()).float().cuda()
    torch.testing.assert_close(y, ref, atol=5e-3, rtol=5e-3)


@pytest.mark.parametrize("C", [64, 128])
def test_conv3x3_winograd_fp16_mode(C):
    x, w, b, r, ref64 = _case(C, 37, C + 9)
    y = _wino_conv(x, w, b, r, True, nat.AZ_CONV_FP16)
    ref = F.relu(ref64 + r.cpu().double()).float().cuda()
    torch.testing.assert_close(y, ref, atol=5e-3, rtol=5e-3)


@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("res", [False, True])
def test_conv3x3_fp16_mode(C, res):
    """fp16 inference (configs[4]): fp16 operands, fp32 accumulation; tolerance of fp16
    rounding of both operands over K = 9C terms."""
    x, w, b, r, ref64 = _case(C, 37, C + 5)
    y = _mx_conv(x, w, b, r if res else None, True, nat.AZ_CONV_FP16)
    ref = F.relu(ref64 + (r.cpu().double() if res else 0)).float().cuda()
    torch.testing.assert_close(y, ref, atol=5e-3, rtol=5e-3)


@pytest.mark.parametrize("kind", ["az", "fast"])
def test_inference_copy_fp16_trunk(kind):
    """config #5: fp16 trunk operands (fp32 accumulation, fp32 activations/heads) stay
    within fp16 rounding of the fp32 module."""
    torch.manual_seed(1)
    net = (AlphaZeroNet(8, 65, 5, 128) if kind == "az" else FastOthelloNet(8, 65)).cuda().eval()
    fused = inference_copy(net, "cuda", dtype=torch.float16)
    assert fused.precision == "fp16"
    x = torch.randint(-1, 2, (129, 64), device="cuda").float()
    with torch.no_grad():
        logits, v = net(x.view(-1, 1, 8, 8))
        p, val = fused.evaluate_planes(x)
    torch.testing.assert_close(p, torch.softmax(logits, -1), atol=2e-3, rtol=2e-2)
    torch.testing.assert_close(val, v.reshape(-1), atol=2e-3, rtol=2e-2)


@pytest.mark.parametrize("kind", ["az", "fast"])
@pytest.mark.parametrize("precision", ["split3", "fp16", "fp16x2"])
def test_stem_fusion_is_bit_identical(kind, precision):
    """The stem evaluated inside the first block's convs (az_conv3x3_mx_stem_gpu) gives the
    same trunk output bit for bit as the stem kernel + plain convs."""
    torch.manual_seed(2)
    net = (AlphaZeroNet(8, 65, 5, 128) if kind == "az" else FastOthelloNet(8, 65)).cuda().eval()
    fused = inference_copy(net, "cuda", precision=precision, conv_algo="direct")
    x = torch.randint(-1, 2, (131, 1, 8, 8), device="cuda").float()
    with torch.no_grad():
        fused.fuse_stem = True
        a = fused._trunk(x)
        fused.fuse_stem = False
        b = fused._trunk(x)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("kind", ["az", "fast"])
def test_trunk_kernel_is_bit_identical(kind):
    """az_trunk_wino_gpu (stem + every residual block in one launch, board pairs carried
    through all layers by one workgroup) gives the layer-by-layer launches' trunk output bit
    for bit, odd board count included."""
    torch.manual_seed(3)
    net = (AlphaZeroNet(8, 65, 5, 128) if kind == "az" else FastOthelloNet(8, 65)).cuda().eval()
    fused = inference_copy(net, "cuda", precision="split3", conv_algo="wino")
    x = torch.randint(-1, 2, (301, 1, 8, 8), device="cuda").float()
    with torch.no_grad():
        fused.fuse_trunk = True
        assert fused._trunk_kernel_ready()
        a = fused._trunk(x)
        fused.fuse_trunk = False
        b = fused._trunk(x)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("B", [257, 1024, 1030, 4096])
@pytest.mark.parametrize("heads", [True, False])
def test_persistent_trunk_bit_identical_to_layer_launches(B, heads, monkeypatch):
    """The fp16x2 tower as one persistent launch (az_trunk_wino4_gpu: each two-board
    workgroup carries its boards through the layers) against one launch per conv: priors
    and values (heads fused into the last conv, or the separate heads kernel after the
    whole tower) and the tower's output, bit for bit, ragged last workgroups included."""
    from Models import FusedInferenceNet

    torch.manual_seed(5)
    net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
    fused = inference_copy(net, "cuda")
    monkeypatch.setattr(FusedInferenceNet, "fuse_heads", heads)
    x = torch.randint(-1, 2, (B, 64), device="cuda").float()
    out = {}
    for flag in (True, False):
        monkeypatch.setattr(FusedInferenceNet, "fuse_trunk4", flag)
        pr = torch.full((B, 65), float("nan"), device="cuda")
        va = torch.full((B,), float("nan"), device="cuda")
        with torch.no_grad():
            fused.evaluate_into(x, pr, va)
            h = fused._trunk(x.view(B, 1, 8, 8))
        torch.cuda.synchronize()
        out[flag] = (pr, va, h)
    for a, b in zip(out[True], out[False]):
        assert torch.equal(a, b)
    assert not torch.isnan(out[True][0]).any()


@pytest.mark.parametrize("heads_boards", ["2", "4"])
@pytest.mark.parametrize("boards", ["2", "4"])
@pytest.mark.parametrize("B", [257, 1024, 1030, 4096])
def test_fused_heads_bit_identical_to_separate_heads(B, boards, heads_boards, monkeypatch):
    """AlphaZeroNet on the fp16x2 trunk: the heads fused into the last conv's epilogue
    (az_conv3x3_wino4_heads_gpu, the trunk output kept in LDS) give the same priors and
    values, bit for bit, as the last conv followed by the separate heads kernel
    (az_heads_az_gpu): heads_az.h runs the same code on the same fp32 values.  Ragged
    batches (a partial last workgroup) included, with two-board (default) and four-board
    (AZ_W4_BOARDS=4) workgroups: heads_az.h adds the FC input quarters in the same order
    for any number of boards per workgroup; the heads-fused conv itself in both forms
    (AZ_W4_HEADS_BOARDS: two-board workgroups two per CU, the default, or four-board)."""
    from Models import FusedInferenceNet

    monkeypatch.setenv("AZ_W4_BOARDS", boards)
    monkeypatch.setenv("AZ_W4_HEADS_BOARDS", heads_boards)

    torch.manual_seed(3)
    net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
    fused = inference_copy(net, "cuda")
    assert fused.precision == "fp16x2"
    x = torch.randint(-1, 2, (B, 64), device="cuda").float()
    out = {}
    for flag in (True, False):
        monkeypatch.setattr(FusedInferenceNet, "fuse_heads", flag)
        pr = torch.full((B, 65), float("nan"), device="cuda")
        va = torch.full((B,), float("nan"), device="cuda")
        with torch.no_grad():
            fused.evaluate_into(x, pr, va)
        torch.cuda.synchronize()
        out[flag] = (pr, va)
    assert torch.equal(out[True][0], out[False][0])
    assert torch.equal(out[True][1], out[False][1])
    with torch.no_grad():
        logits, v = net(x.view(-1, 1, 8, 8))
    torch.testing.assert_close(out[True][0], torch.softmax(logits, -1), atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(out[True][1], v.reshape(-1), atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("B", [1024, 1030])
def test_two_board_fused_heads_stress(B, monkeypatch):
    """Two co-resident two-board heads-fused workgroups per CU (the default last conv) over
    repeated evaluations of the persistent-trunk tower: every launch's priors and values bit
    for bit equal to the separate heads kernel's (round 3 saw a timing-dependent value
    difference on 1-6 boards per launch in an earlier two-board epilogue)."""
    from Models import FusedInferenceNet

    monkeypatch.setenv("AZ_W4_HEADS_BOARDS", "2")
    torch.manual_seed(11)
    net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
    fused = inference_copy(net, "cuda")
    x = torch.randint(-1, 2, (B, 64), device="cuda").float()
    monkeypatch.setattr(FusedInferenceNet, "fuse_heads", False)
    ref_p = torch.empty(B, 65, device="cuda")
    ref_v = torch.empty(B, device="cuda")
    with torch.no_grad():
        fused.evaluate_into(x, ref_p, ref_v)
    monkeypatch.setattr(FusedInferenceNet, "fuse_heads", True)
    reps = 60
    pr = torch.full((reps, B, 65), float("nan"), device="cuda")
    va = torch.full((reps, B), float("nan"), device="cuda")
    with torch.no_grad():
        for i in range(reps):
            fused.evaluate_into(x, pr[i], va[i])
    torch.cuda.synchronize()
    bad_v = (va != ref_v).any(0).nonzero().flatten().tolist()
    bad_p = (pr != ref_p).any(2).any(0).nonzero().flatten().tolist()
    assert not bad_v and not bad_p, (bad_v[:16], bad_p[:16])


@pytest.mark.parametrize("B", [257, 1023, 1024])
def test_trunk_heads_bit_identical(B, monkeypatch):
    """The whole tower and the heads in one persistent launch (az_trunk_wino4_heads_gpu)
    against the tower launch + the heads-fused conv launch, and against the separate heads
    kernel: priors and values bit for bit, repeated launches."""
    from Models import FusedInferenceNet

    torch.manual_seed(7)
    net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
    fused = inference_copy(net, "cuda")
    x = torch.randint(-1, 2, (B, 64), device="cuda").float()
    out = {}
    for name, fh, th in (("separate", False, False), ("conv", True, False), ("trunk", True, True)):
        monkeypatch.setattr(FusedInferenceNet, "fuse_heads", fh)
        monkeypatch.setattr(FusedInferenceNet, "trunk_heads", th)
        reps = 20 if name == "trunk" else 1
        pr = torch.full((reps, B, 65), float("nan"), device="cuda")
        va = torch.full((reps, B), float("nan"), device="cuda")
        with torch.no_grad():
            for i in range(reps):
                fused.evaluate_into(x, pr[i], va[i])
        torch.cuda.synchronize()
        out[name] = (pr, va)
    for name in ("conv", "trunk"):
        pr, va = out[name]
        assert torch.equal(pr, out["separate"][0].expand_as(pr)), name
        assert torch.equal(va, out["separate"][1].expand_as(va)), name


@pytest.mark.parametrize("B", [1, 33, 2048])
@pytest.mark.parametrize("tile,splits", [(32, 4), (32, 8), (64, 8), (64, 16), (128, 16)])
def test_heads_fast_gemm_is_fp32_accurate(B, tile, splits):
    """az_heads_fast_gemm_gpu (FastOthelloNet's heads GEMM on the 16-bit MFMA pipe, fp16 hi /
    lo operands after power-of-two scaling -- per board and slice for the features, per
    matrix for the weights -- three products, column 128 as fp32 FMAs) against fp64: the
    summed partials within 2x torch's fp32 GEMM error (+ 1e-6), per board too (boards from
    1e-3 to 1e3), columns past 128 zero, a ragged last row tile."""
    from Models import FusedInferenceNet

    g = torch.Generator().manual_seed(B * 7 + splits + tile)
    x = torch.randn(B, 4096, generator=g).relu()
    if B > 1:
        x = x * torch.logspace(-3, 3, B).view(B, 1)
    w = torch.randn(4096, 129, generator=g) / 64.0
    ref = x.double() @ w.double()
    xd, wd = x.cuda().contiguous(), w.cuda()
    e = int(torch.frexp(wd[:, :128].abs().max())[1].item())
    ws = wd[:, :128] * (2.0 ** (15 - e))
    hi = ws.half()
    lo = (ws - hi.float()).half()
    wq = torch.stack([p.view(256, 16, 128).permute(0, 2, 1) for p in (hi, lo)], 1).contiguous()
    w128 = wd[:, 128].contiguous()
    ld = 132
    part = torch.full((splits, B, ld), float("nan"), device="cuda")
    nat.check(nat.lib.az_heads_fast_gemm_gpu(nat.ptr(xd), nat.ptr(wq.view(torch.int16)),
                                             nat.ptr(w128), 15 - e, nat.ptr(part), ld, splits,
                                             tile, B, nat.stream_ptr()), "az_heads_fast_gemm_gpu")
    torch.cuda.synchronize()
    assert torch.isfinite(part).all()
    assert (part[:, :, 129:] == 0).all()
    got = part.double().sum(0)[:, :129].cpu()
    f32 = (xd @ wd).double().cpu()
    e_g, e_32 = (got - ref).abs(), (f32 - ref).abs()
    assert e_g.max() <= 2 * e_32.max() + 1e-6, (e_g.max(), e_32.max())
    for bi in range(B):
        assert e_g[bi].max() <= 2 * e_32[bi].max() + 1e-7 * (1 + ref[bi].abs().max()), bi
    assert (FusedInferenceNet.fast_gemm_tile, FusedInferenceNet.fast_gemm_splits) in (
        (32, 4), (32, 8), (64, 8), (64, 16), (128, 16))


@pytest.mark.parametrize("B", [1, 7, 300, 2048])
def test_fast_trunk_bit_identical_to_three_launches(B, monkeypatch):
    """az_fast_trunk_gpu (FastOthelloNet's stem, residual block and conv_add in one launch,
    the activations between the convs kept in LDS) against the three stem-fused / plain direct
    FP16X2 conv launches: the tail output bit for bit, and the priors / values of the fused
    evaluation path the engine runs."""
    from Models import FusedInferenceNet

    torch.manual_seed(11)
    net = FastOthelloNet(8, 65).cuda().eval()
    fused = inference_copy(net, "cuda")
    assert fused._fast_trunk_ready()
    x = torch.randint(-1, 2, (B, 64), device="cuda").float()
    with torch.no_grad():
        a = fused._fast_trunk(x)
        b = fused.tail(fused._trunk(x.view(B, 1, 8, 8)))
        out = {}
        for flag in (True, False):
            monkeypatch.setattr(FusedInferenceNet, "fuse_fast_trunk", flag)
            pr = torch.empty(B, 65, device="cuda")
            va = torch.empty(B, device="cuda")
            fused.evaluate_into(x, pr, va)
            out[flag] = (pr, va)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert torch.equal(out[True][0], out[False][0]) and torch.equal(out[True][1], out[False][1])
