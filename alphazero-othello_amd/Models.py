"""Policy/value networks with the reference's module names and state_dict keys
(reference Models.py:1-221), plus the batched device-side evaluation the engine uses.

The modules are plain PyTorch (they carry the reference's state_dict keys and are the fp32
bar the tests hold the device path to).  What the engine evaluates is `inference_copy`: a
`FusedInferenceNet` whose stem, residual trunk (the Winograd / direct MFMA conv kernels of
csrc/conv*.hip) and heads (csrc/heads.hip) are this library's own HIP kernels.
`Inference.inference` keeps the reference's batch-1 host API (Models.py:11-31);
`evaluate_planes` is what the batched self-play engine calls on the [G, 64] canonical
planes it packs on device.
"""
import os
from typing import Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


class Inference:
    """Mixin: batch-1 host inference (reference Models.py:9-31) and batched device
    inference over packed canonical planes."""

    def inference(self, state: np.ndarray, current_player: int):
        x = torch.from_numpy((current_player * state).astype(np.float32)).unsqueeze(0)
        x = x.to(next(self.parameters()).device)
        self.eval()
        with torch.no_grad():
            logits, value = self(x)
            policy = self.softmax(logits)
        return policy[0].cpu().numpy(), value[0, 0].cpu().numpy().item()

    @torch.no_grad()
    def evaluate_planes(self, planes: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """planes: float [B, 64] canonical boards (player*state) -> (softmax priors
        float32 [B, 65], tanh values float32 [B])."""
        n = getattr(self, "board_size", 3 if planes.shape[-1] == 9 else 8)
        x = planes.view(planes.shape[0], 1, n, n)
        dt = getattr(self, "input_dtype", None) or next(self.parameters()).dtype
        if x.dtype != dt:
            x = x.to(dt)
        logits, value = self(x)
        return (torch.softmax(logits.float(), dim=-1),
                value.float().reshape(-1))


class TicTacToeNet(nn.Module, Inference):
    """3x3 MLP (reference Models.py:34-69)."""

    def __init__(self, state_size, output_size):
        super().__init__()
        self.action_size = output_size
        self.fc1 = nn.Linear(state_size, 64)
        self.fc2 = nn.Linear(64, 64)
        self.policy_head = nn.Linear(64, output_size)
        self.value_head = nn.Linear(64, 1)
        self.softmax = nn.Softmax(dim=-1)
        self._cfg = {"state_size": state_size, "output_size": output_size}

    def get_config(self):
        return dict(self._cfg)

    def forward(self, x):
        h = F.relu(self.fc2(F.relu(self.fc1(x.flatten(start_dim=1)))))
        return self.policy_head(h), torch.tanh(self.value_head(h))


class ResidualBlock(nn.Module):
    """conv-BN-ReLU-conv-BN + skip, ReLU (reference Models.py:72-90)."""

    def __init__(self, channels: int):
        super().__init__()
        self.conv1 = nn.Conv2d(channels, channels, kernel_size=3, padding=1)
        self.bn1 = nn.BatchNorm2d(channels)
        self.conv2 = nn.Conv2d(channels, channels, kernel_size=3, padding=1)
        self.bn2 = nn.BatchNorm2d(channels)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        return F.relu(self.bn2(self.conv2(y)) + x)


class FastOthelloNet(nn.Module, Inference):
    """Small net (reference Models.py:93-161): conv stem, one residual block, one extra
    conv block, FC policy head (65 logits) and a 2-layer FC value head."""

    def __init__(self, board_size: int, action_size: int):
        super().__init__()
        self.board_size = board_size
        self.action_size = action_size
        self.initial_conv = nn.Sequential(nn.Conv2d(1, 64, kernel_size=3, padding=1),
                                          nn.BatchNorm2d(64), nn.ReLU())
        self.res_block = ResidualBlock(64)
        self.conv_add = nn.Sequential(nn.Conv2d(64, 64, kernel_size=3, padding=1),
                                      nn.BatchNorm2d(64), nn.ReLU())
        flat = 64 * board_size * board_size
        self.fc_policy = nn.Linear(flat, action_size)
        self.fc_value1 = nn.Linear(flat, 64)
        self.fc_value2 = nn.Linear(64, 1)
        self.softmax = nn.Softmax(dim=-1)

    def get_config(self):
        return {"board_size": self.board_size, "action_size": self.action_size}

    def forward(self, x):
        if x.dim() == 3:
            x = x.unsqueeze(1)
        h = self.conv_add(self.res_block(self.initial_conv(x)))
        h = h.reshape(h.size(0), -1)
        value = torch.tanh(self.fc_value2(F.relu(self.fc_value1(h))))
        return self.fc_policy(h), value


class AlphaZeroNet(nn.Module, Inference):
    """ResNet trunk + AlphaZero heads (reference Models.py:164-221)."""

    def __init__(self, board_size: int, action_size: int, n_res_blocks: int = 5,
                 channels: int = 128):
        super().__init__()
        self.board_size = board_size
        self.action_size = action_size
        self.n_res_blocks = n_res_blocks
        self.channels = channels
        self.conv0 = nn.Conv2d(1, channels, 3, padding=1, bias=False)
        self.bn0 = nn.BatchNorm2d(channels)
        self.res = nn.Sequential(*[ResidualBlock(channels) for _ in range(n_res_blocks)])
        self.pol_conv = nn.Conv2d(channels, 2, 1, bias=False)
        self.pol_bn = nn.BatchNorm2d(2)
        self.pol_fc = nn.Linear(2 * board_size * board_size, action_size)
        self.val_conv = nn.Conv2d(channels, 1, 1, bias=False)
        self.val_bn = nn.BatchNorm2d(1)
        self.val_fc1 = nn.Linear(board_size * board_size, 256)
        self.val_fc2 = nn.Linear(256, 1)
        self.softmax = nn.Softmax(dim=-1)

    def get_config(self):
        return {"board_size": self.board_size, "action_size": self.action_size,
                "n_res_blocks": self.n_res_blocks, "channels": self.channels}

    def forward(self, x):
        if x.dim() == 3:
            x = x.unsqueeze(1)
        h = self.res(F.relu(self.bn0(self.conv0(x))))
        p = F.relu(self.pol_bn(self.pol_conv(h)))
        v = F.relu(self.val_bn(self.val_conv(h)))
        v = torch.tanh(self.val_fc2(F.relu(self.val_fc1(v.reshape(v.size(0), -1)))))
        return self.pol_fc(p.reshape(p.size(0), -1)), v


def get_config(net):
    return net.get_config()


def inference_copy(net: nn.Module, device, dtype=torch.float32, fused=True,
                   conv="hip", precision=None, conv_algo=None) -> nn.Module:
    """An eval-mode copy of `net` on `device` for the batched engine: BatchNorm folded
    into the preceding convolution (same function in eval mode, fewer kernels per step).
    With `fused` (AlphaZeroNet / FastOthelloNet) the convolutions run without bias and one
    HIP epilogue applies bias + residual + ReLU.  conv="hip" runs the 3x3 trunk on the
    fused MFMA kernels, in `precision`:
      "split3": bf16x3-split operands on the 16-bit MFMA pipe, six
               partial products accumulated in fp32 — fp32-accurate (csrc/conv16.hip, or
               at 128 channels the Winograd F(2x2,3x3) form csrc/conv_wino.hip;
               tests/test_nn_gpu.py bounds both errors by the fp32 kernel's against fp64);
      "fp32":  fp32 MFMA (csrc/conv.hip);
      "fp16x2": fp32-accurate with half of split3's products: both operands as an fp16
               hi + lo pair after exact power-of-two scaling (per layer for the weights, per
               board for the inputs), three products in fp32 (csrc/conv_wino4.hip at 128
               channels, csrc/conv16.hip's direct kernel at 64) -- the default for fp32;
      "fp16":  fp16 operands, fp32 accumulation (config #5's fp16 inference; the default
               when dtype is float16).
    Activations, the stem and the heads stay fp32 on the fused path.  conv_algo ("direct" /
    "wino") overrides default_conv_algo for the 16-bit trunk."""
    if precision is None:
        precision = "fp16" if dtype == torch.float16 else "fp16x2"
    assert precision in ("split3", "fp16x2", "fp32", "fp16"), precision
    import copy

    m = copy.deepcopy(net).eval()

    def fold(conv: nn.Conv2d, bn: nn.BatchNorm2d):
        w = conv.weight.detach()
        b = conv.bias.detach() if conv.bias is not None else torch.zeros(w.shape[0], device=w.device)
        scale = bn.weight.detach() / torch.sqrt(bn.running_var + bn.eps)
        conv.weight = nn.Parameter(w * scale[:, None, None, None])
        conv.bias = nn.Parameter((b - bn.running_mean) * scale + bn.bias.detach())
        return nn.Identity()

    for mod in list(m.modules()):
        if isinstance(mod, ResidualBlock):
            mod.bn1 = fold(mod.conv1, mod.bn1)
            mod.bn2 = fold(mod.conv2, mod.bn2)
        if isinstance(mod, AlphaZeroNet):
            mod.bn0 = fold(mod.conv0, mod.bn0)
            mod.pol_bn = fold(mod.pol_conv, mod.pol_bn)
            mod.val_bn = fold(mod.val_conv, mod.val_bn)
        if isinstance(mod, FastOthelloNet):
            for seq in (mod.initial_conv, mod.conv_add):
                seq[1] = fold(seq[0], seq[1])
    fusable = fused and isinstance(m, (AlphaZeroNet, FastOthelloNet))
    m = m.to(device=device, dtype=torch.float32 if fusable else dtype)
    m = m.to(memory_format=torch.channels_last)
    if fusable:
        return FusedInferenceNet(m, conv=conv, precision=precision, conv_algo=conv_algo).eval()
    return m.eval()


class _ConvEpilogue(nn.Module):
    """conv2d without bias (MIOpen) + the fused bias/residual/ReLU epilogue kernel."""

    def __init__(self, conv: nn.Conv2d):
        super().__init__()
        self.weight = nn.Parameter(conv.weight.detach().contiguous(
            memory_format=torch.channels_last), requires_grad=False)
        self.bias = nn.Parameter(conv.bias.detach().contiguous(), requires_grad=False)
        self.padding = conv.padding

    def forward(self, x, res=None, relu=True):
        import az_native as nat

        y = F.conv2d(x, self.weight, None, padding=self.padding)
        if not y.is_contiguous(memory_format=torch.channels_last):
            y = y.contiguous(memory_format=torch.channels_last)
        if res is not None and not res.is_contiguous(memory_format=torch.channels_last):
            res = res.contiguous(memory_format=torch.channels_last)
        nat.check(nat.lib.az_bias_act_gpu(nat.ptr(y), nat.ptr(self.bias),
                                          None if res is None else nat.ptr(res), y.numel(),
                                          y.shape[1], int(relu), nat.stream_ptr()),
                  "az_bias_act_gpu")
        return y


def default_conv_algo(precision, channels):
    """The 16-bit-pipe 3x3 conv algorithm: "wino4" (csrc/conv_wino4.hip) for fp16x2 and, at
    128 channels, for fp16 (whose leaf evaluation then runs as the persistent fp16 trunk with
    the stem and heads: 196 against 276 us per B = 1,024 evaluation for the direct fp16 conv,
    configs[4] 229 against 171 games/s, profiles/r05_c5_conv_algo.json); "wino"
    (csrc/conv_wino.hip, Winograd F(2x2,3x3)) where it measured faster (split3, 128 channels:
    profiles/r01_conv_mx.jsonl); "direct" (csrc/conv16.hip) elsewhere.  AZ_CONV_ALGO=
    direct|wino|wino4 overrides (fp16x2 stays wino4)."""
    if precision == "fp16x2":
        return "wino4"
    env = os.environ.get("AZ_CONV_ALGO")
    if env in ("direct", "wino", "wino4"):
        return "wino" if env == "wino4" and channels != 128 else env
    if precision == "fp16" and channels == 128:
        return "wino4"
    return "wino" if precision == "split3" and channels == 128 else "direct"


class _HipConv3x3(nn.Module):
    """3x3 conv (Ci = Co in {64, 128}) + bias (+ residual) + ReLU in one MFMA kernel:
    precision "fp32" = csrc/conv.hip (weights re-laid [tap][Co][Ci]); "split3" / "fp16" =
    csrc/conv16.hip (algo "direct": weights split once into 16-bit planes by
    az_conv3x3_mx_prep_gpu) or csrc/conv_wino.hip (algo "wino": weights transformed to the
    Winograd domain and split by az_conv3x3_wino_prep_gpu)."""

    MODES = {"split3": 0, "fp16": 1, "fp16x2": 2}  # AZ_CONV_SPLIT3, AZ_CONV_FP16, _FP16X2

    def __init__(self, conv: nn.Conv2d, precision="split3", algo=None):
        super().__init__()
        import az_native as nat

        w = conv.weight.detach()
        co, ci = w.shape[0], w.shape[1]
        assert co == ci and co in (64, 128) and w.shape[2:] == (3, 3)
        self.channels = co
        if precision == "fp16x2" and co != 128 and os.environ.get("AZ_CONV64_SPLIT3") == "1":
            precision = "split3"  # A/B: the bf16x3 direct kernel at 64 channels (round 5's)
        self.precision = precision
        self.algo = "direct" if precision == "fp32" else (algo or default_conv_algo(precision, co))
        if self.algo == "wino4" and co != 128:  # the 4-board form is built for 128 channels
            self.algo = "wino"
        if precision == "fp16x2" and co != 128:
            # the scaled fp16 pair at 64 channels: the direct kernel (csrc/conv16.hip), each
            # workgroup scaling its board by the max |x| it stages
            self.algo = "direct"
        w9 = w.float().permute(2, 3, 0, 1).reshape(9, co, ci).contiguous()
        self.bias = nn.Parameter(conv.bias.detach().float().contiguous(), requires_grad=False)
        if precision == "fp32":
            self.w9 = nn.Parameter(w9, requires_grad=False)
        else:
            self.mode = self.MODES[precision]
            wino = self.algo in ("wino", "wino4")
            if wino:
                n16 = nat.lib.az_conv3x3_wino_prep_bytes(co, self.mode) // 2
            else:
                n16 = nat.lib.az_conv3x3_mx_prep_bytes(co, self.mode) // 2
            wq = torch.empty(n16, dtype=torch.int16, device=w.device)
            prep = nat.lib.az_conv3x3_wino_prep_gpu if wino else nat.lib.az_conv3x3_mx_prep_gpu
            nat.check(prep(nat.ptr(w9), nat.ptr(wq), co, self.mode, nat.stream_ptr()),
                      "conv3x3 weight prep")
            self.wq = nn.Parameter(wq, requires_grad=False)

    def forward(self, x, res=None, relu=True, in_absmax=None, out_absmax=None, part=None,
                splits=0):
        """in_absmax / out_absmax: float [B] per-board max |x| (consumed: reset to 0) and
        max |y| accumulator (zeros on entry) of the wino4 kernel; fp16x2 needs in_absmax
        (computed here when absent).  splits (2 or 4, fp16x2 only) with part (float
        [splits * B * 64 * C]): the channel-split form for small batches
        (az_conv3x3_wino4_splitk_gpu)."""
        import az_native as nat

        x = x.contiguous(memory_format=torch.channels_last)
        if res is not None:
            res = res.contiguous(memory_format=torch.channels_last)
        y = torch.empty_like(x, memory_format=torch.channels_last)
        rp = None if res is None else nat.ptr(res)
        if self.algo == "wino4":
            if self.precision == "fp16x2" and in_absmax is None:
                in_absmax = board_absmax(x)
            if splits and self.precision == "fp16x2":
                nat.check(nat.lib.az_conv3x3_wino4_splitk_gpu(
                    nat.ptr(x), nat.ptr(self.wq), nat.ptr(self.bias), rp, nat.ptr(y), x.shape[0],
                    self.channels, int(relu), self.mode, nat.ptr(in_absmax), nat.ptr(out_absmax),
                    nat.ptr(part), splits, nat.stream_ptr()), "az_conv3x3_wino4_splitk_gpu")
                return y
            nat.check(nat.lib.az_conv3x3_wino4_gpu(
                nat.ptr(x), nat.ptr(self.wq), nat.ptr(self.bias), rp, nat.ptr(y), x.shape[0],
                self.channels, int(relu), self.mode, nat.ptr(in_absmax), nat.ptr(out_absmax),
                nat.stream_ptr()), "az_conv3x3_wino4_gpu")
            return y
        if self.precision == "fp32":
            rc = nat.lib.az_conv3x3_gpu(nat.ptr(x), nat.ptr(self.w9), nat.ptr(self.bias), rp,
                                        nat.ptr(y), x.shape[0], self.channels, int(relu),
                                        nat.stream_ptr())
            nat.check(rc, "az_conv3x3_gpu")
        else:
            name = {"wino": "az_conv3x3_wino_gpu", "direct": "az_conv3x3_mx_gpu"}[self.algo]
            rc = getattr(nat.lib, name)(nat.ptr(x), nat.ptr(self.wq), nat.ptr(self.bias), rp,
                                        nat.ptr(y), x.shape[0], self.channels, int(relu),
                                        self.mode, nat.stream_ptr())
            nat.check(rc, name)
        return y

    def forward_heads(self, x, res, in_absmax, hw, priors, values):
        """This conv (the trunk's last: residual + ReLU, fp16x2 Winograd) with AlphaZeroNet's
        heads fused into its epilogue (az_conv3x3_wino4_heads_gpu): priors float32 [B, 65]
        and values float32 [B] written directly, the trunk output never stored."""
        import az_native as nat

        assert self.algo == "wino4" and self.precision == "fp16x2"
        x = x.contiguous(memory_format=torch.channels_last)
        res = res.contiguous(memory_format=torch.channels_last)
        nat.check(nat.lib.az_conv3x3_wino4_heads_gpu(
            nat.ptr(x), nat.ptr(self.wq), nat.ptr(self.bias), nat.ptr(res), x.shape[0],
            self.channels, self.mode, nat.ptr(in_absmax), nat.ptr(hw["wpv"]), nat.ptr(hw["bpv"]),
            nat.ptr(hw["wpolT"]), nat.ptr(hw["bpol"]), nat.ptr(hw["w1T"]), nat.ptr(hw["b1"]),
            nat.ptr(hw["w2"]), nat.ptr(hw["b2"]), nat.ptr(priors), nat.ptr(values),
            nat.stream_ptr()), "az_conv3x3_wino4_heads_gpu")

    def forward_stem(self, planes, stem, role, x=None):
        """This conv fused with the stem (`_HipStem`): role 1 = input stem(planes), role 2 =
        residual stem(planes) (input x); bias + ReLU epilogue (csrc/conv16.hip)."""
        import az_native as nat

        B = planes.shape[0]
        y = torch.empty((B, self.channels, 8, 8), dtype=torch.float32, device=planes.device,
                        memory_format=torch.channels_last)
        xp = None
        if role == 2:
            x = x.contiguous(memory_format=torch.channels_last)
            xp = nat.ptr(x)
        nat.check(nat.lib.az_conv3x3_mx_stem_gpu(
            nat.ptr(planes), nat.ptr(stem.w9), nat.ptr(stem.bias), xp, nat.ptr(self.wq),
            nat.ptr(self.bias), nat.ptr(y), B, self.channels, role, self.mode,
            nat.stream_ptr()), "az_conv3x3_mx_stem_gpu")
        return y


class _HipStem(nn.Module):
    """1 -> C 3x3 stem conv + bias + ReLU on the canonical planes (csrc/conv.hip)."""

    def __init__(self, conv: nn.Conv2d):
        super().__init__()
        w = conv.weight.detach()
        assert w.shape[1] == 1 and w.shape[0] in (64, 128)
        self.channels = w.shape[0]
        self.w9 = nn.Parameter(w.reshape(w.shape[0], 9).t().contiguous(), requires_grad=False)
        self.bias = nn.Parameter(conv.bias.detach().float().contiguous(), requires_grad=False)

    def forward(self, x, res=None, relu=True, absmax=None):
        """absmax: optional float [B] receiving each board's max |y| (FP16X2 trunk)."""
        import az_native as nat

        planes = x.reshape(x.shape[0], 64).contiguous()
        y = torch.empty((x.shape[0], self.channels, 8, 8), dtype=torch.float32, device=x.device,
                        memory_format=torch.channels_last)
        nat.check(nat.lib.az_conv_stem2_gpu(nat.ptr(planes), nat.ptr(self.w9), nat.ptr(self.bias),
                                            nat.ptr(y), x.shape[0], self.channels,
                                            nat.ptr(absmax), nat.stream_ptr()), "az_conv_stem2_gpu")
        return y


def board_absmax(x, out=None):
    """float [B] max |x| of each board of an NHWC [B, C, 8, 8] tensor (az_board_absmax_gpu)."""
    import az_native as nat

    x = x.contiguous(memory_format=torch.channels_last)
    if out is None:
        out = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    nat.check(nat.lib.az_board_absmax_gpu(nat.ptr(x), x.shape[0], x.shape[1], nat.ptr(out),
                                          nat.stream_ptr()), "az_board_absmax_gpu")
    return out


def _merge_1x1(a: nn.Conv2d, b: nn.Conv2d) -> nn.Conv2d:
    m = nn.Conv2d(a.in_channels, a.out_channels + b.out_channels, 1)
    m.weight = nn.Parameter(torch.cat([a.weight.detach(), b.weight.detach()], 0))
    m.bias = nn.Parameter(torch.cat([a.bias.detach(), b.bias.detach()], 0))
    return m.to(a.weight.device)


class FusedInferenceNet(nn.Module, Inference):
    """Inference-only form of AlphaZeroNet / FastOthelloNet with BatchNorm folded and every
    conv epilogue fused (same function as the source net in eval mode).  conv="hip": the
    stem and the 3x3 trunk run on the fused MFMA kernels of csrc/conv.hip (stem, fp32 trunk)
    and csrc/conv16.hip (split3 / fp16 trunk); conv="miopen": MIOpen convolutions + the
    az_bias_act_gpu epilogue."""

    input_dtype = torch.float32

    def __init__(self, m: nn.Module, conv="hip", precision="split3", conv_algo=None):
        super().__init__()
        self.conv_impl = conv
        self.precision = precision
        self.kind = "az" if isinstance(m, AlphaZeroNet) else "fast"
        self.board_size = m.board_size
        self.softmax = nn.Softmax(dim=-1)
        if conv == "hip":
            C3 = lambda c: _HipConv3x3(c, precision, conv_algo)  # noqa: E731
        else:
            C3 = _ConvEpilogue
        Stem = _HipStem if conv == "hip" else _ConvEpilogue
        if self.kind == "az":
            self.stem = Stem(m.conv0)
            blocks = list(m.res)
            self.heads = _ConvEpilogue(_merge_1x1(m.pol_conv, m.val_conv))
            self.n_pol = m.pol_conv.out_channels
            self.pol_fc, self.val_fc1, self.val_fc2 = m.pol_fc, m.val_fc1, m.val_fc2
        else:
            self.stem = Stem(m.initial_conv[0])
            blocks = [m.res_block]
            self.tail = C3(m.conv_add[0])
            self.fc_policy, self.fc_value1, self.fc_value2 = m.fc_policy, m.fc_value1, m.fc_value2
        self.c1 = nn.ModuleList([C3(b.conv1) for b in blocks])
        self.c2 = nn.ModuleList([C3(b.conv2) for b in blocks])

    fuse_stem = True  # the stem evaluated inside the first block's convs (never stored)
    # Winograd trunk as one launch (az_trunk_wino_gpu): bit-identical, but measured 3 % slower
    # than the layer-by-layer graph at the bench batch (scripts/trunk_bench.py,
    # profiles/r01_trunk_bench.jsonl), so off by default
    fuse_trunk = False
    # fp16x2 trunk at small batches (a search's few leaves per step): the channel-split conv
    # (az_conv3x3_wino4_splitk_gpu) puts `splits` workgroups on each four boards.  Per-launch
    # times in 20-layer HIP graphs (scripts/splitk_sweep.py, profiles/r02_splitk_sweep.jsonl;
    # one pass / 4 / 8 / 16 splits): 4 boards 32.0 / 13.6 / 10.8 / 9.4 us, 16: 32.6 / 15.4 /
    # 13.6 / 13.8, 64: 33.0 / 19.5 / 20.4 / 23.6, 256: 34.4 / 27.5 / 37.8 / 62.1.
    # AZ_SPLITK=<splits> (0 = off) forces one form.
    splitk_table = ((8, 16), (32, 8), (256, 4))  # (max boards, splits)

    @classmethod
    def splitk_for(cls, n_boards):
        env = os.environ.get("AZ_SPLITK")
        if env is not None:
            return int(env)
        for max_b, splits in cls.splitk_table:
            if n_boards <= max_b:
                return splits
        return 0

    def _trunk_kernel_ready(self):
        """Whether the single-launch trunk (az_trunk_wino_gpu) applies: HIP stem and every
        block conv on the Winograd kernel in one numerics mode."""
        convs = list(self.c1) + list(self.c2)
        if not (self.fuse_trunk and isinstance(self.stem, _HipStem) and convs):
            return False
        if not all(getattr(c, "algo", "") == "wino" and c.mode == convs[0].mode for c in convs):
            return False
        if not hasattr(self, "_tw"):
            dev = self.stem.w9.device
            order = [c for pair in zip(self.c1, self.c2) for c in pair]  # layer order
            self._tw = {
                "wq": torch.tensor([c.wq.data_ptr() for c in order], dtype=torch.int64, device=dev),
                "bias": torch.tensor([c.bias.data_ptr() for c in order], dtype=torch.int64,
                                     device=dev),
                "mode": convs[0].mode, "C": convs[0].channels, "blocks": len(self.c1)}
        return True

    # eager-only batch sizes whose trunk scratch is kept (most recently used first out)
    scratch_cap = 4

    def _scratch(self, device, B):
        """Trunk scratch (per-board ranges, split-K partials) of one (device, batch size).
        Sizes seen while a HIP graph is being captured are pinned for the net's lifetime
        (the graph keeps pointing at their buffers); at most `scratch_cap` other sizes are
        kept, least recently used dropped first (a caller evaluating many ragged batch sizes
        does not accumulate buffers).  release_scratch() drops the unpinned ones."""
        sc = self.__dict__.setdefault("_trunk_scratch", {})
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:  # "cuda" and "cuda:0": one entry
            device = torch.device("cuda", torch.cuda.current_device())
        key = (device, B)
        ent = sc.pop(key, None)  # re-inserted below: dict order = recency
        if ent is None:
            ent = {"absmax": [torch.zeros(B, dtype=torch.float32, device=device)
                              for _ in range(2)], "pinned": False}
        if torch.cuda.is_current_stream_capturing():
            ent["pinned"] = True
        sc[key] = ent
        loose = [k for k, v in sc.items() if not v["pinned"]]
        for k in loose[:max(0, len(loose) - self.scratch_cap)]:
            del sc[k]  # stream-ordered free: queued work on this stream still sees it
        return ent

    def release_scratch(self):
        sc = self.__dict__.get("_trunk_scratch", {})
        for k in [k for k, v in sc.items() if not v["pinned"]]:
            del sc[k]

    # AlphaZeroNet on the fp16x2 Winograd trunk: the heads run in the last conv's epilogue
    # (az_conv3x3_wino4_heads_gpu, bit-identical to the separate heads kernel; one launch and
    # the trunk output's HBM round trip fewer per evaluation).  AZ_FUSE_HEADS=0 turns it off.
    fuse_heads = os.environ.get("AZ_FUSE_HEADS", "1") != "0"

    def _stem_stored(self):
        """Whether the trunk starts with a stored HIP stem output feeding the fp16x2 block
        convs (the branch of _trunk an engine-side stem can replace)."""
        c1s, c2s = list(self.c1), list(self.c2)
        return (isinstance(self.stem, _HipStem) and bool(c1s) and not self._trunk_kernel_ready()
                and not (self.fuse_stem and getattr(c1s[0], "precision", "fp32") != "fp32"
                         and c1s[0].algo == "direct" and c2s[0].algo == "direct")
                and getattr(c1s[0], "precision", "") == "fp16x2")

    def engine_stem(self, device, B):
        """The stem for the engine that packs the planes to run (az_engine_set_stem): its
        weights and this batch size's first-activation buffers (NHWC [B, C, 8, 8] and the
        per-board ranges the first conv reads), pinned for the net's lifetime; None where the
        trunk does not start from a stored HIP stem on the fp16x2 path.  Calls of
        evaluate_into(..., stem_done=True) at that batch size then start at the first block."""
        if not (self._fused_heads_ready() and self._stem_stored()):
            return None
        if self.trunk_stem and self._trunk4_ready(list(self.c1), list(self.c2), B) \
                and self.splitk_for(B) == 0:
            return None  # the persistent trunk runs the stem (its output stays in L2)
        ent = self._scratch(device, B)
        ent["pinned"] = True
        C = self.stem.channels
        if "h0" not in ent:
            ent["h0"] = torch.empty((B, C, 8, 8), dtype=torch.float32, device=device,
                                    memory_format=torch.channels_last)
        return {"w9": self.stem.w9, "bias": self.stem.bias, "y": ent["h0"],
                "absmax": ent["absmax"][0], "channels": C}

    def _trunk(self, x, heads_into=None, stem_done=False):
        """The trunk's output (NHWC [B, C, 8, 8]); with heads_into = (priors, values) the
        heads may be fused into the last conv, which then writes them and None is returned
        (evaluate_into falls back to the separate heads kernel on a tensor).  stem_done: the
        stem's output and ranges are already in this batch size's engine_stem buffers."""
        if x.dim() == 3:
            x = x.unsqueeze(1)
        x = x.contiguous(memory_format=torch.channels_last)
        if stem_done:
            ent = self._scratch(x.device, x.shape[0])
            if not (self._stem_stored() and "h0" in ent):
                raise RuntimeError("stem_done without engine_stem buffers for this batch size")
        if self._trunk_kernel_ready():
            import az_native as nat

            tw = self._tw
            B = x.shape[0]
            planes = x.reshape(B, 64).contiguous()
            h = torch.empty((B, tw["C"], 8, 8), dtype=torch.float32, device=x.device,
                            memory_format=torch.channels_last)
            t = torch.empty_like(h, memory_format=torch.channels_last)
            nat.check(nat.lib.az_trunk_wino_gpu(
                nat.ptr(planes), nat.ptr(self.stem.w9), nat.ptr(self.stem.bias),
                nat.ptr(tw["wq"]), nat.ptr(tw["bias"]), nat.ptr(h), nat.ptr(t), B,
                tw["blocks"], tw["C"], tw["mode"], nat.stream_ptr()), "az_trunk_wino_gpu")
            return h
        c1s, c2s = list(self.c1), list(self.c2)
        if (self.fuse_stem and isinstance(self.stem, _HipStem) and c1s
                and getattr(c1s[0], "precision", "fp32") != "fp32"
                and c1s[0].algo == "direct" and c2s[0].algo == "direct"):
            planes = x.reshape(x.shape[0], 64).contiguous()
            h = c2s[0].forward_stem(planes, self.stem, 2, x=c1s[0].forward_stem(planes, self.stem, 1))
            c1s, c2s = c1s[1:], c2s[1:]
        elif c1s and getattr(c1s[0], "precision", "") == "fp16x2":
            # per-board input ranges ping-pong between two buffers: each conv consumes (and
            # resets) one and accumulates its output's into the other; the stem writes the
            # first (or, for a non-HIP stem, a separate max pass does)
            B = x.shape[0]
            ent = self._scratch(x.device, B)
            bufs = ent["absmax"]
            sk = {}
            splits = self.splitk_for(B)
            if splits and all(c.algo == "wino4" for c in c1s + c2s):
                n = splits * B * 64 * c1s[0].channels
                part = ent.get("part")
                if part is None or part.numel() != n:
                    part = ent["part"] = torch.empty(n, dtype=torch.float32, device=x.device)
                sk = {"part": part, "splits": splits}
            fuse = (heads_into is not None and not sk and self.fuse_heads
                    and self._fused_heads_ready() and c2s[-1].algo == "wino4"
                    and c2s[-1].precision == "fp16x2" and c2s[-1].channels == 128)
            t4 = not sk and self._trunk4_ready(c1s, c2s, B, heads_into_ok=fuse)
            cap = self._trunk4_cap(c1s[0].wq.device) if c1s else B
            if t4 and B > cap:
                # more boards than are resident at once: the persistent trunk per chunk of
                # `cap` boards (every workgroup of a launch resident, at the same layer),
                # heads fused (the tower's output is not returned)
                if not stem_done:
                    if isinstance(self.stem, _HipStem):
                        h0 = self.stem(x, absmax=bufs[0])
                    else:
                        h0 = self.stem(x)
                        board_absmax(h0, out=bufs[0])
                else:
                    h0 = ent["h0"]
                for b0 in range(0, B, cap):
                    b1 = min(B, b0 + cap)
                    self._trunk4(h0[b0:b1], [bufs[0][b0:b1], bufs[1][b0:b1]], c1s, c2s,
                                 (heads_into[0][b0:b1], heads_into[1][b0:b1]))
                return None
            if t4 and not stem_done and isinstance(self.stem, _HipStem):
                # the stem inside the persistent trunk (each workgroup's boards first)
                return self._trunk4(None, bufs, c1s, c2s, heads_into if fuse else None, planes=x)
            if stem_done:  # written by the engine's select launch (engine_stem)
                h = ent["h0"]
            elif isinstance(self.stem, _HipStem):
                h = self.stem(x, absmax=bufs[0])
            else:
                h = self.stem(x)
                board_absmax(h, out=bufs[0])
            if t4:
                return self._trunk4(h, bufs, c1s, c2s, heads_into if fuse else None)
            for i, (c1, c2) in enumerate(zip(c1s, c2s)):
                t = c1(h, in_absmax=bufs[0], out_absmax=bufs[1], **sk)
                if fuse and i == len(c1s) - 1:
                    c2.forward_heads(t, h, bufs[1], self._hw, *heads_into)
                    return None
                h = c2(t, res=h, in_absmax=bufs[1], out_absmax=bufs[0], **sk)
            return h
        elif heads_into is not None and not stem_done and \
                self._trunk4_fp16_ready(c1s, c2s, x.shape[0]):
            # fp16 wino4 convs: the stem, the tower and the heads in one persistent launch
            # per chunk of resident boards (az_trunk_wino4_heads_fp16_gpu)
            B = x.shape[0]
            bufs = self._scratch(x.device, B)["absmax"]
            cap = self._trunk4_cap(c1s[0].wq.device)
            for b0 in range(0, B, cap):
                b1 = min(B, b0 + cap)
                self._trunk4_heads(None, [bufs[0][b0:b1], bufs[1][b0:b1]], c1s,
                                   (heads_into[0][b0:b1], heads_into[1][b0:b1]),
                                   planes=x[b0:b1], fp16=True)
            return None
        else:
            h = self.stem(x)
        for c1, c2 in zip(c1s, c2s):
            h = c2(c1(h), res=h)
        return h

    # fp16x2 tower as one persistent launch (az_trunk_wino4_gpu): every block conv but a
    # fused-heads last one in a single kernel, each two-board workgroup carrying its boards
    # through the layers -- bit-identical to the per-layer launches.  Used while every
    # workgroup is resident at once (two two-board workgroups per CU: B <= 4 x CUs, e.g.
    # configs[2]'s 1,024): configs[2] 97.5 -> 98.0 games/s same box; at 4,096 boards (four
    # rounds of workgroups, each at its own layer, so the layers' weights compete for L2) it
    # measured 1.6 % slower (profiles/r03_trunk4_ab.json).  AZ_FUSE_TRUNK4=0: off.
    fuse_trunk4 = os.environ.get("AZ_FUSE_TRUNK4", "1") != "0"
    # AZ_TRUNK_STEM=1: the stem too (each workgroup's boards before the first layer) instead
    # of in the engine's select launch (engine_stem then returns None).  Off: configs[2] 96.4
    # vs 97.0 games/s with the engine stem, same box (profiles/r03_trunk_stem_ab.json) -- the
    # stem's 33.5 MB store then precedes the first layer instead of hiding under the descents
    trunk_stem = os.environ.get("AZ_TRUNK_STEM", "0") == "1"

    # AZ_TRUNK4_CHUNKS (default on): batches larger than the resident capacity run the
    # persistent trunk once per chunk of 4 x CUs boards (with the heads fused), instead of one
    # launch per layer over the whole batch
    trunk4_chunks = os.environ.get("AZ_TRUNK4_CHUNKS", "1") != "0"

    def _trunk4_cap(self, dev):
        """Boards the persistent trunk keeps resident at once: two two-board workgroups per CU."""
        return 4 * torch.cuda.get_device_properties(dev).multi_processor_count

    def _trunk4_ready(self, c1s, c2s, B, heads_into_ok=False):
        convs = c1s + c2s
        if not (self.fuse_trunk4 and convs and os.environ.get("AZ_W4_BOARDS", "2") == "2"):
            return False
        dev = convs[0].wq.device
        if B > self._trunk4_cap(dev) and not (self.trunk4_chunks and heads_into_ok):
            return False
        if not all(getattr(c, "algo", "") == "wino4" and c.precision == "fp16x2"
                   and c.channels == 128 for c in convs):
            return False
        if not hasattr(self, "_t4"):
            order = [c for pair in zip(c1s, c2s) for c in pair]  # layer order
            self._t4 = {
                "wq": torch.tensor([c.wq.data_ptr() for c in order], dtype=torch.int64, device=dev),
                "bias": torch.tensor([c.bias.data_ptr() for c in order], dtype=torch.int64,
                                     device=dev)}
        return True

    # AZ_TRUNK_FP16 (default on): fp16 wino4 convs (AZ_CONV_ALGO=wino4 at fp16) run as the
    # persistent trunk with the stem and heads (az_trunk_wino4_heads_fp16_gpu) when the caller
    # takes priors / values; 0 = per-layer launches
    trunk_fp16 = os.environ.get("AZ_TRUNK_FP16", "1") == "1"

    def _trunk4_fp16_ready(self, c1s, c2s, B=0):
        convs = c1s + c2s
        if not (self.trunk_fp16 and self.fuse_trunk4 and self.trunk_heads and convs
                and isinstance(self.stem, _HipStem) and self._fused_heads_ready()
                and os.environ.get("AZ_W4_BOARDS", "2") == "2"):
            return False
        if not all(getattr(c, "algo", "") == "wino4" and c.precision == "fp16"
                   and c.channels == 128 for c in convs):
            return False
        # more boards than are resident at once run one launch per chunk: AZ_TRUNK4_CHUNKS=0
        # turns that off here as for the fp16x2 trunk (per-layer launches instead)
        if B > self._trunk4_cap(convs[0].wq.device) and not self.trunk4_chunks:
            return False
        if not hasattr(self, "_t4"):
            dev = convs[0].wq.device
            order = [c for pair in zip(c1s, c2s) for c in pair]  # layer order
            self._t4 = {
                "wq": torch.tensor([c.wq.data_ptr() for c in order], dtype=torch.int64, device=dev),
                "bias": torch.tensor([c.bias.data_ptr() for c in order], dtype=torch.int64,
                                     device=dev)}
        return True

    def _trunk4(self, h, bufs, c1s, c2s, heads_into, planes=None):
        """The tower on az_trunk_wino4_gpu: all 2n convs (returns the output), or with
        heads_into the first 2n - 1 and the last conv with the heads fused (returns None).
        planes (canonical boards [B, 1, 8, 8]) instead of h: the stem runs in the same launch."""
        import az_native as nat

        C = c1s[0].channels
        if heads_into is not None and self.trunk_heads:
            return self._trunk4_heads(h, bufs, c1s, heads_into, planes)
        if planes is not None:
            B = planes.shape[0]
            planes = planes.reshape(B, 64).contiguous()
            h = torch.empty((B, C, 8, 8), dtype=torch.float32, device=planes.device,
                            memory_format=torch.channels_last)
        B = h.shape[0]
        n_convs = 2 * len(c1s) - (1 if heads_into is not None else 0)
        hb = [torch.empty_like(h, memory_format=torch.channels_last) for _ in range(2)]
        t = torch.empty_like(h, memory_format=torch.channels_last)
        st = self.stem if planes is not None else None
        nat.check(nat.lib.az_trunk_wino4_gpu(
            nat.ptr(self._t4["wq"]), nat.ptr(self._t4["bias"]), nat.ptr(planes),
            nat.ptr(st.w9) if st is not None else None, nat.ptr(st.bias) if st is not None else None,
            nat.ptr(h), nat.ptr(hb[0]), nat.ptr(hb[1]), nat.ptr(t), nat.ptr(bufs[0]),
            nat.ptr(bufs[1]), B, n_convs, C, nat.stream_ptr()), "az_trunk_wino4_gpu")
        n_blocks = n_convs // 2
        h_last = hb[(n_blocks - 1) & 1] if n_blocks else h
        if heads_into is not None:
            c2s[-1].forward_heads(t, h_last, bufs[1], self._hw, *heads_into)
            return None
        return h_last

    # AZ_TRUNK_HEADS (default on): the heads inside the persistent trunk's launch
    # (az_trunk_wino4_heads_gpu, bit-identical), its last conv run after the layer loop as the
    # heads-fused body, instead of the heads-fused last conv as a launch of its own: B = 1,024
    # evaluation 423.3 vs 424.6 us, configs[2] 102.8-102.9 vs 102.5-102.7 games/s same box
    # (profiles/r04_trunk_heads_epi_ab.json).  (Its first form stored the last layer's output
    # and read it back for the heads: 4 us slower, profiles/r04_net_ab.json.)  AZ_TRUNK_HEADS=0:
    # the separate heads-fused conv launch
    trunk_heads = os.environ.get("AZ_TRUNK_HEADS", "1") == "1"

    def _trunk4_heads(self, h, bufs, c1s, heads_into, planes=None, fp16=False):
        """The whole tower and the heads in one az_trunk_wino4_heads_gpu launch (fp16: the
        fp16 wino4 convs', az_trunk_wino4_heads_fp16_gpu)."""
        import az_native as nat

        C = c1s[0].channels
        if planes is not None:
            B = planes.shape[0]
            planes = planes.reshape(B, 64).contiguous()
            h = torch.empty((B, C, 8, 8), dtype=torch.float32, device=planes.device,
                            memory_format=torch.channels_last)
        B = h.shape[0]
        hb = [torch.empty_like(h, memory_format=torch.channels_last) for _ in range(2)]
        t = torch.empty_like(h, memory_format=torch.channels_last)
        st = self.stem if planes is not None else None
        hw = self._hw
        priors, values = heads_into
        fn = "az_trunk_wino4_heads_fp16_gpu" if fp16 else "az_trunk_wino4_heads_gpu"
        nat.check(getattr(nat.lib, fn)(
            nat.ptr(self._t4["wq"]), nat.ptr(self._t4["bias"]), nat.ptr(planes),
            nat.ptr(st.w9) if st is not None else None, nat.ptr(st.bias) if st is not None else None,
            nat.ptr(h), nat.ptr(hb[0]), nat.ptr(hb[1]), nat.ptr(t), nat.ptr(bufs[0]),
            nat.ptr(bufs[1]), B, 2 * len(c1s), C, nat.ptr(hw["wpv"]), nat.ptr(hw["bpv"]),
            nat.ptr(hw["wpolT"]), nat.ptr(hw["bpol"]), nat.ptr(hw["w1T"]), nat.ptr(hw["b1"]),
            nat.ptr(hw["w2"]), nat.ptr(hw["b2"]), nat.ptr(priors), nat.ptr(values),
            nat.stream_ptr()), fn)
        return None

    def _fused_heads_ready(self):
        if self.kind != "az" or self.conv_impl != "hip":
            return False
        if not hasattr(self, "_hw"):
            C = self.heads.weight.shape[1]
            pol, v1, v2 = self.pol_fc, self.val_fc1, self.val_fc2
            self._hw = {
                "wpv": self.heads.weight.detach().reshape(3, C).float().contiguous(),
                "bpv": self.heads.bias.detach().float().contiguous(),
                "wpolT": pol.weight.detach().float().t().contiguous(),      # [128][65]
                "bpol": pol.bias.detach().float().contiguous(),
                "w1T": v1.weight.detach().float().t().contiguous(),         # [64][256]
                "b1": v1.bias.detach().float().contiguous(),
                "w2": v2.weight.detach().float().reshape(-1).contiguous(),  # [256]
                "b2": v2.bias.detach().float().contiguous(),
                "C": C,
            }
        return True

    # AZ_FAST_HEADS (default on): FastOthelloNet's heads as ONE GEMM of the tail output, read in
    # its NHWC layout (no flattening copy: the FC weights' columns are permuted instead),
    # against [fc_policy; fc_value1], then az_heads_fast_finish_gpu (softmax, ReLU -> fc_value2
    # -> tanh) straight into the engine's buffers -- instead of a flattening copy, three GEMMs,
    # softmax / ReLU / tanh kernels and two device copies per evaluation
    fuse_fast_heads = os.environ.get("AZ_FAST_HEADS", "1") == "1"

    def _fast_heads_ready(self):
        if not (self.kind == "fast" and self.conv_impl == "hip" and self.fuse_fast_heads):
            return False
        # the finish kernel's layout: 65 policy logits + 64 value hidden units per board (one
        # wavefront per board); any other head shape runs the module heads
        if not (self.fc_policy.out_features == 65 and self.fc_value1.out_features == 64
                and self.fc_value2.in_features == 64 and self.fc_value2.out_features == 1):
            return False
        if not hasattr(self, "_fw"):
            pol, v1, v2 = self.fc_policy, self.fc_value1, self.fc_value2
            w = torch.cat([pol.weight.detach(), v1.weight.detach()]).float()  # [129, C * 64]
            n_out, C = w.shape[0], w.shape[1] // 64
            # reference flattening index c * 64 + square -> the NHWC tail's square * C + c
            w = w.view(n_out, C, 64).permute(0, 2, 1).reshape(n_out, 64 * C)
            ld = 132  # logits row stride (columns 129.. are zero)
            wt = torch.zeros(64 * C, ld, dtype=torch.float32, device=w.device)
            wt[:, :n_out] = w.t()
            bias = torch.zeros(ld, dtype=torch.float32, device=w.device)
            bias[:n_out] = torch.cat([pol.bias.detach(), v1.bias.detach()]).float()
            # split-K (AZ_FAST_SPLITK, experiments): S slices of the reduction as one batched
            # GEMM, the partial sums added in slice order by the finish kernel.  S = 4 cut the
            # GEMM + finish kernels 61.6 -> 53.6 us per 2,048 boards, but configs[1] ran 1,970-1,985
            # games/s against 2,018-2,025 with S = 1 (8: 1,844; profiles/r05_fast_heads_ab.json)
            S = int(os.environ.get("AZ_FAST_SPLITK", "1"))
            if S < 1 or (64 * C) % S:
                raise ValueError(f"AZ_FAST_SPLITK={S} does not divide the {64 * C} inputs")
            self._fw = {"wk": wt.contiguous().view(S, 64 * C // S, ld), "S": S,
                        "bias": bias, "ld": ld,
                        "w2": v2.weight.detach().float().reshape(-1).contiguous(),
                        "b2": v2.bias.detach().float().contiguous()}
            if self.fast_gemm and C == 64:
                # az_heads_fast_gemm_gpu's operands: columns 0..127 scaled by 2^wshift (max
                # |W| < 2^(15 - wshift)) and split into fp16 hi / lo planes laid out as the MFMA
                # B fragments [K/16][hi, lo][128][16]; column 128 stays fp32 (its FMAs)
                w128 = wt[:, :128]
                e = int(torch.frexp(w128.abs().max())[1].item())  # max |W| < 2^e
                ws = w128 * (2.0 ** (15 - e))  # exact: a power of two
                hi = ws.half()
                lo = (ws - hi.float()).half()
                planes = torch.stack([p.view(64 * C // 16, 16, 128).permute(0, 2, 1)
                                      for p in (hi, lo)], 1).contiguous()  # [K/16][2][128][16]
                self._fw.update(gq=planes.view(torch.int16), g128=wt[:, 128].contiguous(),
                                gshift=15 - e, gS=self.fast_gemm_splits,
                                gR=self.fast_gemm_tile)
        return True

    # AZ_FAST_TRUNK (default on): FastOthelloNet's stem + residual block + conv_add in FP16X2 as
    # ONE launch (az_fast_trunk_gpu: the activations between the convs stay in LDS; bit-identical
    # to the three stem-fused / plain direct conv launches); 0 = the three launches
    fuse_fast_trunk = os.environ.get("AZ_FAST_TRUNK", "1") == "1"

    def _fast_trunk_ready(self):
        if not (self.kind == "fast" and self.conv_impl == "hip" and self.fuse_fast_trunk
                and self.fuse_stem and isinstance(self.stem, _HipStem) and len(self.c1) == 1):
            return False
        convs = [self.c1[0], self.c2[0], self.tail]
        return all(getattr(c, "precision", "") == "fp16x2" and c.algo == "direct"
                   and c.channels == 64 for c in convs)

    def _fast_trunk(self, planes):
        """The tail conv's output (NHWC [B, 64, 8, 8]) from canonical planes [B, 64] in one
        launch (az_fast_trunk_gpu)."""
        import az_native as nat

        B = planes.shape[0]
        planes = planes.reshape(B, 64).contiguous()
        t = torch.empty((B, 64, 8, 8), dtype=torch.float32, device=planes.device,
                        memory_format=torch.channels_last)
        c1, c2, c3 = self.c1[0], self.c2[0], self.tail
        nat.check(nat.lib.az_fast_trunk_gpu(
            nat.ptr(planes), nat.ptr(self.stem.w9), nat.ptr(self.stem.bias), nat.ptr(c1.wq),
            nat.ptr(c1.bias), nat.ptr(c2.wq), nat.ptr(c2.bias), nat.ptr(c3.wq), nat.ptr(c3.bias),
            nat.ptr(t), B, 64, c1.mode, nat.stream_ptr()), "az_fast_trunk_gpu")
        return t

    # AZ_FAST_GEMM (default on): the heads GEMM on az_heads_fast_gemm_gpu (fp16x2 MFMA, split
    # over AZ_FAST_GEMM_SPLITS = 8 slices of the 4,096 features) instead of torch.bmm (fp32)
    fast_gemm = os.environ.get("AZ_FAST_GEMM", "1") == "1"
    fast_gemm_splits = int(os.environ.get("AZ_FAST_GEMM_SPLITS", "8"))
    # boards per GEMM workgroup (32 R: each weight fragment feeds R row tiles)
    fast_gemm_tile = int(os.environ.get("AZ_FAST_GEMM_TILE", "32"))

    def evaluate_into(self, planes, priors, values, stem_done=False):
        """Leaf evaluation straight into the engine's buffers: priors float32 [B, 65]
        (softmax), values float32 [B] (tanh).  AlphaZeroNet on the HIP trunk runs both heads
        in one kernel (csrc/heads.hip); otherwise the module's heads + copies.  stem_done:
        the engine has run the stem into engine_stem's buffers (planes are then not read)."""
        if stem_done and not self._fused_heads_ready():
            raise RuntimeError("stem_done on a net without an engine stem")
        if self._fast_heads_ready():
            import az_native as nat

            B = planes.shape[0]
            fw = self._fw
            if self._fast_trunk_ready():
                t = self._fast_trunk(planes)
            else:
                t = self.tail(self._trunk(planes.view(B, 1, 8, 8)))
            hf = t.permute(0, 2, 3, 1).reshape(B, -1)  # a view of the channels-last output
            if "gq" in fw:
                S = fw["gS"]
                part = torch.empty(S, B, fw["ld"], dtype=torch.float32, device=hf.device)
                nat.check(nat.lib.az_heads_fast_gemm_gpu(
                    nat.ptr(hf), nat.ptr(fw["gq"]), nat.ptr(fw["g128"]), fw["gshift"],
                    nat.ptr(part), fw["ld"], S, fw["gR"], B, nat.stream_ptr()),
                    "az_heads_fast_gemm_gpu")
            else:
                S = fw["S"]
                part = torch.bmm(hf.view(B, S, -1).transpose(0, 1), fw["wk"])  # [S, B, ld]
            nat.check(nat.lib.az_heads_fast_finish_gpu(
                nat.ptr(part), fw["ld"], S, nat.ptr(fw["bias"]), nat.ptr(fw["w2"]),
                nat.ptr(fw["b2"]), nat.ptr(priors), nat.ptr(values), B, nat.stream_ptr()),
                "az_heads_fast_finish_gpu")
            return
        if not self._fused_heads_ready():
            p, v = self.evaluate_planes(planes)
            priors.copy_(p)
            values.copy_(v)
            return
        import az_native as nat

        B = planes.shape[0]
        h = self._trunk(planes.view(B, 1, 8, 8), heads_into=(priors, values),
                        stem_done=stem_done)
        if h is None:  # the heads ran in the last conv's epilogue
            return
        hw = self._hw
        nat.check(nat.lib.az_heads_az_gpu(
            nat.ptr(h), nat.ptr(hw["wpv"]), nat.ptr(hw["bpv"]), nat.ptr(hw["wpolT"]),
            nat.ptr(hw["bpol"]), nat.ptr(hw["w1T"]), nat.ptr(hw["b1"]), nat.ptr(hw["w2"]),
            nat.ptr(hw["b2"]), nat.ptr(priors), nat.ptr(values), B, hw["C"], nat.stream_ptr()),
            "az_heads_az_gpu")

    def evaluate_planes(self, planes):
        if not (self._fused_heads_ready() or self._fast_heads_ready()):
            return Inference.evaluate_planes(self, planes)
        B = planes.shape[0]
        pr = torch.empty(B, 65, dtype=torch.float32, device=planes.device)
        va = torch.empty(B, dtype=torch.float32, device=planes.device)
        self.evaluate_into(planes.float(), pr, va)
        return pr, va

    def forward(self, x):
        h = self._trunk(x)
        B = h.shape[0]
        if self.kind == "az":
            y = self.heads(h)
            p = y[:, :self.n_pol].reshape(B, -1)
            v = y[:, self.n_pol:].reshape(B, -1)
            v = torch.tanh(self.val_fc2(F.relu(self.val_fc1(v))))
            return self.pol_fc(p), v
        h = self.tail(h).reshape(B, -1)
        v = torch.tanh(self.fc_value2(F.relu(self.fc_value1(h))))
        return self.fc_policy(h), v
