"""Time the 16-bit MFMA conv (split3 = fp32-accurate, fp16) against the fp32 MFMA kernel and
MIOpen at the bench's batch; report max |err| vs fp64 for each."""
import os, sys, json
import torch
import torch.nn.functional as F
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-othello_amd"))
import az_native as nat  # noqa: E402


def timed(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def run(B, C):
    x = torch.randn(B, C, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x).contiguous(memory_format=torch.channels_last)
    w = torch.randn(C, C, 3, 3, device="cuda") / (3 * C ** 0.5)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    b = torch.randn(C, device="cuda")
    ref = F.relu(F.conv2d(x.double(), w.double(), b.double(), padding=1) + r.double())
    fl = 2.0 * B * 64 * C * C * 9
    out = {"B": B, "C": C}
    y = torch.empty_like(x)
    a32 = [nat.ptr(x), nat.ptr(w9), nat.ptr(b), nat.ptr(r), nat.ptr(y), B, C, 1, nat.stream_ptr()]
    nat.check(nat.lib.az_conv3x3_gpu(*a32), "conv"); torch.cuda.synchronize()
    ms = timed(lambda: nat.lib.az_conv3x3_gpu(*a32))
    out["fp32"] = {"us": round(ms * 1e3, 1), "tf": round(fl / ms / 1e9, 1),
                   "maxerr": float((y.double() - ref).abs().max())}
    for name, mode, cfg in (("split3", nat.AZ_CONV_SPLIT3, 0), ("split3_1b", nat.AZ_CONV_SPLIT3, 1),
                            ("fp16", nat.AZ_CONV_FP16, 0), ("fp16_1b", nat.AZ_CONV_FP16, 1)):
        planes = 3 if mode == nat.AZ_CONV_SPLIT3 else 1
        wq = torch.empty(9 * C * C * planes, dtype=torch.int16, device="cuda")
        nat.check(nat.lib.az_conv3x3_mx_prep_gpu(nat.ptr(w9), nat.ptr(wq), C, mode, nat.stream_ptr()), "prep")
        y = torch.empty_like(x)
        args = [nat.ptr(x), nat.ptr(wq), nat.ptr(b), nat.ptr(r), nat.ptr(y), B, C, 1, mode, cfg,
                nat.stream_ptr()]
        nat.check(nat.lib.az_conv3x3_mx_cfg_gpu(*args), name); torch.cuda.synchronize()
        err = float((y.double() - ref).abs().max())
        ms = timed(lambda: nat.lib.az_conv3x3_mx_cfg_gpu(*args))
        out[name] = {"us": round(ms * 1e3, 1), "tf_equiv": round(fl / ms / 1e9, 1), "maxerr": err}
    for name, mode in (("wino_split3", nat.AZ_CONV_SPLIT3), ("wino_fp16", nat.AZ_CONV_FP16)):
        planes = 3 if mode == nat.AZ_CONV_SPLIT3 else 1
        wq = torch.empty(16 * C * C * planes, dtype=torch.int16, device="cuda")
        nat.check(nat.lib.az_conv3x3_wino_prep_gpu(nat.ptr(w9), nat.ptr(wq), C, mode, nat.stream_ptr()), "prep")
        y = torch.empty_like(x)
        args = [nat.ptr(x), nat.ptr(wq), nat.ptr(b), nat.ptr(r), nat.ptr(y), B, C, 1, mode,
                nat.stream_ptr()]
        nat.check(nat.lib.az_conv3x3_wino_gpu(*args), name); torch.cuda.synchronize()
        err = float((y.double() - ref).abs().max())
        ms = timed(lambda: nat.lib.az_conv3x3_wino_gpu(*args))
        out[name] = {"us": round(ms * 1e3, 1), "tf_equiv": round(fl / ms / 1e9, 1), "maxerr": err}
    return out


for B in (1024, 4096):
    for C in (128, 64):
        print(json.dumps(run(B, C)), flush=True)
