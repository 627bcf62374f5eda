"""Time the fused MFMA conv (every tiling candidate) against MIOpen at the bench's batch;
check each candidate against F.conv2d first."""
import os, sys, json
import torch
import torch.nn.functional as F
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-othello_amd"))
import az_native as nat  # noqa: E402

CFGS = {128: [0, 1, 2, 3, 4, 5], 64: [0, 1, 2]}


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
    ref = F.relu(F.conv2d(x.contiguous(), w, b, padding=1) + r)
    fl = 2.0 * B * 64 * C * C * 9
    out = {"B": B, "C": C}
    wl = w.contiguous(memory_format=torch.channels_last)
    ms = timed(lambda: F.conv2d(x, wl, None, padding=1))
    out["miopen_us"] = round(ms * 1e3, 1)
    out["miopen_tf"] = round(fl / ms / 1e9, 1)
    for cfg in CFGS[C]:
        y = torch.empty_like(x)
        args = [nat.ptr(x), nat.ptr(w9), nat.ptr(b), nat.ptr(r), nat.ptr(y), B, C, 1, cfg, nat.stream_ptr()]
        nat.check(nat.lib.az_conv3x3_cfg_gpu(*args), "conv")
        torch.cuda.synchronize()
        ok = bool(torch.allclose(y, ref, atol=2e-5, rtol=2e-5))
        ms = timed(lambda: nat.lib.az_conv3x3_cfg_gpu(*args))
        out[f"cfg{cfg}"] = {"us": round(ms * 1e3, 1), "tf": round(fl / ms / 1e9, 1), "ok": ok}
    return out


for B in (1024, 4096):
    for C in (128, 64):
        print(json.dumps(run(B, C)), flush=True)
