"""Run one trunk-conv kernel `reps` times (for rocprofv3 counter passes):
    python scripts/conv_one.py az_conv3x3_wino4_gpu split3 1024 20"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402


def main():
    name, mode_name, B, reps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    mode = {"split3": nat.AZ_CONV_SPLIT3, "fp16": nat.AZ_CONV_FP16}[mode_name]
    dev = torch.device("cuda")
    C = 128
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(dev)
    bias = torch.randn(C, generator=g).to(dev)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    planes = 3 if mode == nat.AZ_CONV_SPLIT3 else 1
    direct = name == "az_conv3x3_mx_gpu"
    wq = torch.empty((9 if direct else 16) * C * C * planes, dtype=torch.int16, device=dev)
    prep = nat.lib.az_conv3x3_mx_prep_gpu if direct else nat.lib.az_conv3x3_wino_prep_gpu
    nat.check(prep(nat.ptr(w9), nat.ptr(wq), C, mode, nat.stream_ptr()), "prep")
    x = torch.randn(B, C, 8, 8, device=dev).relu().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x).relu().contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(x)
    fn = getattr(nat.lib, name)
    for _ in range(reps):
        nat.check(fn(nat.ptr(x), nat.ptr(wq), nat.ptr(bias), nat.ptr(r), nat.ptr(y), B, C, 1, mode,
                     nat.stream_ptr()), name)
    torch.cuda.synchronize()
    print("ok", name, mode_name, B, reps)


if __name__ == "__main__":
    main()
