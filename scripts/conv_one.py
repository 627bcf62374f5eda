"""Run one trunk-conv kernel `reps` times (for rocprofv3 counter passes):
    python scripts/conv_one.py az_conv3x3_wino4_gpu split3 1024 20 [calib]
With `calib`, a torch copy_ of 2 x 256 MiB follows (the HBM-counter calibration of
scripts/step_kernel_bench.py: 268,435,456 bytes read + written)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402


def main():
    name, mode_name, B, reps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    mode = {"split3": nat.AZ_CONV_SPLIT3, "fp16": nat.AZ_CONV_FP16,
            "fp16x2": nat.AZ_CONV_FP16X2}[mode_name]
    dev = torch.device("cuda")
    C = 128
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(dev)
    bias = torch.randn(C, generator=g).to(dev)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    planes = 3 if mode == nat.AZ_CONV_SPLIT3 else 1
    direct = name == "az_conv3x3_mx_gpu"
    nbytes = (9 * C * C * planes * 2 if direct else nat.lib.az_conv3x3_wino_prep_bytes(C, mode))
    wq = torch.empty(nbytes // 2, dtype=torch.int16, device=dev)
    prep = nat.lib.az_conv3x3_mx_prep_gpu if direct else nat.lib.az_conv3x3_wino_prep_gpu
    nat.check(prep(nat.ptr(w9), nat.ptr(wq), C, mode, nat.stream_ptr()), "prep")
    x = torch.randn(B, C, 8, 8, device=dev).relu().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x).relu().contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(x)
    fn = getattr(nat.lib, name)
    args = [nat.ptr(x), nat.ptr(wq), nat.ptr(bias), nat.ptr(r), nat.ptr(y), B, C, 1, mode]
    amax = work = None
    if "wino4" in name:
        from Models import board_absmax
        amax = board_absmax(x)
        work = amax.clone()
        args += [nat.ptr(work), None]
    for _ in range(reps):
        if work is not None:
            work.copy_(amax)  # the kernel consumes (zeroes) its in_absmax
        nat.check(fn(*args, nat.stream_ptr()), name)
    if len(sys.argv) > 5 and sys.argv[5] == "calib":
        a = torch.empty(64 << 20, dtype=torch.float32, device=dev)
        b = torch.empty_like(a)
        b.copy_(a)
    torch.cuda.synchronize()
    print("ok", name, mode_name, B, reps)


if __name__ == "__main__":
    main()
