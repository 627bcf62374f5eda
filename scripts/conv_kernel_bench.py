"""Standalone driver of the trunk conv (az_conv3x3_wino_gpu, split3, C = 128, B = 1,024 with
residual + ReLU: the bench's dominant kernel) for rocprofv3 counter passes, plus the same
calibration copy as scripts/step_kernel_bench.py (torch copy_ of 2 x 256 MiB)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda")
    from Models import inference_copy

    net = inference_copy(bench.make_net("az5x128").to(dev).eval(), dev, conv="hip",
                         precision="split3", conv_algo="wino")
    import az_native as nat

    conv = net.c2[0]
    B, C = 1024, conv.channels
    x = torch.randn(B, C, 8, 8, device=dev).relu().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x).relu().contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(x)
    args = [nat.ptr(x), nat.ptr(conv.wq), nat.ptr(conv.bias), nat.ptr(r), nat.ptr(y), B, C, 1,
            conv.mode, nat.stream_ptr()]
    for _ in range(reps):
        nat.check(nat.lib.az_conv3x3_wino_gpu(*args), "az_conv3x3_wino_gpu")
    a = torch.empty(64 << 20, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    print("ok", B, C, reps)


if __name__ == "__main__":
    main()
