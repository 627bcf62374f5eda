"""A/B of the trunk conv kernels at the bench's batch (same weights, same inputs): the
two-board Winograd form (az_conv3x3_wino_gpu), the four-board form (az_conv3x3_wino4_gpu)
and the direct form (az_conv3x3_mx_gpu), split3 and fp16, timed with a HIP event pair per
launch after 400 untimed launches (past the power-management transient).  One JSON line per
(kernel, mode, batch), plus the max |difference| against the two-board form."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402
import bench  # noqa: E402


def main():
    dev = torch.device("cuda")
    C = 128
    batches = [int(b) for b in (sys.argv[1:] or ["1024", "4096"])]
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(dev)
    bias = torch.randn(C, generator=g).to(dev)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    for mode_name, mode in (("split3", nat.AZ_CONV_SPLIT3), ("fp16", nat.AZ_CONV_FP16)):
        planes = 3 if mode == nat.AZ_CONV_SPLIT3 else 1
        wqw = torch.empty(16 * C * C * planes, dtype=torch.int16, device=dev)
        nat.check(nat.lib.az_conv3x3_wino_prep_gpu(nat.ptr(w9), nat.ptr(wqw), C, mode,
                                                   nat.stream_ptr()), "prep")
        wqd = torch.empty(9 * C * C * planes, dtype=torch.int16, device=dev)
        nat.check(nat.lib.az_conv3x3_mx_prep_gpu(nat.ptr(w9), nat.ptr(wqd), C, mode,
                                                 nat.stream_ptr()), "prep")
        for B in batches:
            x = torch.randn(B, C, 8, 8, device=dev).relu().contiguous(memory_format=torch.channels_last)
            r = torch.randn_like(x).relu().contiguous(memory_format=torch.channels_last)
            outs = {}
            for name, wq in (("az_conv3x3_wino_gpu", wqw), ("az_conv3x3_wino4_gpu", wqw),
                             ("az_conv3x3_mx_gpu", wqd)):
                y = torch.empty_like(x)
                fn = getattr(nat.lib, name)
                args = [nat.ptr(x), nat.ptr(wq), nat.ptr(bias), nat.ptr(r), nat.ptr(y), B, C, 1,
                        mode, nat.stream_ptr()]
                for _ in range(400):
                    nat.check(fn(*args), name)
                torch.cuda.synchronize()
                ms = bench.launch_ms(lambda: fn(*args), 100)
                outs[name] = y
                flop = 2.0 * B * 64 * C * C * 9
                print(json.dumps({"kernel": name, "mode": mode_name, "boards": B,
                                  "avg_launch_us": round(ms * 1e3, 2),
                                  "algorithmic_tflops": round(flop / (ms * 1e-3) / 1e12, 1),
                                  "max_abs_diff_vs_wino": float((y - outs["az_conv3x3_wino_gpu"]).abs().max())}),
                      flush=True)


if __name__ == "__main__":
    main()
