"""A/B of the trunk conv kernels at the bench's batch (same weights, same inputs): the
two-board Winograd form (az_conv3x3_wino_gpu), the four-board form (az_conv3x3_wino4_gpu,
also in FP16X2) and the direct form (az_conv3x3_mx_gpu), timed with a HIP event pair per
launch after 400 untimed launches (past the power-management transient).  One JSON line per
(kernel, mode, batch) with the max |difference| against the split3 two-board form."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402
from Models import board_absmax  # noqa: E402

MODES = {"split3": nat.AZ_CONV_SPLIT3, "fp16": nat.AZ_CONV_FP16, "fp16x2": nat.AZ_CONV_FP16X2}
CASES = [("az_conv3x3_wino_gpu", "split3"), ("az_conv3x3_wino4_gpu", "split3"),
         ("az_conv3x3_wino4_gpu", "fp16x2"), ("az_conv3x3_mx_gpu", "split3"),
         ("az_conv3x3_wino_gpu", "fp16"), ("az_conv3x3_wino4_gpu", "fp16"),
         ("az_conv3x3_mx_gpu", "fp16")]


def main():
    dev = torch.device("cuda")
    C = 128
    batches = [int(b) for b in (sys.argv[1:] or ["1024", "4096"])]
    only = os.environ.get("CONV_AB_ONLY")  # e.g. "wino4"
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(dev)
    bias = torch.randn(C, generator=g).to(dev)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    wq = {}
    for mname, mode in MODES.items():
        t = torch.empty(nat.lib.az_conv3x3_wino_prep_bytes(C, mode) // 2, dtype=torch.int16, device=dev)
        nat.check(nat.lib.az_conv3x3_wino_prep_gpu(nat.ptr(w9), nat.ptr(t), C, mode, nat.stream_ptr()), "prep")
        wq[("wino", mname)] = t
        if mode != nat.AZ_CONV_FP16X2:
            planes = 3 if mode == nat.AZ_CONV_SPLIT3 else 1
            t = torch.empty(9 * C * C * planes, dtype=torch.int16, device=dev)
            nat.check(nat.lib.az_conv3x3_mx_prep_gpu(nat.ptr(w9), nat.ptr(t), C, mode, nat.stream_ptr()), "prep")
            wq[("direct", mname)] = t
    for B in batches:
        torch.manual_seed(B)  # the same inputs in every run (y_sha compares builds)
        x = torch.randn(B, C, 8, 8, device=dev).relu().contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x).relu().contiguous(memory_format=torch.channels_last)
        amax = board_absmax(x)
        base = None
        cases = [(n, m, True) for n, m in CASES]
        cases += [(n, m, False) for n, m in CASES if "wino4" in n]  # also without residual
        for name, mname, with_res in cases:
            if only and only not in name:
                continue
            mode = MODES[mname]
            y = torch.empty_like(x)
            fn = getattr(nat.lib, name)
            args = [nat.ptr(x), nat.ptr(wq[("direct" if "mx" in name else "wino", mname)]),
                    nat.ptr(bias), nat.ptr(r) if with_res else None, nat.ptr(y), B, C, 1, mode]
            if "wino4" in name:
                # fp16x2 consumes in_absmax: give every launch a fresh copy (a device copy
                # beside the timed kernel, the same in every timed launch)
                work = amax.clone()
                args += [nat.ptr(work), None]

                def launch():
                    work.copy_(amax)
                    return fn(*args, nat.stream_ptr())
            else:
                def launch():
                    return fn(*args, nat.stream_ptr())
            for _ in range(400):
                nat.check(launch(), name)
            torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(100)]
            for e0, e1 in evs:
                if "wino4" in name:
                    work.copy_(amax)  # outside the timed pair
                e0.record()
                fn(*args, nat.stream_ptr())
                e1.record()
            torch.cuda.synchronize()
            ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / len(evs)
            import hashlib

            y_sha = hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest()[:16]
            if not with_res:
                y = y + r  # compare the residual-free form on the same footing (ReLU aside)
            if base is None:
                base = y.clone()
            flop = 2.0 * B * 64 * C * C * 9
            print(json.dumps({"kernel": name, "mode": mname, "boards": B, "residual": with_res,
                              "avg_launch_us": round(ms * 1e3, 2),
                              "algorithmic_tflops": round(flop / (ms * 1e-3) / 1e12, 1),
                              "max_abs_diff_vs_first": float((y - base).abs().max()),
                              "y_sha": y_sha, "lib": os.environ.get("AZ_LIB_PATH", "product")}),
                  flush=True)


if __name__ == "__main__":
    main()
