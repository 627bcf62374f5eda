"""Per-phase timeline of the four-board Winograd conv from an AZ_W4_STAMP build (any
mode: split3 / fp16 / fp16x2; an AZ_W4_EXP ablation build shows the clock of that loop)
(AZ_LIB_PATH=expbuild/stamp/libaz_othello.so): prologue, the four transform-grid rows,
epilogue; medians over workgroups of one launch after warm-up launches, in microseconds,
and the in-kernel clock."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402


def main():
    mode_name = sys.argv[1] if len(sys.argv) > 1 else "split3"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    mode = {"split3": nat.AZ_CONV_SPLIT3, "fp16": nat.AZ_CONV_FP16,
            "fp16x2": nat.AZ_CONV_FP16X2}[mode_name]
    dev = torch.device("cuda")
    C = 128
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(dev)
    bias = torch.randn(C, generator=g).to(dev)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    wq = torch.empty(nat.lib.az_conv3x3_wino_prep_bytes(C, mode) // 2, dtype=torch.int16,
                     device=dev)
    nat.check(nat.lib.az_conv3x3_wino_prep_gpu(nat.ptr(w9), nat.ptr(wq), C, mode, nat.stream_ptr()), "prep")
    x = torch.randn(B, C, 8, 8, device=dev).relu().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x).relu().contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(x)
    from Models import board_absmax
    amax = board_absmax(x)
    work = amax.clone()
    for _ in range(300):
        work.copy_(amax)  # FP16X2 consumes the input ranges
        nat.check(nat.lib.az_conv3x3_wino4_gpu(nat.ptr(x), nat.ptr(wq), nat.ptr(bias), nat.ptr(r),
                                               nat.ptr(y), B, C, 1, mode, nat.ptr(work), None,
                                               nat.stream_ptr()), "w4")
    torch.cuda.synchronize()
    n = 1024 * 16
    buf = (ctypes.c_ulonglong * n)()
    f = nat.lib.az_w4_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nat.check(f(ctypes.addressof(buf), n), "az_w4_stamps")
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8, 2).astype(np.float64)
    wgs = min(1024, (B + 3) // 4)
    a = a[:wgs]
    cyc, rt = a[:, :, 0], a[:, :, 1]  # s_memtime (shader clock), s_memrealtime (100 MHz)
    d_rt = np.diff(rt[:, :7], axis=1) / 100.0  # microseconds
    clk = (cyc[:, 6] - cyc[:, 0]) / ((rt[:, 6] - rt[:, 0]) / 100.0) / 1e3  # GHz
    names = ["prologue", "row0", "row1", "row2", "row3", "epilogue"]
    span = (rt[:, 6].max() - rt[:, 0].min()) / 100.0
    print(json.dumps({"mode": mode_name, "boards": B, "workgroups": int(wgs),
                      "median_us": {k: round(float(np.median(d_rt[:, i])), 2) for i, k in enumerate(names)},
                      "wg_total_median_us": round(float(np.median((rt[:, 6] - rt[:, 0]) / 100.0)), 2),
                      "launch_span_us": round(float(span), 2),
                      "start_spread_us": round(float((rt[:, 0].max() - rt[:, 0].min()) / 100.0), 2),
                      "clock_ghz_median": round(float(np.median(clk)), 3)}))


if __name__ == "__main__":
    main()
