"""Per-chunk timeline of the four-board Winograd conv from an AZ_W4_CSTAMP build
(AZ_LIB_PATH=expbuild/cstamp/libaz_othello.so): every wave's s_memtime at each chunk's
start, before its closing barrier and after it.  Reports, in shader cycles (medians over
the first 256 workgroups' waves of the last of 50 launches): the chunk period, the part a
wave spends before the barrier (issuing its MFMAs, transform, loads) and the barrier wait,
per chunk index and overall, plus the workgroup span.

    AZ_LIB_PATH=expbuild/cstamp/libaz_othello.so python scripts/w4_chunk_stamps.py fp16x2 1024
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402
from Models import board_absmax  # noqa: E402


def main():
    mode_name = sys.argv[1] if len(sys.argv) > 1 else "fp16x2"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    mode = {"split3": nat.AZ_CONV_SPLIT3, "fp16": nat.AZ_CONV_FP16,
            "fp16x2": nat.AZ_CONV_FP16X2}[mode_name]
    dev = torch.device("cuda")
    C = 128
    torch.manual_seed(0)
    w = (torch.randn(C, C, 3, 3) / (3 * C ** 0.5)).to(dev)
    bias = torch.randn(C).to(dev)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    wq = torch.empty(nat.lib.az_conv3x3_wino_prep_bytes(C, mode) // 2, dtype=torch.int16, device=dev)
    nat.check(nat.lib.az_conv3x3_wino_prep_gpu(nat.ptr(w9), nat.ptr(wq), C, mode, nat.stream_ptr()), "prep")
    x = torch.randn(B, C, 8, 8, device=dev).relu().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x).relu().contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(x)
    amax = board_absmax(x)
    work = amax.clone()
    args = [nat.ptr(x), nat.ptr(wq), nat.ptr(bias), nat.ptr(r), nat.ptr(y), B, C, 1, mode,
            nat.ptr(work), None, nat.stream_ptr()]
    for _ in range(50):
        work.copy_(amax)
        nat.check(nat.lib.az_conv3x3_wino4_gpu(*args), "conv")
    torch.cuda.synchronize()
    n = 256 * 8 * 32 * 3
    buf = (ctypes.c_ulonglong * n)()
    nat.lib.az_w4_cstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nat.check(nat.lib.az_w4_cstamps(ctypes.addressof(buf), n), "az_w4_cstamps")
    st = np.frombuffer(buf, dtype=np.uint64).reshape(256, 8, 32, 3).astype(np.int64)
    nwg = min(256, (B + 3) // 4)
    st = st[:nwg]
    period = st[:, :, 1:, 0] - st[:, :, :-1, 0]      # chunk start to next chunk start
    work_ = st[:, :, :, 1] - st[:, :, :, 0]          # start -> before the barrier
    wait = st[:, :, :, 2] - st[:, :, :, 1]           # the barrier
    span = st[:, :, -1, 2] - st[:, :, 0, 0]
    out = {"mode": mode_name, "boards": B, "workgroups": nwg,
           "median_period_cycles": float(np.median(period)),
           "median_pre_barrier_cycles": float(np.median(work_)),
           "median_barrier_wait_cycles": float(np.median(wait)),
           "median_chunks_span_cycles": float(np.median(span)),
           "per_chunk_period": [float(np.median(period[:, :, c])) for c in range(31)],
           "per_chunk_barrier_wait": [float(np.median(wait[:, :, c])) for c in range(32)],
           "per_wave_pre_barrier": [float(np.median(work_[:, wv, :])) for wv in range(8)],
           "per_wave_wait": [float(np.median(wait[:, wv, :])) for wv in range(8)]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
