"""Trunk conv time per launch at small batches: the one-pass fp16x2 kernel
(az_conv3x3_wino4_gpu) against the channel-split form (az_conv3x3_wino4_splitk_gpu, 2 / 4 /
8 / 16 / 32 splits, conv + combine), 128 channels, residual + ReLU, 20 launches per HIP graph
replayed back to back, timed with HIP events on the launch stream.  One JSON line per batch size.

    python scripts/splitk_sweep.py [reps]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402
from Models import board_absmax  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    dev = torch.device("cuda")
    C, mode = 128, nat.AZ_CONV_FP16X2
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(dev)
    bias = torch.randn(C, generator=g).to(dev)
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    wq = torch.empty(nat.lib.az_conv3x3_wino_prep_bytes(C, mode) // 2, dtype=torch.int16,
                     device=dev)
    nat.check(nat.lib.az_conv3x3_wino_prep_gpu(nat.ptr(w9), nat.ptr(wq), C, mode,
                                               nat.stream_ptr()), "prep")
    for B in (1, 4, 8, 16, 32, 64, 128, 256):
        x = torch.randn(B, C, 8, 8, device=dev).relu().contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x).relu().contiguous(memory_format=torch.channels_last)
        y = torch.empty_like(x)
        a0 = board_absmax(x)
        a1 = torch.zeros_like(a0)
        part = torch.empty(32 * x.numel(), device=dev)
        row = {"boards": B}
        for splits in (0, 2, 4, 8, 16, 32):
            def call(i):
                ai, ao = (a0, a1) if i % 2 == 0 else (a1, a0)
                base = [nat.ptr(x), nat.ptr(wq), nat.ptr(bias), nat.ptr(r), nat.ptr(y), B, C, 1,
                        mode, nat.ptr(ai), nat.ptr(ao)]
                if splits:
                    nat.check(nat.lib.az_conv3x3_wino4_splitk_gpu(*base, nat.ptr(part), splits,
                                                                  nat.stream_ptr()), "splitk")
                else:
                    nat.check(nat.lib.az_conv3x3_wino4_gpu(*base, nat.stream_ptr()), "wino4")
            for i in range(20):
                call(i)
            torch.cuda.synchronize()
            # 20 layers per HIP graph, as the engine replays them (no per-launch host cost)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for i in range(20):
                    call(i)
            graph.replay()
            torch.cuda.synchronize()
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps // 20):
                graph.replay()
            e1.record(s)
            torch.cuda.synchronize()
            row[f"us_splits{splits}"] = round(e0.elapsed_time(e1) * 1e3 / (reps // 20 * 20), 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
