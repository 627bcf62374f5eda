"""k_heads_az time per launch (az_heads_az_gpu, AlphaZeroNet 5x128 random init, 20 launches
per HIP graph replayed back to back, HIP events on the launch stream) at a search's batch
sizes.  One JSON line.

    python scripts/heads_time.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402
from Models import AlphaZeroNet, inference_copy  # noqa: E402


def main():
    torch.manual_seed(0)
    net = inference_copy(AlphaZeroNet(8, 65, 5, 128).cuda().eval(), "cuda")
    assert net._fused_heads_ready()
    hw = net._hw
    out = {}
    for B in (4, 64, 1024, 4096):
        h = torch.randn(B, 128, 8, 8, device="cuda").relu().contiguous(
            memory_format=torch.channels_last)
        pri = torch.empty(B, 65, device="cuda")
        val = torch.empty(B, device="cuda")

        def call():
            nat.check(nat.lib.az_heads_az_gpu(
                nat.ptr(h), nat.ptr(hw["wpv"]), nat.ptr(hw["bpv"]), nat.ptr(hw["wpolT"]),
                nat.ptr(hw["bpol"]), nat.ptr(hw["w1T"]), nat.ptr(hw["b1"]), nat.ptr(hw["w2"]),
                nat.ptr(hw["b2"]), nat.ptr(pri), nat.ptr(val), B, 128, nat.stream_ptr()),
                "az_heads_az_gpu")
        call()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                call()
        g.replay()
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(50):
            g.replay()
        e1.record(s)
        torch.cuda.synchronize()
        out[f"us_B{B}"] = round(e0.elapsed_time(e1) * 1e3 / 1000, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
