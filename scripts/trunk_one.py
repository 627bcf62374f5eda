"""Run the persistent fp16x2 trunk (az_trunk_wino4_gpu: the 10 block convs of AlphaZeroNet 5x128,
two-board workgroups) `reps` times on random post-ReLU activations, B boards (rocprofv3 counter
passes; counters per dispatch / 10 = per conv):
    python scripts/trunk_one.py 1024 20 [calib]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
from Models import AlphaZeroNet, board_absmax, inference_copy  # noqa: E402

B, reps = int(sys.argv[1]), int(sys.argv[2])
torch.manual_seed(0)
m = inference_copy(AlphaZeroNet(8, 65, 5, 128).cuda().eval(), "cuda")
c1s, c2s = list(m.c1), list(m.c2)
assert m._trunk4_ready(c1s, c2s, B)
x = torch.randn(B, 128, 8, 8, device="cuda").relu().contiguous(memory_format=torch.channels_last)
bufs = m._scratch(x.device, B)["absmax"]
with torch.no_grad():
    for _ in range(reps):
        board_absmax(x, out=bufs[0])
        bufs[1].zero_()
        m._trunk4(x, bufs, c1s, c2s, None)
if len(sys.argv) > 3 and sys.argv[3] == "calib":
    a = torch.empty(64 << 20, dtype=torch.float32, device="cuda")
    torch.empty_like(a).copy_(a)
torch.cuda.synchronize()
