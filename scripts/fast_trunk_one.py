"""FastOthelloNet's one-launch trunk (az_fast_trunk_gpu) launched `n` times eagerly at B boards,
for rocprofv3 --pmc passes (one dispatch per launch):
    python scripts/fast_trunk_one.py [B] [n]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
from Models import FastOthelloNet, inference_copy  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.manual_seed(0)
m = inference_copy(FastOthelloNet(8, 65).cuda().eval(), "cuda")
assert m._fast_trunk_ready()
x = torch.randint(-1, 2, (B, 64), device="cuda").float()
with torch.no_grad():
    for _ in range(n):
        m._fast_trunk(x)
torch.cuda.synchronize()
print("ok", B, n)
