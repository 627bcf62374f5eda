"""Run the bench's leaf evaluation launch eagerly (FusedInferenceNet.evaluate_into on random
canonical boards: az_trunk_wino4_heads_gpu = stem + every block conv + heads in one persistent
launch, as bench.py's roofline_trunk times it) `reps` times at B boards -- the program for the
rocprofv3 --pmc passes behind profiles/trunk_traffic.json:
    python scripts/trunk_heads_one.py 1024 20"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
from Models import AlphaZeroNet, inference_copy  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.manual_seed(0)
m = inference_copy(AlphaZeroNet(8, 65, 5, 128).cuda().eval(), "cuda")
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randint(-1, 2, (B, 64), generator=g).float().cuda()
pr = torch.empty(B, 65, device="cuda")
va = torch.empty(B, device="cuda")
with torch.no_grad():
    for _ in range(reps):
        m.evaluate_into(x, pr, va)
torch.cuda.synchronize()
print("ok", float(pr.sum()), float(va.sum()))
