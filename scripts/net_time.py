"""Time the bench's leaf evaluation (AlphaZeroNet 5x128 inference copy: persistent fp16x2
trunk + heads-fused last conv) at B boards, replayed from a HIP graph of 20 evaluations on
random positions; the library is AZ_LIB_PATH's (experiment builds) or the tree's.  One JSON
line: median / min microseconds per evaluation over `reps` replays.
    python scripts/net_time.py [B] [reps] [fp16|fast]   (fp16: configs[4]'s fp16 inference copy;
    fast: configs[1]'s FastOthelloNet inference copy)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
from Models import AlphaZeroNet, FastOthelloNet, inference_copy  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
torch.manual_seed(0)
mode = sys.argv[3] if len(sys.argv) > 3 else ""
net = (FastOthelloNet(8, 65) if mode == "fast" else AlphaZeroNet(8, 65, 5, 128)).cuda().eval()
fp16 = mode == "fp16"
m = inference_copy(net, "cuda", dtype=torch.float16) if fp16 else inference_copy(net, "cuda")
x = torch.randint(-1, 2, (B, 64), device="cuda").float()
pr = torch.empty(B, 65, device="cuda")
va = torch.empty(B, device="cuda")
with torch.no_grad():
    for _ in range(3):
        m.evaluate_into(x, pr, va)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            m.evaluate_into(x, pr, va)
    for _ in range(20):  # past the power-management transient
        g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
ts.sort()
print(json.dumps({"lib": os.environ.get("AZ_LIB_PATH", "tree"), "B": B, "net": mode or "az",
                  "heads_boards": os.environ.get("AZ_W4_HEADS_BOARDS", "2"),
                  "us_median": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2),
                  "prior_sum": round(float(pr.sum()), 6), "value_sum": round(float(va.sum()), 6)}),
      flush=True)
