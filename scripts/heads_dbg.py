"""Debug: fused heads (2- / 4-board workgroups) against the separate heads kernel, per board."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
from Models import AlphaZeroNet, FusedInferenceNet, inference_copy  # noqa: E402

torch.manual_seed(3)
net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
fused = inference_copy(net, "cuda")
for B in (257, 1024, 1030):
    x = torch.randint(-1, 2, (B, 64), device="cuda").float()
    out = {}
    for boards in ("2", "4"):
        os.environ["AZ_W4_BOARDS"] = boards
        for flag in (True, False):
            FusedInferenceNet.fuse_heads = flag
            pr = torch.full((B, 65), float("nan"), device="cuda")
            va = torch.full((B,), float("nan"), device="cuda")
            with torch.no_grad():
                fused.evaluate_into(x, pr, va)
            torch.cuda.synchronize()
            out[(boards, flag)] = (pr.clone(), va.clone())
    base = out[("4", False)]
    for k, (pr, va) in out.items():
        dv = (va != base[1]).nonzero().flatten().tolist()
        dp = (pr != base[0]).any(dim=1).nonzero().flatten().tolist()
        print(B, k, "value boards differing:", len(dv), dv[:12], "prior boards differing:", len(dp), dp[:12],
              "max |dv|", (va - base[1]).abs().max().item())
