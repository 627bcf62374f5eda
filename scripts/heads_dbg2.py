"""Debug: the separate heads kernel with two boards per workgroup (AZ_HEADS_NB2) vs four."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
from Models import AlphaZeroNet, FusedInferenceNet, inference_copy  # noqa: E402

torch.manual_seed(3)
net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
fused = inference_copy(net, "cuda")
FusedInferenceNet.fuse_heads = False
os.environ["AZ_W4_BOARDS"] = "4"
for B in (257, 1024, 1030, 4096):
    x = torch.randint(-1, 2, (B, 64), device="cuda").float()
    out = {}
    for nb2 in (False, True):
        if nb2:
            os.environ["AZ_HEADS_NB2"] = "1"
        else:
            os.environ.pop("AZ_HEADS_NB2", None)
        for rep in range(3):
            pr = torch.full((B, 65), float("nan"), device="cuda")
            va = torch.full((B,), float("nan"), device="cuda")
            with torch.no_grad():
                fused.evaluate_into(x, pr, va)
            torch.cuda.synchronize()
            out[(nb2, rep)] = (pr.clone(), va.clone())
    base = out[(False, 0)]
    for k, (pr, va) in out.items():
        dv = (va != base[1]).nonzero().flatten().tolist()
        dp = (pr != base[0]).any(dim=1).nonzero().flatten().tolist()
        print(B, k, "values differ:", len(dv), dv[:10], "priors differ:", len(dp), "max |dv|", (va - base[1]).abs().max().item(), flush=True)
