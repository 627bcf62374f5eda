"""Stress check of the persistent fp16x2 trunk (az_trunk_wino4_gpu: two-board workgroups,
two per CU, each carrying its boards through the block convs with only a workgroup barrier
between layers): many evaluations compared bit for bit against one launch per conv
(FusedInferenceNet.fuse_trunk4 = False) -- priors, values and the tower output -- on several
random positions batches, full and ragged."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
from Models import AlphaZeroNet, FusedInferenceNet, inference_copy  # noqa: E402


def main():
    reps = int(os.environ.get("REPS", 50))
    torch.manual_seed(11)
    net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
    fused = inference_copy(net, "cuda")
    res = {}
    for B in (1024, 1030, 512):
        for seed in range(3):
            torch.manual_seed(100 * B + seed)
            x = torch.randint(-1, 2, (B, 64), device="cuda").float()

            def run(flag):
                FusedInferenceNet.fuse_trunk4 = flag
                pr = torch.full((B, 65), float("nan"), device="cuda")
                va = torch.full((B,), float("nan"), device="cuda")
                with torch.no_grad():
                    fused.evaluate_into(x, pr, va)
                    h = fused._trunk(x.view(B, 1, 8, 8)).clone()
                return pr, va, h

            ref = run(False)
            bad = 0
            for _ in range(reps):
                got = run(True)
                bad += int(not all(torch.equal(a, b) for a, b in zip(got, ref)))
            torch.cuda.synchronize()
            assert not torch.isnan(ref[0]).any()
            res[f"B{B}_s{seed}"] = {"evaluations": reps, "mismatches": bad}
            print(B, seed, bad, flush=True)
    FusedInferenceNet.fuse_trunk4 = True
    print(json.dumps(res))


if __name__ == "__main__":
    main()
