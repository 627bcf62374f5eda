"""Stress check of the two-board conv workgroups: many launches at batch sizes where two
workgroups share each CU, outputs and per-board max |y| compared bit for bit against the
four-board form (AZ_W4_BOARDS=4), fp16x2 and fp16, with and without a residual."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402
from Models import board_absmax  # noqa: E402


def main():
    C = 128
    reps = int(os.environ.get("REPS", 100))
    g = torch.Generator().manual_seed(7)
    w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).cuda()
    bias = torch.randn(C, generator=g).cuda()
    w9 = w.permute(2, 3, 0, 1).reshape(9, C, C).contiguous()
    res = {}
    for mname, mode in (("fp16x2", nat.AZ_CONV_FP16X2), ("fp16", nat.AZ_CONV_FP16)):
        wq = torch.empty(nat.lib.az_conv3x3_wino_prep_bytes(C, mode) // 2, dtype=torch.int16, device="cuda")
        nat.check(nat.lib.az_conv3x3_wino_prep_gpu(nat.ptr(w9), nat.ptr(wq), C, mode, nat.stream_ptr()), "prep")
        for B in (1024, 1030, 4096):
            torch.manual_seed(B)
            x = torch.randn(B, C, 8, 8, device="cuda").relu().contiguous(memory_format=torch.channels_last)
            r = torch.randn_like(x).relu().contiguous(memory_format=torch.channels_last)
            for with_res in (True, False):
                def run():
                    y = torch.empty_like(x)
                    am = torch.zeros(B, device="cuda")
                    nat.check(nat.lib.az_conv3x3_wino4_gpu(
                        nat.ptr(x), nat.ptr(wq), nat.ptr(bias), nat.ptr(r) if with_res else None,
                        nat.ptr(y), B, C, 1, mode, nat.ptr(board_absmax(x)), nat.ptr(am),
                        nat.stream_ptr()), "conv")
                    return y, am
                os.environ["AZ_W4_BOARDS"] = "4"
                y4, a4 = run()
                os.environ["AZ_W4_BOARDS"] = "2"
                bad = 0
                for _ in range(reps):
                    y2, a2 = run()
                    bad += int(not (torch.equal(y2, y4) and torch.equal(a2, a4)))
                torch.cuda.synchronize()
                res[f"{mname}_{B}_{'res' if with_res else 'nores'}"] = {"launches": reps, "mismatches": bad}
                print(mname, B, with_res, bad, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
