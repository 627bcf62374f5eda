"""Standalone driver of the bitboard-step kernel (oth_step_gpu) for rocprofv3 counter
passes: N positions resident in HBM, R launches, plus a calibration copy of a known byte
count (torch copy_ of 2 x 256 MiB) so FETCH_SIZE / WRITE_SIZE can be read against known
traffic on this GPU.  Positions: reachable boards from the golden corpus (random playouts),
each with a legal action (or pass), tiled to N."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-othello_amd"))
import az_native as nat  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    d = np.load(os.path.join(ROOT, "tests", "golden", "board_corpus.npz"))
    pl = d["player"]
    own = np.where(pl == 1, d["pos"], d["neg"]).astype(np.uint64)
    opp = np.where(pl == 1, d["neg"], d["pos"]).astype(np.uint64)
    act = d["action"].astype(np.uint8)
    k = -(-n // len(own))
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(np.tile(a, k)[:n])).to(dev)
    d_own, d_opp, d_act = t(own.view(np.int64)), t(opp.view(np.int64)), t(act)
    outs = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(3)]
    st = torch.empty(n, dtype=torch.int16, device=dev)
    args = [nat.ptr(d_own), nat.ptr(d_opp), nat.ptr(d_act)] + [nat.ptr(x) for x in outs] + \
        [nat.ptr(st), n, nat.stream_ptr()]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    nat.check(nat.lib.oth_step_gpu(*args), "oth_step_gpu")
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        nat.lib.oth_step_gpu(*args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    # calibration: a plain device copy of 256 MiB (read 256 MiB, write 256 MiB)
    a = torch.empty(64 << 20, dtype=torch.float32, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    print(f"oth_step_gpu n={n} avg_ms={ms:.4f} gsteps_per_s={n / ms / 1e6:.2f} "
          f"alg_GBps={43 * n / ms / 1e6:.1f} calib_copy_bytes={a.numel() * 4}")


if __name__ == "__main__":
    main()
