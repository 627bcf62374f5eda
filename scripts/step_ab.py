"""Same-box A/B of oth_step_gpu across library builds: every library given on the command
line is loaded side by side (ctypes, RTLD_LOCAL), run on the same 2^24 seeded corpus
positions, checked bit-identical to the first, and timed in interleaved rounds (400 untimed
launches past the power-management transient, then 200 timed, per round).

    python scripts/step_ab.py base.so new.so [...]
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    libs = sys.argv[1:]
    n = int(os.environ.get("N", 1 << 24))
    rounds = int(os.environ.get("ROUNDS", 3))
    d = np.load(os.path.join(ROOT, "tests", "golden", "board_corpus.npz"))
    pl = d["player"]
    own = np.where(pl == 1, d["pos"], d["neg"]).astype(np.uint64)
    opp = np.where(pl == 1, d["neg"], d["pos"]).astype(np.uint64)
    act = d["action"].astype(np.uint8)
    k = -(-n // len(own))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(np.tile(a, k)[:n])).cuda()
    ins = [t(own.view(np.int64)), t(opp.view(np.int64)), t(act)]
    stream = torch.cuda.current_stream().cuda_stream
    fns, outs = [], []
    for p in libs:
        L = ctypes.CDLL(os.path.abspath(p))
        f = L.oth_step_gpu
        f.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_int64, ctypes.c_void_p]
        f.restype = ctypes.c_int
        o = [torch.zeros(n, dtype=torch.int64, device="cuda") for _ in range(3)] + \
            [torch.zeros(n, dtype=torch.int16, device="cuda")]
        args = [x.data_ptr() for x in ins + o] + [n, stream]
        assert f(*args) == 0
        fns.append((f, args))
        outs.append(o)
    torch.cuda.synchronize()
    res = {p: {"ms": [], "same_as_first": all(bool((a == b).all()) for a, b in zip(outs[i], outs[0]))}
           for i, p in enumerate(libs)}
    for _ in range(rounds):
        for p, (f, args) in zip(libs, fns):
            for _ in range(400):
                f(*args)
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(200):
                f(*args)
            e1.record()
            torch.cuda.synchronize()
            res[p]["ms"].append(round(e0.elapsed_time(e1) / 200, 4))
    for p in libs:
        ms = min(res[p]["ms"])
        res[p]["best_frac_of_8TBps"] = round(43 * n / ms / 1e9 / 8.0, 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
