"""Per-layer timeline of the persistent trunk from an AZ_W4_TSTAMP build
(AZ_LIB_PATH=expbuild/tstamp/libaz_othello.so): the configs[2] net evaluated at B boards
(scripts/net_time.py's setup), then per layer the medians over workgroups of the prologue
(layer start -> first chunk), the K loop up to the first epilogue, the rest (two groups'
tail, epilogues), and the gap to the next layer's start (layer fence), in microseconds at
the clock s_memtime counts (100 MHz realtime is not stamped: cycles / 2.1 GHz shown too)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402
from Models import AlphaZeroNet, inference_copy  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
torch.manual_seed(0)
net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
m = inference_copy(net, "cuda")
x = torch.randint(-1, 2, (B, 64), device="cuda").float()
pr = torch.empty(B, 65, device="cuda")
va = torch.empty(B, device="cuda")
with torch.no_grad():
    for _ in range(200):
        m.evaluate_into(x, pr, va)
    torch.cuda.synchronize()
n = 1024 * 16 * 4
buf = (ctypes.c_ulonglong * n)()
nat.lib.az_w4_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
nat.check(nat.lib.az_w4_tstamps(ctypes.addressof(buf), n), "az_w4_tstamps")
t = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(1024, 16, 4)
wgs = (B + 1) // 2
t = t[:wgs]
L = int((t[:, :, 0] > 0).sum(axis=1).max())
out = {"B": B, "workgroups": wgs, "layers": L, "per_layer_cycles": []}
start = t[:, 0, 0].min()
for i in range(L):
    row = t[:, i]
    d = {"prologue": np.median(row[:, 1] - row[:, 0]), "groups_0_2": np.median(row[:, 2] - row[:, 1]),
         "group_3_epilogues": np.median(row[:, 3] - row[:, 2])}
    if i + 1 < L:
        d["fence_to_next"] = np.median(t[:, i + 1, 0] - row[:, 3])
    d["layer_start_spread"] = float(np.percentile(row[:, 0] - start, 95) - np.percentile(row[:, 0] - start, 5))
    out["per_layer_cycles"].append({k: round(float(v), 0) for k, v in d.items()})
tot = t[:, L - 1, 3] - t[:, 0, 0]
out["trunk_cycles_median"] = float(np.median(tot))
out["trunk_cycles_max"] = float(tot.max())
print(json.dumps(out, indent=1))
