"""configs[1]'s evaluation by part, each alone: FastOthelloNet's one-launch trunk
(az_fast_trunk_gpu), the heads GEMM (az_heads_fast_gemm_gpu) and the finish kernel
(az_heads_fast_finish_gpu) at B boards, each replayed from a HIP graph of 20 launches; one
JSON line of median microseconds per launch over `reps` replays.
    python scripts/fast_parts_time.py [B] [reps]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402
from Models import FastOthelloNet, inference_copy  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
torch.manual_seed(0)
m = inference_copy(FastOthelloNet(8, 65).cuda().eval(), "cuda")
x = torch.randint(-1, 2, (B, 64), device="cuda").float()
pr = torch.empty(B, 65, device="cuda")
va = torch.empty(B, device="cuda")
with torch.no_grad():
    m.evaluate_into(x, pr, va)  # builds the prepared operands
    fw = m._fw
    t = m._fast_trunk(x)
    hf = t.permute(0, 2, 3, 1).reshape(B, -1)
    S = fw["gS"]
    part = torch.empty(S, B, fw["ld"], device="cuda")

    def trunk():
        c1, c2, c3 = m.c1[0], m.c2[0], m.tail
        nat.check(nat.lib.az_fast_trunk_gpu(
            nat.ptr(x), nat.ptr(m.stem.w9), nat.ptr(m.stem.bias), nat.ptr(c1.wq), nat.ptr(c1.bias),
            nat.ptr(c2.wq), nat.ptr(c2.bias), nat.ptr(c3.wq), nat.ptr(c3.bias), nat.ptr(t), B, 64,
            c1.mode, nat.stream_ptr()), "trunk")

    def gemm():
        nat.check(nat.lib.az_heads_fast_gemm_gpu(
            nat.ptr(hf), nat.ptr(fw["gq"]), nat.ptr(fw["g128"]), fw["gshift"], nat.ptr(part),
            fw["ld"], S, fw["gR"], B, nat.stream_ptr()), "gemm")

    def finish():
        nat.check(nat.lib.az_heads_fast_finish_gpu(
            nat.ptr(part), fw["ld"], S, nat.ptr(fw["bias"]), nat.ptr(fw["w2"]), nat.ptr(fw["b2"]),
            nat.ptr(pr), nat.ptr(va), B, nat.stream_ptr()), "finish")

    def whole():
        m.evaluate_into(x, pr, va)

    out = {"B": B, "lib": os.environ.get("AZ_LIB_PATH", "tree")}
    for name, fn in (("trunk", trunk), ("gemm", gemm), ("finish", finish), ("whole", whole)):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                fn()
        for _ in range(10):
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
        out[name + "_us"] = round(ts[len(ts) // 2], 2)
print(json.dumps(out), flush=True)
