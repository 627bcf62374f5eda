"""Time the policy/value net forward at the bench's leaf batch on the GPU, by variant:
plain eval module, BatchNorm-folded channels-last copy (what the engine runs), with
MIOpen find mode (cudnn.benchmark), and fp16 (config #5).  Prints one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-othello_amd"))
from Models import AlphaZeroNet, FastOthelloNet, inference_copy  # noqa: E402


def timeit(fn, x, reps=50):
    for _ in range(5):
        fn(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn(x)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def plain_p(net, x):
    return torch.softmax(net(x.view(-1, 1, 8, 8))[0], -1)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    dev = torch.device("cuda")
    torch.manual_seed(0)
    out = {"batch": B}
    for name, net in (("az5x128", AlphaZeroNet(8, 65, 5, 128)), ("fast", FastOthelloNet(8, 65))):
        x = torch.randint(-1, 2, (B, 64), device=dev).float()
        plain = net.to(dev).eval()
        r = {}
        with torch.no_grad():
            r["plain_ms"] = timeit(lambda t: plain(t.view(-1, 1, 8, 8)), x)
            fold = inference_copy(net, dev, fused=False)
            r["folded_cl_ms"] = timeit(fold.evaluate_planes, x)
            fused = inference_copy(net, dev, fused=True, conv="miopen")
            r["fused_ms"] = timeit(fused.evaluate_planes, x)
            hip = inference_copy(net, dev, fused=True, conv="hip")
            r["hipconv_ms"] = timeit(hip.evaluate_planes, x)
            c2 = hip.evaluate_planes(x)
            r["max_abs_prior_diff_hipconv"] = float((c2[0] - plain_p(plain, x)).abs().max())
            c = fused.evaluate_planes(x)
            b0 = fold.evaluate_planes(x)
            r["max_abs_prior_diff_fused"] = float((c[0] - b0[0]).abs().max())
            r["max_abs_value_diff_fused"] = float((c[1] - b0[1]).abs().max())
            torch.backends.cudnn.benchmark = True
            fold2 = inference_copy(net, dev, fused=False)
            r["folded_cl_find_ms"] = timeit(fold2.evaluate_planes, x)
            fused2 = inference_copy(net, dev, fused=True, conv="miopen")
            r["fused_find_ms"] = timeit(fused2.evaluate_planes, x)
            torch.backends.cudnn.benchmark = False
            h = inference_copy(net, dev, torch.float16)
            r["fp16_ms"] = timeit(h.evaluate_planes, x)
            a, b = plain(x.view(-1, 1, 8, 8)), fused.evaluate_planes(x)
            r["max_abs_prior_diff_fold"] = float((torch.softmax(a[0], -1) - b[0]).abs().max())
        flops = {"az5x128": 189.0e6, "fast": 15.29e6}[name] * B
        r["tflops_folded"] = flops / (r["folded_cl_ms"] * 1e-3) / 1e12
        r["tflops_fused"] = flops / (r["fused_ms"] * 1e-3) / 1e12
        r["tflops_hipconv"] = flops / (r["hipconv_ms"] * 1e-3) / 1e12
        out[name] = r
    print(json.dumps(out))


if __name__ == "__main__":
    main()
