"""A/B timing of the leaf-evaluation net variants in one process (same box, same inputs):
stem fused into the first block or not, per trunk precision.  Batch = the bench's 1,024."""
import json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-othello_amd"))
from Models import AlphaZeroNet, inference_copy  # noqa: E402


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


torch.manual_seed(0)
net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
B = 1024
planes = torch.randint(-1, 2, (B, 64), device="cuda").float()
pr = torch.empty(B, 65, device="cuda"); va = torch.empty(B, device="cuda")
out = {}
for prec in ("split3", "fp16"):
    m = inference_copy(net, "cuda", precision=prec)
    for fuse in (False, True, False, True):
        m.fuse_stem = fuse
        g = torch.cuda.CUDAGraph()
        with torch.no_grad():
            m.evaluate_into(planes, pr, va)
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                m.evaluate_into(planes, pr, va)
        out.setdefault(f"{prec}_fuse{int(fuse)}_us", []).append(round(timed(g.replay), 1))
print(json.dumps(out))
