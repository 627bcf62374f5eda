"""Time the single-launch Winograd trunk (az_trunk_wino_gpu) against the layer-by-layer
launches (stem + 2 x blocks convs) on the bench net at the bench's leaf batch."""
import json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-othello_amd"))
from Models import AlphaZeroNet, inference_copy  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
torch.manual_seed(0)
net = AlphaZeroNet(8, 65, 5, 128).cuda().eval()
m = inference_copy(net, "cuda", precision="split3", conv_algo="wino")
x = torch.randint(-1, 2, (B, 1, 8, 8), device="cuda").float()
out = {"B": B}
for fuse in (True, False, True, False):
    m.fuse_trunk = fuse
    with torch.no_grad():
        for _ in range(3):
            m._trunk(x)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(10):
                m._trunk(x)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
    out[f"{'fused' if fuse else 'layers'}_us"] = round(e0.elapsed_time(e1) / 50 * 1e3, 1)
print(json.dumps(out))
