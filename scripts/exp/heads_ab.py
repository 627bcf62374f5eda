"""Time k_heads_az (AZ_HEADS_STAGE=1: FC weights staged in LDS; 0: read from L2) at the
bench batch on the bench net's fused heads; run once per setting."""
import json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "alphazero-othello_amd"))
from Models import AlphaZeroNet, inference_copy  # noqa: E402

torch.manual_seed(0)
m = inference_copy(AlphaZeroNet(8, 65, 5, 128).cuda().eval(), "cuda")
B = 1024
x = torch.randint(-1, 2, (B, 64), device="cuda").float()
pr = torch.empty(B, 65, device="cuda")
va = torch.empty(B, device="cuda")
with torch.no_grad():
    m.evaluate_into(x, pr, va)
    h = m._trunk(x.view(B, 1, 8, 8))
    import az_native as nat
    hw = m._hw
    args = [nat.ptr(h), nat.ptr(hw["wpv"]), nat.ptr(hw["bpv"]), nat.ptr(hw["wpolT"]), nat.ptr(hw["bpol"]),
            nat.ptr(hw["w1T"]), nat.ptr(hw["b1"]), nat.ptr(hw["w2"]), nat.ptr(hw["b2"]), nat.ptr(pr),
            nat.ptr(va), B, 128, nat.stream_ptr()]
    for _ in range(5):
        nat.lib.az_heads_az_gpu(*args)
    torch.cuda.synchronize()
    ref = pr.clone()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(50):
        nat.lib.az_heads_az_gpu(*args)
    e1.record()
    torch.cuda.synchronize()
print(json.dumps({"stage": os.environ.get("AZ_HEADS_STAGE", "1"),
                  "us": round(e0.elapsed_time(e1) / 50 * 1e3, 2),
                  "prior_sum": float(pr.sum())}))
