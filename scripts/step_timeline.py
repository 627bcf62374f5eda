"""Sustained self-play step time: ms/step per block of steps over a long run, for the
fused HIP conv and the MIOpen conv inference copies (diagnoses clock drift / overheads)."""
import json, os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "alphazero-othello_amd"))
from engine import BatchedSelfPlay  # noqa: E402
from Models import AlphaZeroNet, inference_copy  # noqa: E402
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 12000
block = 1000
for conv in ("hip", "miopen"):
    torch.manual_seed(0)
    net = AlphaZeroNet(8, 65, 5, 128)
    sp = BatchedSelfPlay(net, bench.SELFPLAY_ARGS, 1024, seed=1)
    sp.net = inference_copy(net, sp.device, conv=conv)
    sp.reset(-1, 4000)
    out = []
    sp.step(2)
    torch.cuda.synchronize()
    for b in range(steps // block):
        t0 = time.perf_counter()
        sp.step(block)
        torch.cuda.synchronize()
        out.append(round((time.perf_counter() - t0) * 1000 / block, 3))
    # GPU time of one step via events (graph replay)
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record(); sp.step(200); e1.record(); torch.cuda.synchronize()
    print(json.dumps({"conv": conv, "ms_per_step_blocks": out, "event_ms_per_step": round(e0.elapsed_time(e1) / 200, 3),
                      "graph": sp.graph is not None}), flush=True)
