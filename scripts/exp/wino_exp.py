"""Experiment: where the time of the Winograd conv goes.  Builds copies of
csrc/conv_wino.hip with AZ_WN_EXP bits (see the file) and times each at B = 1024 (results of
the hollowed copies are not checked); bit 16 reports the shader clock and the main loop's
wall time of workgroup 0."""
import ctypes, json, os, subprocess
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(ROOT, "alphazero-othello_amd", "csrc", "conv_wino.hip")
out = {}
B = int(os.environ.get("B", "1024"))
for C in [int(c) for c in os.environ.get("CS", "128").split(",")]:
    x = torch.randn(B, C, 8, 8, device="cuda").relu().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x).contiguous(memory_format=torch.channels_last)
    wq = torch.zeros(16 * C * C * 3, dtype=torch.int16, device="cuda")
    w9 = (torch.randn(9, C, C, device="cuda") / (3 * C ** 0.5)).contiguous()
    b = torch.zeros(C, device="cuda")
    y = torch.empty_like(x)
    for tag in os.environ.get("EXPS", "0,1,2,4,8,16,32,7,23").split(","):
        # a tag is an AZ_WN_EXP value, optionally prefixed by a build name ("head0": the
        # committed source, built beforehand into _build/wino_exphead0.so)
        exp = int(tag.lstrip("abcdefghijklmnopqrstuvwxyz") or 0)
        so = os.path.join(HERE, "_build", f"wino_exp{tag}.so")
        os.makedirs(os.path.dirname(so), exist_ok=True)
        if not os.path.exists(so):
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                                   "-shared", "-std=c++17", "-ffp-contract=off", f"-DAZ_WN_EXP={exp}",
                                   SRC, os.path.join(ROOT, "alphazero-othello_amd", "csrc", "board.hip"),
                                   "-o", so])
        L = ctypes.CDLL(so)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert L.az_conv3x3_wino_prep_gpu(ctypes.c_void_p(w9.data_ptr()), ctypes.c_void_p(wq.data_ptr()),
                                          C, 0, st) == 0
        args = [ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wq.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                ctypes.c_void_p(r.data_ptr()), ctypes.c_void_p(y.data_ptr()), B, C, 1, 0, st]
        for mode in (0,):
            args[8] = mode
            for _ in range(3):
                assert L.az_conv3x3_wino_gpu(*args) == 0
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(30):
                L.az_conv3x3_wino_gpu(*args)
            e1.record(); torch.cuda.synchronize()
            key = f"C{C}_exp{tag}_mode{mode}"
            out[key] = round(e0.elapsed_time(e1) / 30 * 1e3, 1)
            if exp & 16:
                stp = torch.as_strided(y, (4,), (1,)).clone().view(torch.int64)[:2].cpu().numpy()
                out[key + "_clockGHz"] = round(float(stp[0]) / float(stp[1]) * 0.1, 3)
                out[key + "_loop_us"] = round(float(stp[1]) / 100.0, 1)
                nwg = (B + 1) // 2
                tl = torch.as_strided(y, (8 + 8 * nwg,), (1,)).clone().view(torch.int64)[4:4 + 4 * nwg]
                tl = tl.view(nwg, 4).cpu().double().numpy()
                t0 = tl[:, 0].min()
                out[key + "_timeline_us"] = {
                    "kernel_span": round((tl[:, 3].max() - t0) / 100, 1),
                    "prologue_med": round(float(np.median(tl[:, 1] - tl[:, 0])) / 100, 2),
                    "loop_med": round(float(np.median(tl[:, 2] - tl[:, 1])) / 100, 2),
                    "epilogue_med": round(float(np.median(tl[:, 3] - tl[:, 2])) / 100, 2),
                    "wg_total_med": round(float(np.median(tl[:, 3] - tl[:, 0])) / 100, 2),
                    "start_quantiles": [round(float(q) / 100, 1) for q in np.quantile(tl[:, 0] - t0, [0, .25, .5, .75, 1])],
                }
        print(json.dumps(out), flush=True)
