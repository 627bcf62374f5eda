"""Experiment: where the time of the 16-bit MFMA conv goes.  Builds copies of csrc/conv16.hip
with AZ_MX_EXP bits (1 no A reads, 2 no weight loads, 4 no staging, 8 no epilogue stores)
and times each at B = 1024, C = 128 (results of the hollowed copies are not checked)."""
import ctypes, json, os, subprocess, sys
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(ROOT, "alphazero-othello_amd", "csrc", "conv16.hip")
out = {}
B, C = 1024, 128
x = torch.randn(B, C, 8, 8, device="cuda").relu().contiguous(memory_format=torch.channels_last)
r = torch.randn_like(x).contiguous(memory_format=torch.channels_last)
wq = torch.zeros(9 * C * C * 3, dtype=torch.int16, device="cuda")
w9 = (torch.randn(9, C, C, device="cuda") / (3 * C ** 0.5)).contiguous()
b = torch.zeros(C, device="cuda")
y = torch.empty_like(x)
for exp in [int(v) for v in os.environ.get("EXPS", "0,1,2,3,4,8,12,15").split(",")]:
    so = os.path.join(ROOT, "gpurun_out", f"conv16_exp{exp}.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                           "-std=c++17", "-ffp-contract=off", f"-DAZ_MX_EXP={exp}", SRC,
                           os.path.join(ROOT, "alphazero-othello_amd", "csrc", "board.hip"), "-o", so])
    L = ctypes.CDLL(so)
    if os.environ.get("RANDOM_W"):
        assert L.az_conv3x3_mx_prep_gpu(ctypes.c_void_p(w9.data_ptr()), ctypes.c_void_p(wq.data_ptr()), C, 0,
                                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    args = [ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wq.data_ptr()), ctypes.c_void_p(b.data_ptr()),
            ctypes.c_void_p(r.data_ptr()), ctypes.c_void_p(y.data_ptr()), B, C, 1, 0,
            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)]
    for mode in (0, 1):
        args[8] = mode
        for _ in range(3):
            assert L.az_conv3x3_mx_gpu(*args) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(30):
            L.az_conv3x3_mx_gpu(*args)
        e1.record(); torch.cuda.synchronize()
        out[f"exp{exp}_mode{mode}"] = round(e0.elapsed_time(e1) / 30 * 1e3, 1)
        if exp & 16:
            st = torch.as_strided(y, (4,), (1,)).clone().view(torch.int64)[:2].cpu().numpy()
            out[f"exp{exp}_mode{mode}_clockGHz"] = round(float(st[0]) / float(st[1]) * 0.1, 3)
            out[f"exp{exp}_mode{mode}_loop_us"] = round(float(st[1]) / 100.0, 1)
    print(json.dumps(out), flush=True)
