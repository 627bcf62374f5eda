"""HBM bytes per trunk-conv launch from scripts/pmc_conv.sh's passes (gfx950 corrections
of MI355X_MICROARCH.md: FETCH_SIZE x2, WRITE_SIZE as read; the calibration copy checks
them on this GPU).  Writes profiles/conv_traffic.json (read by bench.py's roofline_conv,
which uses it when its kernel_tag names the conv form the bench times)."""
import collections, csv, glob, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(src, "pmcc_*", "pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = "conv" if "k_conv3x3_wino4" in r["Kernel_Name"] else (
            "calib_copy" if "copyBuffer" in r["Kernel_Name"] or "copy" in r["Kernel_Name"] else None)
        if k:
            vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
# the calibration row is the largest copy (the per-launch absmax refills are copies too)
avg = {k: (max(v) if k[0] == "calib_copy" else sum(v) / len(v)) for k, v in vals.items()}
B, C = 1024, 128
rd = 2 * avg[("conv", "FETCH_SIZE")] * 1024
wr = avg[("conv", "WRITE_SIZE")] * 1024
act = B * 64 * C * 4  # fp32 channels-last activations
wq = 16 * C * C * 2 * 2 + 16  # az_conv3x3_wino_prep_bytes(128, FP16X2)
alg = 3 * act + wq + C * 4 + 2 * B * 4  # x, residual, y; weights and bias once; absmax in/out
cal = {k[1]: v for k, v in avg.items() if k[0] == "calib_copy"}
out = {"kernel": "k_conv3x3_wino4 (fp16x2, 2 boards per workgroup, residual + ReLU)",
       "kernel_tag": f"wino4_fp16x2_{C}", "boards": B, "channels": C,
       "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
       "algorithmic_hbm_bytes": alg, "traffic_over_algorithmic": (rd + wr) / alg,
       "calibration": {"copy_bytes_each_way": 268435456,
                       "read_bytes_measured": 2 * cal.get("FETCH_SIZE", 0) * 1024,
                       "write_bytes_measured": cal.get("WRITE_SIZE", 0) * 1024}}
json.dump(out, open(os.path.join(ROOT, "profiles", "conv_traffic.json"), "w"), indent=1)
print(json.dumps(out))
