"""Summarise the rocprofv3 PMC passes of scripts/pmc_step.sh: HBM bytes per k_step launch,
with the gfx950 corrections of MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts 128-B
read requests as 64 B (x2, confirmed here on the calibration copy of a known 256 MiB and by
TCC_EA0_RDREQ x 128 B); WRITE_SIZE reads exact.  Writes profiles/<tag>_oth_step_pmc.md and
profiles/oth_step_traffic.json (read by bench.py's roofline.traffic)."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out")
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 24
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(src, "pmc_*", "pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = "k_step" if "k_step" in r["Kernel_Name"] else (
            "calib_copy" if "copyBuffer" in r["Kernel_Name"] else None)
        if k:
            vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in vals.items()}
calib_bytes = 64 << 22  # 256 MiB copied (read and written)
rd = 2 * avg[("k_step", "FETCH_SIZE")] * 1024
wr = avg[("k_step", "WRITE_SIZE")] * 1024
alg = 43 * n
out = {"kernel": "k_step2 (oth_step_gpu)", "positions": n, "hbm_read_bytes": rd,
       "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes": alg,
       "traffic_over_algorithmic": (rd + wr) / alg,
       "calibration": {"copy_bytes_each_way": calib_bytes,
                       "FETCH_SIZE_x2_bytes": 2 * avg[("calib_copy", "FETCH_SIZE")] * 1024,
                       "WRITE_SIZE_bytes": avg[("calib_copy", "WRITE_SIZE")] * 1024},
       "raw_averages": {f"{k}:{c}": v for (k, c), v in sorted(avg.items())}}
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "profiles", "oth_step_traffic.json"), "w"), indent=1)
with open(os.path.join(ROOT, "profiles", f"{tag}_oth_step_pmc.md"), "w") as f:
    f.write(f"# k_step HBM traffic ({tag}), {n} positions per launch\n\n")
    f.write("rocprofv3 --pmc, one counter group per pass (scripts/pmc_step.sh); "
            "FETCH_SIZE x2 (gfx950 128-B request tally), WRITE_SIZE as read.\n\n")
    f.write("| quantity | bytes per launch | per position |\n|---|---|---|\n")
    for name, b in (("HBM read (FETCH_SIZE x 2 x 1024)", rd), ("HBM write (WRITE_SIZE x 1024)", wr),
                    ("HBM total", rd + wr), ("algorithmic (43 B/position)", alg)):
        f.write(f"| {name} | {b:,.0f} | {b / n:.2f} |\n")
    f.write(f"\ncalibration copy (256 MiB each way): FETCH_SIZE x2 = "
            f"{out['calibration']['FETCH_SIZE_x2_bytes']:,.0f} B, WRITE_SIZE = "
            f"{out['calibration']['WRITE_SIZE_bytes']:,.0f} B\n\nraw counter averages:\n\n")
    for k, v in sorted(avg.items()):
        f.write(f"- {k[0]} {k[1]}: {v:,.1f}\n")
print(json.dumps({k: out[k] for k in ("hbm_bytes_per_launch", "algorithmic_bytes", "traffic_over_algorithmic")}))
