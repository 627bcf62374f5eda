"""Average per-dispatch counter values of rocprofv3 --pmc CSVs (gpurun_out/sq_<tag>_<pass>/),
skipping the first dispatches (warm-up): python scripts/sq_summary.py gpurun_out/sq_wino4_fp16"""
import csv
import os
import glob
import sys
from collections import defaultdict

for prefix in sys.argv[1:]:
    vals = defaultdict(list)
    for f in sorted(glob.glob(prefix + "_[0-9]*/pmc_counter_collection.csv")):
        rows = list(csv.DictReader(open(f)))
        per = defaultdict(lambda: defaultdict(float))
        for r in rows:
            if os.environ.get("SQ_KERNEL", "conv3x3") not in r["Kernel_Name"]:
                continue
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        ids = sorted(per)[5:]
        for i in ids:
            for k, v in per[i].items():
                vals[k].append(v)
    print(prefix)
    for k in sorted(vals):
        v = vals[k]
        print(f"  {k:28s} {sum(v) / len(v):16.1f}")
