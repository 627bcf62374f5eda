"""Mean per dispatch of each PMC counter, per kernel, from a rocprofv3 --pmc csv run
(counter_collection.csv): python scripts/pmc_kernel_avg.py <dir> > out.json"""
import collections
import csv
import glob
import json
import re
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(json.dumps({k: {c: round(sum(v) / len(v), 1) for c, v in d.items()}
                      for k, d in acc.items()}, indent=1))


if __name__ == "__main__":
    main()
