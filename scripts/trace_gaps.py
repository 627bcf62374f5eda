"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace (csv): for the last
`n` dispatches, end(i) -> start(i+1) per (kernel i, kernel i+1) pair, and the busy / span
fraction.  Usage: python scripts/trace_gaps.py <run_kernel_trace.csv> [n] > gaps.json"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+)(<[^()]*>)?", name)
    s = m.group(0) if m else name[:40]
    return s.replace("(anonymous namespace)::", "")


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    rows = rows[-n:]
    gaps = defaultdict(list)
    busy = 0
    for (s0, e0, k0), (s1, e1, k1) in zip(rows, rows[1:]):
        gaps[(k0, k1)].append(s1 - e0)
        busy += e0 - s0
    span = rows[-1][1] - rows[0][0]
    out = {"dispatches": len(rows), "span_us": span / 1e3, "busy_frac": busy / span,
           "pairs": {f"{a} -> {b}": {"n": len(v), "mean_gap_us": sum(v) / len(v) / 1e3,
                                      "min_gap_us": min(v) / 1e3}
                     for (a, b), v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
