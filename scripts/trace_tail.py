"""Per-kernel mean durations and the step span over the LAST n steps of a rocprofv3 kernel
trace (csv): the steady state of a long bench run, where every slot plays.  Runs on the GPU
box next to the trace (which stays out of gpurun_out/: too large to copy back).

    python scripts/trace_tail.py <run_kernel_trace.csv> [n_steps] > steady.json"""
import collections
import csv
import json
import re
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            m = re.search(r"(k_\w+)(<[^()]*>)?", r["Kernel_Name"])
            name = (m.group(0) if m else r["Kernel_Name"][:40]).replace("(anonymous namespace)::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    sel = [i for i, r in enumerate(rows) if r[2].startswith("k_select")]
    first = sel[-n] if len(sel) >= n else sel[0]
    last = sel[-1]
    tail = rows[first:last]
    steps = sum(1 for r in tail if r[2].startswith("k_select"))
    d = collections.defaultdict(list)
    for s, e, k in tail:
        d[k].append((e - s) / 1e3)
    span = (tail[-1][0] - tail[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in tail) / 1e3
    print(json.dumps({"steps": steps, "span_us_per_step": round(span / steps, 2),
                      "busy_us_per_step": round(busy / steps, 2),
                      "kernels": {k: {"calls": len(v), "mean_us": round(sum(v) / len(v), 2),
                                      "us_per_step": round(sum(v) / steps, 2),
                                      "max_us": round(max(v), 2)} for k, v in d.items()}},
                     indent=1))


if __name__ == "__main__":
    main()
