"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd SQLite) as a markdown
table: per kernel calls, total/avg duration (us) and share, plus per-step figures when the
number of steps is given.

    python scripts/prof_summary.py gpurun_out/prof/run_results.db [--steps N] > profiles/x.md
"""
import argparse
import re
import sqlite3


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    if name.startswith("void "):
        name = name[5:]
    return name if len(name) < 90 else name[:87] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    if a.db.endswith(".csv"):
        # rocprofv3 --stats --output-format csv: <run>_kernel_stats.csv (durations in ns)
        import csv

        rows = []
        for r in csv.DictReader(open(a.db)):
            rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                         float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
        rows.sort(key=lambda r: -r[2])
    else:
        c = sqlite3.connect(a.db)
        rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                              "from top_kernels order by total_duration desc"))
    tot = sum(r[2] for r in rows)
    print(f"source: `{a.db}` (rocprofv3 --kernel-trace --stats); durations in microseconds\n")
    hdr = "| kernel | calls | total us | avg us | % |"
    if a.steps:
        hdr += " calls/step | us/step |"
    print(hdr)
    print("|" + "---|" * (hdr.count("|") - 1))
    for name, calls, total, avg, pct in rows[:a.top]:
        line = f"| `{short(name)}` | {calls} | {total:.1f} | {avg:.2f} | {pct:.2f} |"
        if a.steps:
            line += f" {calls / a.steps:.2f} | {total / a.steps:.2f} |"
        print(line)
    print(f"\nall kernels: {tot:.1f} us total")


if __name__ == "__main__":
    main()
