"""profiles/trunk_traffic.json from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over
scripts/trunk_heads_one.py 1024 20 (the launch bench.py's roofline_trunk times), with the
hash of the trunk kernel's sources (and the library's), so bench.py reports the figure only while
the kernel is the one it was measured on.
    python scripts/trunk_traffic.py <fetch pass dir> <write pass dir> <source note> > profiles/trunk_traffic.json
gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half the bytes of wide
reads -> x 2 (checked on the calibration copy in profiles/oth_step_traffic.json); WRITE_SIZE as
is.  Dispatches 6.. are averaged (the first ones fault in pages and fill the L2s)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]


def per_dispatch(d, counter):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        if "k_trunk_wino4" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            k = int(r["Dispatch_Id"])
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    xs = [vals[k] for k in sorted(vals)][5:]
    return sum(xs) / len(xs), len(xs)


def main():
    import az_build

    fetch, nf = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write, nw = per_dispatch(sys.argv[2], "WRITE_SIZE")
    rd, wr = fetch * 1024 * 2, write * 1024
    print(json.dumps({
        "kernel": "k_trunk_wino4<..., heads> (az_trunk_wino4_heads_gpu: stem + 10 block convs + "
                  "heads, the layer input resident in LDS), the launch bench.py's roofline_trunk times",
        "boards": 1024, "source": sys.argv[3], "build_id": az_build.source_hash(),
        "trunk_sources_hash": az_build.sources_hash(az_build.TRUNK_SOURCES),
        "dispatches_averaged": [nf, nw],
        "FETCH_SIZE_KB": fetch, "WRITE_SIZE_KB": write,
        "correction": "gfx950: FETCH_SIZE counts half the bytes of wide reads -> x 2 "
                      "(MI355X_MICROARCH.md HBM section; calibration copy in "
                      "profiles/oth_step_traffic.json); WRITE_SIZE as is",
        "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": ALGORITHMIC,
        "traffic_over_algorithmic": (rd + wr) / ALGORITHMIC}, indent=1))


# the launch's algorithmic HBM bytes at B = 1,024: the canonical planes in (64 fp32 per board),
# priors (65) + value (1) fp32 out, and the prepared weights once (10 convs x 16 points x 128 x
# 128 x 2 fp16 planes x 2 B + biases, stem and heads: ~10.6 MB)
ALGORITHMIC = 1024 * 64 * 4 + 1024 * 66 * 4 + 10 * (16 * 128 * 128 * 2 * 2 + 128 * 4) \
    + 9 * 128 * 4 + 128 * 4 + (3 * 128 + 65 * 128 + 64 * 256 + 256) * 4


if __name__ == "__main__":
    main()
