"""Instruction mix of one kernel in a hipcc -S listing, per basic block (largest first) and in
total: MFMA, packed-f32 VALU, other VALU, LDS, vector memory, SALU, waits.
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S \
        -o /tmp/w4.s alphazero-othello_amd/csrc/conv_wino4.hip
    python scripts/isa_mix.py /tmp/w4.s k_trunk_wino4 [blocks]"""
import collections
import re
import sys


def kind(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith("v_pk_") and op.endswith("f32"):
        return "pk_f32"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt") or op == "s_barrier":
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    nblk = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    lines = open(path).read().split("\n")
    s = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + pat + r"\S*:", l))
    e = next(j for j in range(s, len(lines)) if lines[j].startswith(".Lfunc_end"))
    blocks, cur, name = [], [], "entry"
    for l in lines[s + 1:e]:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            blocks.append((name, cur))
            cur, name = [], m.group(1)
            continue
        t = l.strip()
        if l.startswith("\t") and t and not t.startswith((".", ";")):
            cur.append(t.split()[0])
    blocks.append((name, cur))
    tot = collections.Counter(kind(op) for _, b in blocks for op in b)
    print(lines[s][:100], "total", dict(tot))
    for name, b in sorted(blocks, key=lambda x: -len(x[1]))[:nblk]:
        c = collections.Counter(kind(op) for op in b)
        pk = collections.Counter(op for op in b if kind(op) == "pk_f32")
        print(f"{name:14s} {len(b):5d}", dict(c), dict(pk))


if __name__ == "__main__":
    main()
