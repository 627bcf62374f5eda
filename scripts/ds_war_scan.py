"""Scan gfx950 machine code for two LDS-store patterns (the two-board heads).

Rule 1 (this module's default CLI mode; diagnostic only): an LDS store whose data VGPRs are
overwritten before the store is known complete.  The compiler does this routinely (over a
thousand times in the conv kernels, which pass every bit-exact test), so it is NOT a hazard;
kept to show that.  Rule 2 (--pk; enforced by tests/test_isa_scan_cpu.py): see
scan_pk_stores.

For every `ds_write*` (and `ds_write2*`), the data VGPRs are the operands after the address.
The store stays "in flight" until an `s_waitcnt` whose lgkmcnt(N) leaves at most N younger
LGKM operations outstanding (DS operations complete in issue order; SMEM and message ops
count too).  The scan reports every instruction in that window that WRITES one of the data
VGPRs: a `ds_read*` / returning DS atomic destination, a vector-memory load destination, or
a VALU / MFMA destination.  A kernel boundary or an `s_barrier` preceded by lgkmcnt(0) ends
every window; branches and labels are scanned in layout order (straight-line windows only,
which is where the compiler schedules a store and the reuse of its registers together).

    python scripts/ds_war_scan.py <file.s | libaz_othello.so> [...]

Input: compiler assembly (.s) or a shared library, whose gfx950 code objects are extracted
with llvm-objdump --offloading into a temporary directory and disassembled.  Prints one line
per finding and exits 1 if there is any."""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
_REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def regs(op):
    """VGPR/AGPR set named by one operand string: {('v', n), ...}."""
    out = set()
    for m in _REG.finditer(op):
        if m.group(1):
            k, a, b = m.group(1), int(m.group(2)), int(m.group(3))
            out.update((k, i) for i in range(a, b + 1))
        elif m.group(4):
            out.add((m.group(4), int(m.group(5))))
    return out


def split_operands(rest):
    """Operands of one instruction (modifiers like offset:16 stay attached to the last)."""
    ops, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


def parse_lines(text):
    """(function, mnemonic, operand list, raw line) per instruction, in layout order."""
    fn = "?"
    for raw in text.splitlines():
        line = raw.split("//")[0].split(";")[0].rstrip()
        if not line.strip():
            continue
        s = line.strip()
        if s.endswith(":") and not s.startswith("."):
            if not s.startswith(".L") and not s.startswith("LBB"):
                fn = s[:-1]
            yield fn, ":label", [], raw
            continue
        m = re.match(r"^([0-9a-f]+ )?<(.+)>:$", s)  # objdump function header
        if m:
            fn = m.group(2)
            yield fn, ":label", [], raw
            continue
        if s.startswith("."):
            continue
        parts = s.split(None, 1)
        mn = parts[0]
        if not re.match(r"^[sv]_|^ds_|^buffer_|^global_|^flat_|^scratch_", mn):
            continue
        yield fn, mn, split_operands(parts[1]) if len(parts) > 1 else [], raw


def lgkm_wait(mn, ops):
    """N of an s_waitcnt's lgkmcnt(N), or None."""
    if mn != "s_waitcnt":
        return None
    m = re.search(r"lgkmcnt\((\d+)\)", " ".join(ops))
    return int(m.group(1)) if m else None


def is_lgkm(mn):
    return mn.startswith("ds_") or mn.startswith("s_load") or mn.startswith("s_buffer_load") \
        or mn in ("s_sendmsg", "s_memtime", "s_memrealtime", "s_dcache_inv")


def written_vregs(mn, ops):
    """Vector registers an instruction writes (its destination), if any."""
    if not ops:
        return set()
    if mn.startswith("ds_write") or mn.startswith("ds_store") or "_store" in mn:
        return set()
    if mn.startswith("ds_"):
        if mn.startswith("ds_read") or mn.startswith("ds_load") or "_rtn" in mn \
                or mn.startswith("ds_swizzle") or mn.startswith("ds_permute") \
                or mn.startswith("ds_bpermute"):
            return regs(ops[0])
        return set()
    if mn.startswith(("buffer_load", "global_load", "flat_load", "scratch_load")):
        if " lds" in " ".join(ops) or "_lds" in mn:
            return set()
        return regs(ops[0])
    if "atomic" in mn:
        return regs(ops[0]) if "glc" in " ".join(ops) or "sc0" in " ".join(ops) else set()
    if mn.startswith("v_"):
        if mn.startswith(("v_cmp", "v_readlane", "v_readfirstlane", "v_cmpx")):
            return set()
        return regs(ops[0])
    return set()


def store_data(mn, ops):
    if not (mn.startswith("ds_write") or mn.startswith("ds_store")):
        return None
    if mn.startswith("ds_write_addtid"):
        return regs(ops[0]) if ops else set()
    return set().union(*[regs(o.split(" offset")[0]) for o in ops[1:]]) if len(ops) > 1 else set()


# Rule 2 (the one tests/test_isa_scan_cpu.py enforces on the product library): a multi-dword
# LDS store (ds_write_b64 / b96 / b128, ds_write2_b64, ds_write2st64_b64) whose data VGPRs were
# written by a packed-FP32 VALU instruction (v_pk_add / v_pk_mul / v_pk_fma _f32) within the
# PK_WINDOW instructions before it.  Round 3's two-board heads (heads_az.h with the val_fc1
# partial-sum quad left to the compiler's SLP pairing) stored wrong words in lanes 48-63 with
# two workgroups per CU; that build has this pattern at every partial-sum store (30 sites,
# all in the heads kernels) and the product library has none.
PK_PRODUCER = re.compile(r"^v_pk_(add|mul|fma)_f32")
PK_STORES = ("ds_write_b64", "ds_write_b96", "ds_write_b128", "ds_write2_b64",
             "ds_write2st64_b64")
PK_WINDOW = 3


def scan_pk_stores(text, where="", window=PK_WINDOW):
    """Rule 2 findings: (where, function, distance, producer line, store line)."""
    found = []
    hist = []
    for fn, mn, ops, raw in parse_lines(text):
        if mn == ":label":
            continue
        if mn in PK_STORES:
            data = store_data(mn, ops) or set()
            for dist, (pm, pw, praw) in enumerate(reversed(hist[-window:])):
                if PK_PRODUCER.match(pm) and pw & data:
                    found.append((where, fn, dist, praw.strip(), raw.strip()))
        hist.append((mn, written_vregs(mn, ops), raw))
    return found


def scan_text(text, where=""):
    findings = []
    pending = []  # [fn, store raw line, data regs, younger lgkm ops]
    for fn, mn, ops, raw in parse_lines(text):
        if pending and pending[0][0] != fn:
            pending = []
        n = lgkm_wait(mn, ops)
        if n is not None:
            pending = [p for p in pending if p[3] < n]
            continue
        if mn == ":label":
            continue
        w = written_vregs(mn, ops)
        if w:
            for p in pending:
                hit = w & p[2]
                if hit:
                    findings.append((where, fn, p[1].strip(), raw.strip(), sorted(hit)))
        if is_lgkm(mn):
            for p in pending:
                p[3] += 1
        d = store_data(mn, ops)
        if d:
            pending.append([fn, raw, d, 0])
    return findings


def disassemble_so(path):
    """gfx950 code objects of a HIP shared library, disassembled (text per object)."""
    tmp = tempfile.mkdtemp(prefix="dswar_")
    try:
        lib = os.path.join(tmp, "lib.so")
        shutil.copy(path, lib)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", lib], cwd=tmp, check=True,
                       capture_output=True)
        out = []
        for f in sorted(os.listdir(tmp)):
            if "amdgcn" in f and "gfx950" in f:
                r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950",
                                    "--no-show-raw-insn", os.path.join(tmp, f)],
                                   check=True, capture_output=True, text=True)
                out.append((f, r.stdout))
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def kernel_static_lds(path):
    """{kernel symbol: .group_segment_fixed_size} from the gfx950 code objects' metadata notes
    (static LDS: a kernel's dynamic LDS starts right after it)."""
    tmp = tempfile.mkdtemp(prefix="dslds_")
    try:
        lib = os.path.join(tmp, "lib.so")
        shutil.copy(path, lib)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", lib], cwd=tmp, check=True,
                       capture_output=True)
        out = {}
        for f in sorted(os.listdir(tmp)):
            if "amdgcn" in f and "gfx950" in f:
                notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(tmp, f)],
                                       check=True, capture_output=True, text=True).stdout
                for block in notes.split("\n  - ")[1:]:
                    name = re.search(r"^\s*\.name:\s+(\S+)", block, re.M)
                    size = re.search(r"^\s*\.group_segment_fixed_size:\s+(\d+)", block, re.M)
                    if name and size:
                        out[name.group(1)] = int(size.group(1))
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def texts_of(path):
    if path.endswith(".s"):
        return [(os.path.basename(path), open(path).read())]
    return disassemble_so(path)


def scan_path(path):
    found = []
    for name, text in texts_of(path):
        found += scan_text(text, name)
    return found


def main(argv):
    """--pk: rule 2 (packed-FP32 result -> multi-dword LDS store); default: rule 1."""
    pk = "--pk" in argv
    bad = []
    for p in [a for a in argv if a != "--pk"]:
        if pk:
            for name, text in texts_of(p):
                bad += scan_pk_stores(text, name)
        else:
            bad += scan_path(p)
    for f in bad:
        if pk:
            where, fn, dist, prod, st = f
            print(f"{where}: {fn}\n    producer ({dist} between): {prod}\n    store: {st}")
        else:
            where, fn, st, wr, hit = f
            print(f"{where}: {fn}\n    store: {st}\n    write: {wr}   regs {hit}")
    print(f"{len(bad)} finding(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
