"""Build libaz_othello.so for gfx950 in-tree (hipcc; no cmake, no JIT cache).

    python alphazero-othello_amd/az_build.py [--force]

-ffp-contract=off keeps every float expression in the reference's operation order (no
fused multiply-add), which the bit-exact MCTS parity (PUCT, prior renormalisation, TD(lambda))
depends on.

The library carries the sha256 of its sources, headers and flags (`source_hash()`), embedded
as AZ_BUILD_ID and returned by az_build_id().  build() recompiles whenever the id in the
existing .so differs from the tree's hash (never by file times), and smoke() / the CPU tests
assert that the library a process loaded was built from the tree under test.
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = ["csrc/board.hip", "csrc/engine.hip", "csrc/nn_fused.hip", "csrc/conv.hip",
           "csrc/conv16.hip", "csrc/conv_wino.hip", "csrc/conv_wino4.hip", "csrc/heads.hip",
           "csrc/replay.hip"]
HEADERS = ["csrc/bitboard.h", "csrc/common.h", "csrc/philox.h", "csrc/heads_az.h",
           "../include/az_othello.h"]
OUT = os.path.join(HERE, "libaz_othello.so")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function"]
_TAG = b"AZ_BUILD_ID="


def source_hash():
    """sha256 over the flags and every source/header (name and bytes), in a fixed order."""
    h = hashlib.sha256()
    h.update(" ".join(FLAGS).encode())
    for f in SOURCES + HEADERS:
        h.update(b"\0" + f.encode() + b"\0")
        with open(os.path.join(HERE, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


# the persistent trunk's kernel sources: what profiles/trunk_traffic.json's PMC figure depends
# on (the az_othello.h declarations and the other kernels do not change its code)
TRUNK_SOURCES = ["csrc/conv_wino4.hip", "csrc/heads_az.h", "csrc/common.h"]


def sources_hash(files):
    """sha256 over the flags and the given sources (name and bytes), in the given order."""
    h = hashlib.sha256()
    h.update(" ".join(FLAGS).encode())
    for f in files:
        h.update(b"\0" + f.encode() + b"\0")
        with open(os.path.join(HERE, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def built_id(path=OUT):
    """The AZ_BUILD_ID embedded in a built library (read from the file, not loaded)."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as fh:
        data = fh.read()
    i = data.find(_TAG)
    return data[i + len(_TAG):i + len(_TAG) + 64].decode("ascii", "replace") if i >= 0 else None


def _object(src, want, hipcc, verbose):
    """Compile one translation unit (cached by the hash of its text, the headers and the
    flags; board.hip also carries the build id) into build/."""
    h = hashlib.sha256(" ".join(FLAGS).encode())
    for f in [src] + HEADERS:
        with open(os.path.join(HERE, f), "rb") as fh:
            h.update(fh.read())
    if src == "csrc/board.hip":
        h.update(want.encode())
    obj = os.path.join(HERE, "build", f"{os.path.basename(src)}-{h.hexdigest()[:16]}.o")
    if not os.path.exists(obj):
        flags = [f for f in FLAGS if f != "-shared"]
        cmd = [hipcc] + flags + [f'-DAZ_BUILD_ID="{want}"', "-c", os.path.join(HERE, src),
                                 "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd, cwd=HERE)
        os.replace(obj + ".tmp", obj)
    return obj


def build(force=False, verbose=True, jobs=None):
    want = source_hash()
    if not force and built_id() == want:
        if verbose:
            print(f"libaz_othello.so is current (build id {want[:16]})", flush=True)
        return OUT
    from concurrent.futures import ThreadPoolExecutor

    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    jobs = jobs or min(len(SOURCES), max(1, min(8, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:  # each worker just waits on its hipcc process
        objs = list(ex.map(lambda s: _object(s, want, hipcc, verbose), SOURCES))
    cmd = [hipcc] + FLAGS + objs + ["-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=HERE)
    os.replace(OUT + ".tmp", OUT)
    assert built_id() == want, "build id missing from the built library"
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
