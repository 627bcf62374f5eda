"""Build libaz_othello.so for gfx950 in-tree (hipcc; no cmake, no JIT cache).

    python alphazero-othello_amd/az_build.py

-ffp-contract=off keeps every float expression in the reference's operation order (no
fused multiply-add), which the bit-exact MCTS parity (PUCT, prior renormalisation, TD(lambda))
depends on.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = ["csrc/board.hip", "csrc/engine.hip", "csrc/nn_fused.hip", "csrc/conv.hip", "csrc/conv16.hip", "csrc/conv_wino.hip", "csrc/heads.hip", "csrc/replay.hip"]
HEADERS = ["csrc/bitboard.h", "csrc/common.h", "csrc/philox.h", "../include/az_othello.h"]
OUT = os.path.join(HERE, "libaz_othello.so")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function"]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(os.path.join(HERE, f)) > t for f in SOURCES + HEADERS)


def build(force=False, verbose=True):
    if not force and not _stale():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc] + FLAGS + [os.path.join(HERE, s) for s in SOURCES] + ["-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=HERE)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
