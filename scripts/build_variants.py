"""Build experiment variants of libaz_othello.so with extra -D flags (A/B runs on the GPU
box load one through AZ_LIB_PATH):
    python scripts/build_variants.py NAME "-DFOO=1 -DBAR=2" [NAME2 "..."]
Outputs expbuild/<NAME>/libaz_othello.so (git-ignored; travels with gpurun)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-othello_amd"))
import az_build  # noqa: E402


def build(name, extra):
    out = os.path.join(ROOT, os.environ.get("EXP_OUT", "expbuild"), name)  # exp6/: travels
    os.makedirs(out, exist_ok=True)
    want = az_build.source_hash()
    flags = [f for f in az_build.FLAGS if f != "-shared"] + extra.split()
    objs = []
    only = os.environ.get("ONLY")  # e.g. ONLY=board.hip: the rest from az_build's object cache
    cached = []
    for src in az_build.SOURCES:
        if only and os.path.basename(src) not in only.split(","):
            objs.append(az_build._object(src, want, "/opt/rocm/bin/hipcc", False))
            cached.append(objs[-1])
            continue
        obj = os.path.join(out, os.path.basename(src) + ".o")
        subprocess.check_call(["/opt/rocm/bin/hipcc"] + flags + [f'-DAZ_BUILD_ID="{want}"', "-c",
                               os.path.join(az_build.HERE, src), "-o", obj])
        objs.append(obj)
    subprocess.check_call(["/opt/rocm/bin/hipcc"] + az_build.FLAGS + objs +
                          ["-o", os.path.join(out, "libaz_othello.so")])
    for o in objs:
        if o not in cached:
            os.remove(o)
    return name


if __name__ == "__main__":
    args = sys.argv[1:]
    pairs = list(zip(args[0::2], args[1::2]))
    with ThreadPoolExecutor(len(pairs)) as ex:
        for n in ex.map(lambda p: build(*p), pairs):
            print("built", n)
