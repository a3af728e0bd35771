"""Build libmswegnn.so in-tree for gfx950 (hipcc, no torch involvement).

    python mswe-gnn_amd/build_engine.py [--force]

Objects go to mswe-gnn_amd/_obj/, the library to mswe-gnn_amd/lib/libmswegnn.so.
Rebuilds an object only when its source or a header is newer.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = ["csrc/kernels.hip", "csrc/plan.hip"]
HDR = ["csrc/engine.h", os.path.join(ROOT, "include", "mswegnn.h")]
ARCH = os.environ.get("MSW_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
         "-I", os.path.join(ROOT, "include")]


def _newer(a, b):
    return not os.path.exists(b) or os.path.getmtime(a) > os.path.getmtime(b)


def build(force=False, verbose=True):
    os.makedirs(os.path.join(HERE, "_obj"), exist_ok=True)
    os.makedirs(os.path.join(HERE, "lib"), exist_ok=True)
    objs = []
    hdr_t = max(os.path.getmtime(h if os.path.isabs(h) else os.path.join(HERE, h)) for h in HDR)
    for s in SRC:
        src = os.path.join(HERE, s)
        obj = os.path.join(HERE, "_obj", os.path.basename(s) + ".o")
        objs.append(obj)
        stale = force or _newer(src, obj) or (os.path.exists(obj) and hdr_t > os.path.getmtime(obj))
        if stale:
            cmd = ["hipcc", *FLAGS, "-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
    out = os.path.join(HERE, "lib", "libmswegnn.so")
    if force or any(_newer(o, out) for o in objs):
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
