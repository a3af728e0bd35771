"""Build libmswegnn.so in-tree for gfx950 (hipcc, no torch involvement).

    python mswe-gnn_amd/build_engine.py [--force]

Objects go to mswe-gnn_amd/_obj/, the library to mswe-gnn_amd/lib/libmswegnn.so.
Rebuilds an object when its source or a header is newer, and everything when the sha256 of
the sources + flags differs from the one recorded beside the library at its last build
(lib/libmswegnn.so.srchash): a library copied in with fresh mtimes but built from other
sources is rebuilt.  ``source_hash()`` / ``library_matches_sources()`` let the bench record
which build it measured.
"""
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = ["csrc/kernels_nt1.hip", "csrc/kernels_nt2.hip", "csrc/kernels_nt4.hip",
       "csrc/kernels_common.hip", "csrc/plan.hip", "csrc/metrics.hip", "csrc/train.hip"]
HDR = ["csrc/engine.h", "csrc/kernels_impl.h", "csrc/tiling.h", "csrc/graph_build.h", os.path.join(ROOT, "include", "mswegnn.h")]
HDR += sorted(os.path.join("csrc", "kernels", f) for f in os.listdir(os.path.join(HERE, "csrc", "kernels")) if f.endswith(".h"))
ARCH = os.environ.get("MSW_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
         "-I", os.path.join(ROOT, "include")]


def source_hash(variant=""):
    """sha256 over the engine sources, headers, compiler flags and variant."""
    h = hashlib.sha256()
    for f in SRC + HDR:
        path = f if os.path.isabs(f) else os.path.join(HERE, f)
        h.update(os.path.basename(path).encode())
        with open(path, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS + [variant]).replace(ROOT, "<root>").encode())  # path-independent
    return h.hexdigest()


def lib_path(variant=""):
    return os.path.join(HERE, "lib", f"libmswegnn_{variant}.so" if variant else "libmswegnn.so")


def library_matches_sources(variant=""):
    """True when the library's recorded source hash equals the current sources' hash."""
    try:
        with open(lib_path(variant) + ".srchash") as f:
            return f.read().strip() == source_hash(variant)
    except OSError:
        return False


def _newer(a, b):
    return not os.path.exists(b) or os.path.getmtime(a) > os.path.getmtime(b)


def build(force=False, verbose=True, variant=""):
    """variant "trace": diagnostic library lib/libmswegnn_trace.so (-DMSW_TRACE)."""
    odir = os.path.join(HERE, "_obj" + (f"_{variant}" if variant else ""))
    # build variants: the -DMSW_TRACE diagnostic library, and the speed A/Bs of the current
    # round (each bit-identical to the default: test_build_variant_matches_default_bitwise)
    extra = {"trace": ["-DMSW_TRACE"],
             # the round-5 VALU diets off (PReLU as max, FULL edge kernels):
             # test_build_variant_matches_default_bitwise[valubase]
             "valubase": ["-DMSW_PRELU_MAX=0", "-DMSW_EDGE_FULL=0"],
             # plain stores in place of the large-mesh launches' streaming stores
             "nostream": ["-DMSW_STREAM_ST=0"]}.get(variant, [])
    os.makedirs(odir, exist_ok=True)
    os.makedirs(os.path.join(HERE, "lib"), exist_ok=True)
    out = lib_path(variant)
    if os.path.exists(out) and not library_matches_sources(variant):
        force = True  # built from other sources (or unrecorded): rebuild everything
    objs, cmds = [], []
    hdr_t = max(os.path.getmtime(h if os.path.isabs(h) else os.path.join(HERE, h)) for h in HDR)
    for s in SRC:
        src = os.path.join(HERE, s)
        obj = os.path.join(odir, os.path.basename(s) + ".o")
        objs.append(obj)
        stale = force or _newer(src, obj) or (os.path.exists(obj) and hdr_t > os.path.getmtime(obj))
        if stale:
            cmds.append(["hipcc", *FLAGS, *extra, "-c", src, "-o", obj])
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 8))
    with ThreadPoolExecutor(jobs) as ex:  # one hipcc per translation unit, in parallel
        for cmd in cmds:
            if verbose:
                print(" ".join(cmd), flush=True)
        for r in list(ex.map(lambda c: subprocess.run(c, check=False), cmds)):
            if r.returncode != 0:
                raise subprocess.CalledProcessError(r.returncode, r.args)
    if force or any(_newer(o, out) for o in objs):
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    with open(out + ".srchash", "w") as f:
        f.write(source_hash(variant) + "\n")
    return out


if __name__ == "__main__":
    var = [a[len("--variant="):] for a in sys.argv if a.startswith("--variant=")]
    build(force="--force" in sys.argv, variant="trace" if "--trace" in sys.argv else (var[0] if var else ""))
