"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into profiles/<round>/pmc_summary.json.

    python tools/pmc_summary.py OUT.json DIR_FETCH DIR_WRITE

Per (kernel, grid) the counters are averaged over dispatches.  gfx950 correction
(MI355X_MICROARCH.md §HBM): FETCH_SIZE (KB) reports half the bytes of 16-B/lane
coalesced reads -> read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE (KB) is exact for
16-B/lane stores.  Infinity-Cache hits are counted too (memory-side L2 requests), so at
sizes that fit the 256 MB L3 this is L2-miss traffic, an upper bound on HBM bytes.
"key" entries: the fine-scale middle hop (the bench roofline kernel) = the k_hop grid with
the most dispatches (bench.py times it 200+ times).
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def library_sha256():
    """sha256 of the engine library the profiled command loaded (bench.py compares it with the
    library it loads: roofline.rocprof / traffic_source .stale)."""
    import hashlib
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mswe-gnn_amd", "lib",
                        "libmswegnn.so")
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def load(d, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void msw::", "").replace("msw::", "")
            grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)))
            acc[(name, grid)].append(float(r["Counter_Value"]))
    return acc


def main():
    out, dfetch, dwrite = sys.argv[1:4]
    fe, wr = load(dfetch, "FETCH_SIZE"), load(dwrite, "WRITE_SIZE")
    table = {}
    for key in sorted(set(fe) | set(wr)):
        f, w = fe.get(key, []), wr.get(key, [])
        rd = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        table[f"{key[0]} grid={key[1]}"] = {
            "dispatches": max(len(f), len(w)), "read_bytes_per_launch": rd,
            "write_bytes_per_launch": wb,
            "hbm_bytes_per_launch": (rd or 0) + (wb or 0) if (rd is not None or wb is not None) else None}
    hops = [(k, v) for k, v in table.items() if k.startswith("k_hop")]
    res = {"note": __doc__.strip().splitlines()[2], "library_sha256": library_sha256(), "kernels": table}
    if hops:
        k, v = max(hops, key=lambda kv: kv[1]["dispatches"])
        res["k_hop"] = dict(v, kernel=k)
        # bench.py's large-mesh roofline (config 5): the middle hop (LAST = false, the third
        # template argument) moving the most bytes per launch (grid-stride launches have
        # capped grids, so the grid size does not identify it)
        def middle(kk):  # k_hop_rows (row layout) is a middle hop; k_hop<NT, ACT, LAST, LOOP>
            if kk.startswith("k_hop_rows"):
                return True
            args = kk.split("<")[1].split(">")[0].split(",")
            return kk.startswith("k_hop<") and len(args) >= 3 and args[2].strip() == "false"
        mids = [(kk, vv) for kk, vv in hops if middle(kk)]
        kl, vl = max(mids or hops, key=lambda kv: kv[1]["hbm_bytes_per_launch"] or 0)
        res["k_hop_large"] = dict(vl, kernel=kl)
    # bench.py's large-mesh edge-MLP roofline: the grid-stride fused edge MLP + hop without an
    # epilogue (k_edge_hop<NT, ACT, true, 0>); its launches of every scale share one grid, so
    # only the dispatches within 10 % of the largest read (the finest scale's) are averaged
    eh = [key for key in fe if key[0].startswith("k_edge_hop") and key[0].replace(" ", "").endswith(",true,0>")]
    if eh:
        key = max(eh, key=lambda k: max(fe[k]))
        f, w = fe[key], wr.get(key, [])
        fb = [x for x in f if x >= 0.9 * max(f)]
        wb = [x for x in w if w and x >= 0.9 * max(w)]
        rd = 2 * 1024 * sum(fb) / len(fb)
        wbv = 1024 * sum(wb) / len(wb) if wb else 0.0
        res["k_edge_hop_large"] = {"kernel": f"{key[0]} grid={key[1]}", "dispatches": len(fb),
                                   "read_bytes_per_launch": rd, "write_bytes_per_launch": wbv,
                                   "hbm_bytes_per_launch": rd + wbv}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res.get("k_hop"), indent=1))


if __name__ == "__main__":
    main()
