"""Per-kernel averages of any rocprofv3 --pmc pass (counter_collection.csv).

usage: python tools/pmc_generic.py [--split-duration] DIR [DIR ...]
Groups dispatches by (kernel name, grid size); prints, per group, the dispatch count, the
average duration and the per-dispatch average of every counter, plus derived ratios where
the counters needed are present (MFMA busy share, wave-parked share, issue-active share).
--split-duration: a group whose dispatches are different launches of the same kernel with the
same (capped) grid -- e.g. config 5's fused edge MLP + hop on the finest and on the next scale,
both at the resident-grid cap -- is split at its largest duration ratio between consecutive
sorted dispatches (> 1.5x), so each launch's counters are averaged over that launch alone.
Each pass of a multi-pass collection sees the same launches, so the split applies per pass."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for p in path:
        rows += list(csv.DictReader(open(p)))
    return rows


def duration_class(rows_by_key):
    """{(dir, dispatch id): class index} per (name, grid) group: 0 = the shorter launches, 1 =
    the longer ones, split at the largest ratio (> 1.5x) between consecutive sorted durations."""
    cls = {}
    for key, items in rows_by_key.items():
        durs = sorted(set(items.values()))
        cut = None
        best = 1.5
        for a, b in zip(durs, durs[1:]):
            if a > 0 and b / a > best:
                best, cut = b / a, b
        for did, us in items.items():
            cls[(key, did)] = 0 if cut is None or us < cut else 1
    return cls


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    split = "--split-duration" in sys.argv
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)
    seen = defaultdict(lambda: defaultdict(set))  # dispatches that reported each counter (one pass each)
    cls = {}
    if split:
        by = defaultdict(dict)
        for d in args:
            for r in load(d):
                name = r["Kernel_Name"].replace("msw::", "").split("(")[0].replace("void ", "")
                by[(name, int(r["Grid_Size"]))][(d, r["Dispatch_Id"])] = \
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cls = duration_class(by)
    for d in args:
        for r in load(d):
            name = r["Kernel_Name"].replace("msw::", "").split("(")[0].replace("void ", "")
            key = (name, int(r["Grid_Size"]))
            if split:
                key = key + (cls[(key, (d, r["Dispatch_Id"]))],)
            did = (d, r["Dispatch_Id"])
            disp[key].add(did)
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            seen[key][r["Counter_Name"]].add(did)
            dur[key][did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for key in sorted(agg, key=lambda k: -sum(dur[k].values())):
        n = len(disp[key])
        c = {k: v / max(len(seen[key][k]), 1) for k, v in agg[key].items()}
        us = sum(dur[key].values()) / max(len(dur[key]), 1)
        line = f"{key[0]:<32} grid={key[1]:>8}" + (f" cls={key[2]}" if len(key) > 2 else "") + f" n={n:<5} dur={us:9.2f}us"
        for k in sorted(c):
            line += f" {k}={c[k]:.4g}"
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in c:
                    line += f" {k[3:]}/WAVE={c[k] / wc:.2f}"
        bc = c.get("SQ_BUSY_CYCLES")
        if bc and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            line += f" MFMA_BUSY/BUSY={c['SQ_VALU_MFMA_BUSY_CYCLES'] / bc:.3f}"
        print(line)


if __name__ == "__main__":
    main()
