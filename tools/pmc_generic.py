"""Per-kernel averages of any rocprofv3 --pmc pass (counter_collection.csv).

usage: python tools/pmc_generic.py DIR [DIR ...]
Groups dispatches by (kernel name, grid size); prints, per group, the dispatch count, the
average duration and the per-dispatch average of every counter, plus derived ratios where
the counters needed are present (MFMA busy share, wave-parked share, issue-active share)."""
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


def main():
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)
    seen = defaultdict(lambda: defaultdict(set))  # dispatches that reported each counter (one pass each)
    for d in sys.argv[1:]:
        for r in load(d):
            name = r["Kernel_Name"].replace("msw::", "").split("(")[0].replace("void ", "")
            key = (name, int(r["Grid_Size"]))
            did = (d, r["Dispatch_Id"])
            disp[key].add(did)
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            seen[key][r["Counter_Name"]].add(did)
            dur[key][did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for key in sorted(agg, key=lambda k: -sum(dur[k].values())):
        n = len(disp[key])
        c = {k: v / max(len(seen[key][k]), 1) for k, v in agg[key].items()}
        us = sum(dur[key].values()) / max(len(dur[key]), 1)
        line = f"{key[0]:<32} grid={key[1]:>8} n={n:<5} dur={us:9.2f}us"
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
