"""Cross-check bench.py's live roofline timing against the rocprofv3 kernel trace of the
same command: bench.py times `iters` back-to-back launches of one kernel with HIP events
(msw_bench_kernel); this finds those runs in the trace (>= 20 consecutive launches of one
kernel name) and reports their average duration and their launch-to-launch period (what
the HIP events measure: duration + boundary).

    python tools/roofline_check.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    runs, i = [], 0
    while i < len(rows):
        j = i
        while j + 1 < len(rows) and rows[j + 1]["Kernel_Name"] == rows[i]["Kernel_Name"]:
            j += 1
        if j - i + 1 >= 20:
            runs.append(rows[i:j + 1])
        i = j + 1
    for run in runs:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in run]
        span = (int(run[-1]["End_Timestamp"]) - int(run[0]["Start_Timestamp"])) / 1e3
        grid = run[0].get("Grid_Size", run[0].get("Grid_Size_X", "?"))
        print(f"{run[0]['Kernel_Name'][:60]:60s} grid={grid:>8} launches={len(run):4d} "
              f"avg duration {sum(d) / len(d):9.2f} us  period {span / len(run):9.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
