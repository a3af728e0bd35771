"""Cross-check bench.py's live roofline timing against the rocprofv3 kernel trace of the
same command: bench.py times back-to-back launches of one kernel with HIP events
(msw_bench_kernel); this finds those runs in the trace (>= 20 consecutive launches of one
kernel name) and reports their average duration and their launch-to-launch period (what
the HIP events measure: duration + boundary).

    python tools/roofline_check.py gpurun_out/prof/run_kernel_trace.csv [--json out.json]

--json: the runs in bench.py's order (default workload: finest middle hop, fused edge MLP +
hop, pooling; then the ~1M-node mesh's middle hop and edge MLP + hop), named by role -- the
file bench.py reads into `roofline.rocprof` (profiles/roofline_rocprof.json).
"""
import csv
import json
import sys

ROLES = ["hop", "edge_hop", "pool", "hop_large", "edge_hop_large"]


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


def runs_of(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    runs, i = [], 0
    while i < len(rows):
        j = i
        while j + 1 < len(rows) and rows[j + 1]["Kernel_Name"] == rows[i]["Kernel_Name"]:
            j += 1
        if j - i + 1 >= 20:
            runs.append(rows[i:j + 1])
        i = j + 1
    out = []
    for run in runs:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in run]
        span = (int(run[-1]["End_Timestamp"]) - int(run[0]["Start_Timestamp"])) / 1e3
        grid = run[0].get("Grid_Size", run[0].get("Grid_Size_X", "?"))
        out.append({"kernel": run[0]["Kernel_Name"].split("(")[0].replace("void msw::", "").replace("msw::", ""),
                    "grid": grid,
                    "launches": len(run), "avg_duration_us": sum(d) / len(d), "period_us": span / len(run)})
    return out


def roles_of(runs):
    """bench.py's timing runs by role, in its order: the default workload's finest middle hop
    (k_hop), fused edge MLP + hop (k_edge_hop), pooling (k_pool*, when the schedule has a
    pooling launch), then the ~1M-node mesh's middle hop (k_hop / k_hop_rows) and edge MLP +
    hop -- matched by kernel kind, so a role the run does not time is absent, never shifted."""
    ours = [r for r in runs if r["kernel"].startswith("k_")]  # engine kernels only
    kind = {"hop": ("k_hop<", "k_hop_rows", "k_hop_split"), "edge_hop": ("k_edge_hop",), "pool": ("k_pool",)}
    want = [("hop", "hop"), ("edge_hop", "edge_hop"), ("pool", "pool"), ("hop_large", "hop"),
            ("edge_hop_large", "edge_hop")]
    out, i = {}, 0
    for role, k in want:
        for j in range(i, len(ours)):
            if ours[j]["kernel"].startswith(kind[k]):
                out[role] = ours[j]
                i = j + 1
                break
    return out


def main(argv):
    path = argv[1]
    runs = runs_of(path)
    for r in runs:
        print(f"{r['kernel'][:60]:60s} grid={r['grid']:>8} launches={r['launches']:4d} "
              f"avg duration {r['avg_duration_us']:9.2f} us  period {r['period_us']:9.2f} us")
    if "--json" in argv:
        out = argv[argv.index("--json") + 1]
        with open(out, "w") as f:
            json.dump({"source": path, "library_sha256": library_sha256(), "runs": runs,
                       "by_role": roles_of(runs)}, f, indent=1)


if __name__ == "__main__":
    main(sys.argv)
