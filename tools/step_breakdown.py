"""Per-launch breakdown of one rollout step from a rocprofv3 kernel trace.

usage: python tools/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv [kernels_per_step]
Finds runs of consecutive k_encode-started steps, averages duration and the gap to the
next launch per position in the step."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
kps = int(sys.argv[2]) if len(sys.argv) > 2 else None
starts = [i for i, r in enumerate(rows) if "k_encode" in r["Kernel_Name"]]
if kps is None:  # the most common distance between encoder launches (rollout steps), not the
    # rollout prologue's shorter one
    diffs = [b - a for a, b in zip(starts, starts[1:])]
    kps = max(set(diffs), key=diffs.count)
dur = defaultdict(list)
gap = defaultdict(list)
name = {}
grid = {}
steps = 0
for a in starts:
    seq = rows[a:a + kps]
    if len(seq) < kps or any("k_encode" in r["Kernel_Name"] for r in seq[1:]):
        continue
    if a + kps < len(rows) and "k_encode" not in rows[a + kps]["Kernel_Name"]:
        continue
    steps += 1
    for p, r in enumerate(seq):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[p].append((e - s) / 1e3)
        nx = rows[a + p + 1] if a + p + 1 < len(rows) else None
        if nx is not None:
            gap[p].append((int(nx["Start_Timestamp"]) - e) / 1e3)
        name[p] = r["Kernel_Name"].split("(")[0].replace("void msw::", "").replace(", ", ",")
        grid[p] = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
tot_d = tot_g = 0.0
print(f"{steps} steps of {kps} launches")
for p in range(kps):
    d = sorted(dur[p])[len(dur[p]) // 2]
    g = sorted(gap[p])[len(gap[p]) // 2] if gap[p] else 0.0
    tot_d += d
    tot_g += g
    print(f"{p:3d} {name[p]:28s} wg={grid[p]:6d} dur={d:8.2f}us gap={g:6.2f}us")
print(f"sum dur {tot_d:.1f} us, sum gap {tot_g:.1f} us, step {tot_d + tot_g:.1f} us")
