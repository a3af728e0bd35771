"""A few rollout steps of one workload and nothing else -- the program to run under a
rocprofv3 --pmc pass (every dispatch is serialised with its counters there, so bench.py's
timing loops take minutes).

    rocprofv3 --pmc ... -- python3 tools/pmc_step.py [workload] [T]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mswe-gnn_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from mswegnn.engine import plan_for  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "zenodo4"
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda:0")
    g, m, _, _ = bench.build_workload(wl, seed=0, T=T)
    g = g.to(dev)
    m = m.to(dev)
    m.engine = "hip"
    plan = plan_for(m, g)
    print(f"{wl}: plan ready", flush=True)
    plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, T)
    torch.cuda.synchronize()
    print(f"{wl}: {T}-step rollout done", flush=True)


if __name__ == "__main__":
    main()
