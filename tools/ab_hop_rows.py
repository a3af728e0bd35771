"""A/B of the row-layout middle hop (k_hop_rows) against the edge-tile k_hop on the ~1M-node
mesh (config 5) in ONE process: per setting of MSW_HOP_ROWS a fresh plan, the finest middle
hop timed with HIP events on the launching stream (bench.time_kernel), a 10-step rollout, and
the rollout compared bit for bit with the first setting's.  The library variant comes from
MSW_LIB_VARIANT (build_engine.py --variant=rdc2 / rdc3: edges in flight per lane).

    python tools/ab_hop_rows.py [--settings 0 1] [--T 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mswe-gnn_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--settings", nargs="+", default=["0", "1"])
    ap.add_argument("--T", type=int, default=10)
    ap.add_argument("--workload", default="hbm1m")
    a = ap.parse_args()
    from mswegnn.engine import EnginePlan
    dev = torch.device("cuda", 0)
    g, m, w, desc = bench.build_workload(a.workload, seed=0, T=a.T)
    g = g.to(dev)
    m = m.to(dev)
    F = desc["hid_features"]
    ref = None
    for sv in a.settings:
        os.environ["MSW_HOP_ROWS"] = sv
        plan = EnginePlan(m, g, dev)
        out = plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, a.T)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            out = plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, a.T)
        torch.cuda.synchronize()
        t_roll = (time.perf_counter() - t0) / 3
        th, (rows, edges) = bench.time_kernel(plan, "hop", 0, iters=50)
        hb = edges * (4 * F + 4) + rows * (12 * F + 4)
        res = {"MSW_HOP_ROWS": sv, "lib": os.environ.get("MSW_LIB_VARIANT", ""), "workload": a.workload,
               "hop_us": th * 1e6, "hop_GBs": hb / th / 1e9, "hop_frac": hb / th / 1e9 / 8000.0,
               "rollout_ms": t_roll * 1e3, "fine_node_steps_per_s": desc["fine_nodes"] * a.T / t_roll,
               "kernels_per_step": plan.stats()["kernels_per_step"]}
        if ref is None:
            ref = out.clone()
        else:
            res["bit_identical_to_first"] = bool(torch.equal(out, ref))
            res["max_abs_diff"] = float((out - ref).abs().max())
        print(json.dumps(res), flush=True)
        plan.close()
        del out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
