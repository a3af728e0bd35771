"""Cost of the single-mesh decomposition on one GPU.

Runs the undivided rollout and the in-process partitioned rollout (mswegnn.partition
PartitionedRollout: all W parts stepped in lockstep by msw_group_rollout, halo rows copied
between the parts' buffers) of the same mesh, and reports the time of each and their
parity.  On one GPU the parts run one after the other, so W x (time of one part) ~ the
undivided time plus the decomposition's overhead (halo rows computed twice, exchange
copies, W x the launches): the ratio bounds the strong-scaling efficiency W GPUs could
reach before any interconnect cost.

    python tools/partition_bench.py [--workload zenodo4|hbm1m] [--T 24] [--parts 2 4]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mswe-gnn_amd")]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="zenodo4")
    ap.add_argument("--T", type=int, default=24)
    ap.add_argument("--parts", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--eager", action="store_true",
                    help="step the group eagerly (msw_set_group_graph(plans[0], 0)) instead of its captured graphs")
    a = ap.parse_args()
    import bench
    from mswegnn.partition import PartitionedRollout
    dev = torch.device("cuda", 0)
    g, m, _, desc = bench.build_workload(a.workload, seed=0, T=a.T)
    m = m.to(dev)
    m.engine = "hip"
    gd = g.to(dev)
    t_whole, r_whole = timed(lambda: m.rollout(gd, a.T), a.reps)
    res = {"workload": a.workload, "fine_nodes": desc["fine_nodes"], "all_nodes": desc["all_nodes"],
           "T": a.T, "undivided_ms": t_whole * 1e3, "group": "eager" if a.eager else "graph", "parts": {}}
    ref = r_whole.cpu()
    den = [max(ref[..., t].abs().max().item(), 1e-30) for t in range(a.T)]
    for W in a.parts:
        pr = PartitionedRollout(m, g, W, device=dev)
        if a.eager:
            from mswegnn import _lib as L
            L.check(L.lib().msw_set_group_graph(pr.plans[0]._h, 0))
        t_p, r_p = timed(lambda: pr.rollout(g.x, g.BC, g.node_BC, g.type_BC, a.T), a.reps)
        r_p = r_p.cpu()
        err = max((r_p[..., t] - ref[..., t]).abs().max().item() / den[t] for t in range(a.T))
        halo = sum(int(lp.graph.x.shape[0]) for lp in pr.parts) - desc["all_nodes"]
        res["parts"][W] = {"ms_all_parts_one_gpu": t_p * 1e3, "vs_undivided": t_p / t_whole,
                           "halo_rows": halo, "max_rel_err_vs_undivided": err,
                           "bit_identical": bool(torch.equal(r_p, ref))}
        pr.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
