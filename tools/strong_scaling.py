"""Strong-scaling projection of `bench.py --global-batch G` from ONE GPU.

For W ranks, rank r runs simulations {i : i mod W = r} of a fixed set of G as one batch
(bench.simulations_of_rank / rank_batch).  The W-GPU rollout time is the slowest rank's, so
timing every rank's share on this one GPU, one after the other, gives the W-GPU time
without the end-of-rollout all-gather (a one-shot ≈ G·N0·2·T·4 B collective, priced
separately from xGMI bandwidth).  Output: JSON lines per (G, W) with the per-rank times, the
projected whole-job throughput and the speed-up over W = 1.

    python tools/strong_scaling.py [--workload config3] [--G 8 20 64] [--W 1 2 4 8] [--steps 5]
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

XGMI_GBS = 153.0  # one xGMI link, GB/s per direction (MI355X_MICROARCH.md); ring all-gather is per-link bound


def time_share(workload, ids, T, steps, warmup, dev):
    from mswegnn.engine import plan_for
    sims, gb, rows, fine = bench.rank_batch(workload, ids, T)
    g = gb.to(dev)
    m = sims[0][1].to(dev)
    m.engine = "hip"
    plan = plan_for(m, g)
    out = torch.empty(g.num_nodes, 2, T, device=dev)
    for _ in range(warmup):
        plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, T, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, T, out=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    plan.close()
    del plan, g, out
    torch.cuda.empty_cache()
    return dt, fine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="config3")
    ap.add_argument("--G", type=int, nargs="+", default=[8, 20, 64])
    ap.add_argument("--W", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--T", type=int, default=48)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for G in args.G:
        base = None
        for W in args.W:
            if W > G:
                continue
            ns = argparse.Namespace(global_batch=G, batch=1)
            per_rank = []
            total_fine = 0
            for r in range(W):
                ids, _ = bench.simulations_of_rank(ns, r, W)
                dt, fine = time_share(args.workload, ids, args.T, args.steps, args.warmup, dev)
                per_rank.append(dt)
                total_fine += fine
            t_w = max(per_rank)
            gather_bytes = total_fine * 2 * args.T * 4 * (W - 1) / W if W > 1 else 0
            t_gather = gather_bytes / (XGMI_GBS * 1e9)
            val = total_fine * args.T / t_w
            val_g = total_fine * args.T / (t_w + t_gather)
            if W == 1:
                base = val
            print(json.dumps({"workload": args.workload, "G": G, "W": W, "T": args.T,
                              "rank_rollout_ms": [round(x * 1e3, 3) for x in per_rank],
                              "projected_ms": t_w * 1e3, "fine_node_steps_per_s": val,
                              "allgather_est_ms": t_gather * 1e3,
                              "fine_node_steps_per_s_with_allgather": val_g,
                              "speedup_vs_W1": val / base if base else None,
                              "speedup_vs_W1_with_allgather": val_g / base if base else None}),
                  flush=True)


if __name__ == "__main__":
    main()
