"""RCCL transport of the single-mesh decomposition (mswegnn/partition.py DistributedRollout):
W processes, one GPU and one part each, the halo exchange over RCCL inside msw_rollout
(grouped ncclSend / ncclRecv) and the owned rows gathered by ONE padded tensor
all-gather over RCCL (gather_owned), compared with the undivided rollout of the same mesh.
Prints one JSON line.  Needs W GPUs (RCCL refuses two ranks on one device); bench.py runs it
at N > 1 with a time limit.

    python tools/rccl_partition_check.py [W] [--mesh zenodo4|hbm1m|small] [--steps 5] [--T 48]

--mesh names a bench.py workload (its mesh, model and weights: zenodo4 = K4_F32 on the
4-scale Zenodo-size mesh, hbm1m = config 5's ~1.3M-node 3-scale mesh, fully wet) or `small`
(K4_F32 on the small test mesh).  The record holds both times, so on the ~1M-node mesh it is
the single-mesh strong-scaling number of SURVEY §8 f2 (undivided / distributed).  After the
eager record the same rollouts run with the RCCL exchanges captured into the rollout graphs
("captured": bit identity to the eager rollout, time; a failure or hang there is recorded under
"captured" and the eager record is kept).
"""
import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def worker(rank, world, port, q, mesh, steps, T):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dev = torch.device(f"cuda:{rank}")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        from conftest import build_msgnn, weights, per_step_rel
        from mswegnn.mesh import make_multiscale_mesh, mesh_config
        from mswegnn.partition import DistributedRollout
        if mesh == "small":
            g = make_multiscale_mesh(**mesh_config(mesh), T=T)
            m = build_msgnn(4, 32, 4, state=weights("K4_F32"))
        else:
            sys.path.insert(0, ROOT)
            import bench
            g, m, _, _ = bench.build_workload(mesh, seed=0, T=T)
        m = m.to(dev)
        m.engine = "hip"
        dr = DistributedRollout(m, g, device=dev)
        x0 = g.x.to(dev)
        out = dr.rollout(x0, g.BC, g.node_BC, g.type_BC, T)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = dr.rollout(x0, g.BC, g.node_BC, g.type_BC, T)
        torch.cuda.synchronize()
        dist.barrier()
        dt = torch.tensor([(time.perf_counter() - t0) / steps], device=dev, dtype=torch.float64)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        full = dr.gather_owned(out)  # RCCL all-gather of the owned rows
        if rank == 0:
            gd = g.to(dev)
            whole = m.rollout(gd)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                whole = m.rollout(gd)
            torch.cuda.synchronize()
            t_whole = (time.perf_counter() - t0) / steps
            lp = dr.part
            q.put({"world": world, "mesh": mesh, "fine_nodes": int(g.node_ptr[1]), "all_nodes": g.num_nodes,
                   "halo_rows_rank0": int((~lp.owned).sum()), "rollout_steps": T,
                   "max_rel_err_vs_undivided": per_step_rel(full.cpu(), whole.cpu()),
                   "bit_identical": bool(torch.equal(full, whole)),
                   "distributed_ms_per_rollout": float(dt.item()) * 1e3,
                   "undivided_ms_per_rollout": t_whole * 1e3,
                   "speedup_vs_undivided": t_whole / float(dt.item()),
                   "transport": "RCCL (msw_plan_set_comm: grouped ncclSend/ncclRecv halo exchange; "
                                "gather_owned: torch.distributed all_gather on nccl)"})
        # then the same rollouts with the RCCL exchanges captured into the plan's rollout graphs
        # (msw_set_graph_capture(plan, 1)): every rank records its sends / receives once and
        # replays them; reported separately (main() keeps the eager record if this part hangs)
        eager_full = full
        try:
            dr.plan.set_graph_capture(1)
            out = dr.rollout(x0, g.BC, g.node_BC, g.type_BC, T)  # captures
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                out = dr.rollout(x0, g.BC, g.node_BC, g.type_BC, T)
            torch.cuda.synchronize()
            dist.barrier()
            dtc = torch.tensor([(time.perf_counter() - t0) / steps], device=dev, dtype=torch.float64)
            dist.all_reduce(dtc, op=dist.ReduceOp.MAX)
            full = dr.gather_owned(out)
            st = dr.plan.stats()
            if rank == 0:
                q.put({"captured": {"bit_identical_to_eager": bool(torch.equal(full, eager_full)),
                                    "distributed_ms_per_rollout": float(dtc.item()) * 1e3,
                                    "graph_captured": st["graph_captured"], "rccl_calls": st["rccl_calls"],
                                    "rccl_steps": st["rccl_steps"]}})
        except Exception as e:  # noqa: BLE001  (recorded under "captured"; the eager record stands)
            q.put({"captured": {"error": repr(e), "rank": rank}})
        dr.close()
    except Exception as e:  # report, do not hang the peer
        q.put({"error": repr(e), "rank": rank})
        raise
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("W", nargs="?", type=int, default=2)
    ap.add_argument("--mesh", default="small")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--T", type=int, default=48)
    ap.add_argument("--wait", type=float, default=240.0, help="seconds to wait for rank 0's records")
    ap.add_argument("--capture-share", type=float, default=0.3,
                    help="share of --wait kept for the captured-exchange part after the eager record")
    a = ap.parse_args()
    if torch.cuda.device_count() < a.W:
        print(json.dumps({"error": f"needs {a.W} GPUs, {torch.cuda.device_count()} visible"}))
        sys.exit(1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=worker, args=(r, a.W, port, q, a.mesh, a.steps, a.T), daemon=True)
             for r in range(a.W)]
    for p in procs:
        p.start()
    t_end = time.perf_counter() + a.wait
    try:
        res = q.get(timeout=a.wait * (1.0 - a.capture_share))
    except Exception:  # noqa: BLE001  (queue.Empty: a rank hung)
        res = {"error": f"no result within {a.wait * (1.0 - a.capture_share):.0f} s"}
    if "error" not in res:
        try:
            res.update(q.get(timeout=max(1.0, t_end - time.perf_counter())))
        except Exception:  # noqa: BLE001
            res["captured"] = {"error": "no captured-exchange result in time (eager record kept)"}
    for p in procs:  # within what is left of --wait (a rank hung in the captured part is killed)
        p.join(max(5.0, t_end - time.perf_counter()))
        if p.is_alive():
            p.kill()
            p.join(5)
    res["exitcodes"] = [p.exitcode for p in procs]
    print(json.dumps(res), flush=True)
    ok = "error" not in res and res["max_rel_err_vs_undivided"] <= 1e-4
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
