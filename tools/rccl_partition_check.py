"""RCCL transport of the single-mesh decomposition (mswegnn/partition.py DistributedRollout):
W processes, one part each, halo exchange over RCCL inside msw_rollout, compared with the
undivided rollout of the same mesh.  On a multi-GPU node every rank takes its own GPU; with
one GPU all ranks share cuda:0 (works only if RCCL accepts several ranks per device).

    python tools/rccl_partition_check.py [W]
"""
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    ndev = torch.cuda.device_count()
    dev = torch.device(f"cuda:{rank % ndev}")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from conftest import build_msgnn, weights, per_step_rel
        from mswegnn.mesh import make_multiscale_mesh, mesh_config
        from mswegnn.partition import DistributedRollout
        g = make_multiscale_mesh(**mesh_config("small"), T=48)
        m = build_msgnn(4, 32, 4, state=weights("K4_F32")).to(dev)
        m.engine = "hip"
        dr = DistributedRollout(m, g, device=dev)
        out = dr.rollout(g.x.to(dev), g.BC, g.node_BC, g.type_BC, 48)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            out = dr.rollout(g.x.to(dev), g.BC, g.node_BC, g.type_BC, 48)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        full = dr.gather_owned(out)
        if rank == 0:
            whole = m.rollout(g.to(dev)).cpu()
            q.put((per_step_rel(full, whole), dt))
        dr.close()
    except Exception as e:  # report, do not hang the peer
        q.put(("error", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=worker, args=(r, W, port, q)) for r in range(W)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(60)
    print({"world": W, "result": res, "exitcodes": [p.exitcode for p in procs]})
    ok = res[0] != "error" and res[0] <= 1e-4
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
