"""Data-parallel training through the HIP training kernels: W processes wrap the
drop-in MSGNN in torch DistributedDataParallel -- what the reference's Lightning Trainer
(main.py:106-119, accelerator / devices 'auto') does on a multi-GPU node -- and run one
training step (loss backward with every layer on mswegnn/autograd.py's Functions, DDP's
gradient all-reduce hooks on the parameters).  Rank 0 checks the all-reduced gradients
against one process computing the mean of the W ranks' loss gradients itself.

    python tools/ddp_train_check.py [W] [--backend gloo|nccl]

nccl (RCCL) needs W GPUs, one per rank; gloo runs every rank on cuda:0 (the one-GPU box:
tests/test_gpu_train.py).  Prints one JSON line; exit 0 when the gradients agree to 1e-5.
"""
import argparse
import json
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def _setup(dev):
    from conftest import build_msgnn, weights
    from mswegnn.mesh import make_multiscale_mesh, mesh_config, wet_state
    g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), T=4), seed=1).to(dev)
    m = build_msgnn(4, 32, 4, state=weights("K4_F32")).to(dev)
    m.train()
    return g, m


def _target(g, r, dev):
    return torch.rand(g.x.shape[0], 2, device=dev, generator=torch.Generator(dev).manual_seed(100 + r))


def worker(rank, world, port, q, backend):
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dev = torch.device("cuda", rank if backend == "nccl" else 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from mswegnn import autograd as ag
        g, m = _setup(dev)
        ddp = DDP(m, device_ids=[dev.index])
        ((ddp(g) - _target(g, rank, dev)) ** 2).mean().backward()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
        hip_ran = ag.MLP_CALLS[0] > 0 and ag.POOL_CALLS[0] > 0 and len(ag._CSR_CACHE) > 0
        dist.barrier()
        if rank == 0:
            g2, m2 = _setup(dev)  # one process: the mean of the W ranks' loss gradients
            m2.zero_grad(set_to_none=True)
            for r in range(world):
                (((m2(g2) - _target(g2, r, dev)) ** 2).mean() / world).backward()
            ref = {n: p.grad.detach() for n, p in m2.named_parameters() if p.grad is not None}
            worst = max(((grads[k] - ref[k]).abs().max() / ref[k].abs().max().clamp(min=1e-30)).item() for k in ref)
            q.put({"world": world, "backend": backend, "devices": "one per rank" if backend == "nccl" else "cuda:0",
                   "gradients": len(ref), "same_parameter_set": grads.keys() == ref.keys(),
                   "max_rel_err_vs_single_process_mean": worst, "hip_training_kernels_ran": bool(hip_ran),
                   "wrapper": "torch.nn.parallel.DistributedDataParallel"})
    except Exception as e:  # report, do not hang the peers
        q.put({"error": repr(e), "rank": rank})
        raise
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("W", nargs="?", type=int, default=2)
    ap.add_argument("--backend", default="gloo", choices=["gloo", "nccl"])
    ap.add_argument("--wait", type=float, default=150.0)
    a = ap.parse_args()
    if a.backend == "nccl" and torch.cuda.device_count() < a.W:
        print(json.dumps({"error": f"nccl needs {a.W} GPUs, {torch.cuda.device_count()} visible"}))
        sys.exit(1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=worker, args=(r, a.W, port, q, a.backend), daemon=True) for r in range(a.W)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=a.wait)
    except Exception:  # noqa: BLE001  (queue.Empty: a rank hung)
        res = {"error": f"no result within {a.wait:.0f} s"}
    for p in procs:
        p.join(60)
        if p.is_alive():
            p.kill()
    res["exitcodes"] = [p.exitcode for p in procs]
    print(json.dumps(res), flush=True)
    ok = ("error" not in res and res["same_parameter_set"] and res["hip_training_kernels_ran"]
          and res["max_rel_err_vs_single_process_mean"] <= 1e-5)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
