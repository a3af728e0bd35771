"""One-rank nccl (RCCL) process group on one GPU: the torch.distributed side of the multi-GPU
path, run by tests/test_gpu_rccl.py::test_nccl_world1_process_group in a fresh process.

  1. bench.make_gatherer's end-of-rollout all-gather (bench.py) over RCCL, world size 1
     (the sizes exchange and the payload all-gather);
  2. DistributedRollout (mswegnn/partition.py): the rank-0 ncclGetUniqueId, its broadcast over
     the process group and ncclCommInitRank inside the engine (msw_plan_set_comm), the rollout,
     and gather_owned's all-gather of the owned rows -- against the plain plan bit for bit.
Prints one JSON record."""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=dev)
    rec = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    import bench
    from conftest import build_msgnn, weights
    from mswegnn.mesh import make_multiscale_mesh, mesh_config
    from mswegnn.partition import DistributedRollout

    T = 12
    g = make_multiscale_mesh(**mesh_config("small"), T=T).to(dev)
    m = build_msgnn(4, 32, 4, state=weights("K4_F32")).to(dev)
    m.engine = "hip"
    whole = m.rollout(g, T).clone()
    n0 = int(g.node_ptr[1])
    gather = bench.make_gatherer(dist, 1, n0, T, dev)
    got = gather(whole[:n0])
    rec["gather_equal"] = len(got) == 1 and torch.equal(got[0], whole[:n0])
    # a second gatherer (its own size exchange) on a row slice of the rollout
    gather_s = bench.make_gatherer(dist, 1, n0 - 7, T, dev)
    got_s = gather_s(whole[7:n0])
    rec["gather_second_equal"] = torch.equal(got_s[0], whole[7:n0])

    dr = DistributedRollout(m, g, dev)
    rec["comm_set"] = True  # msw_plan_set_comm raised otherwise
    out = dr.rollout(g.x, g.BC, g.node_BC, g.type_BC, T)
    rec["distributed_rollout_equal"] = torch.equal(out, whole)
    full = dr.gather_owned(out)
    rec["gather_owned_equal"] = torch.equal(full, whole)
    torch.cuda.synchronize()
    rec["stats"] = {k: v for k, v in dr.plan.stats().items() if k in ("rollout_steps", "rccl_calls", "rccl_steps")}
    dr.close()
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
