"""CPU-side tests: the C ABI library (loads, exports every symbol include/mswegnn.h declares,
struct layouts agree with the ctypes binding), the synthetic mesh generator, the drop-in
model modules' torch path, batching, and the multi-rank (gloo, world size 2) rollout
sharding + end-of-rollout all-gather of bench.py.  No GPU is touched.
"""
import ctypes as C
import os
import re
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT, PKG, build_msgnn, golden, manifest, per_step_rel, rel_err, weights
import msgnn_torch as orc
from mswegnn.mesh import make_multiscale_mesh, make_single_scale_mesh, mesh_config, wet_state

HEADER = os.path.join(ROOT, "include", "mswegnn.h")


@pytest.fixture(scope="module")
def libso():
    from mswegnn import _lib
    if not os.path.exists(_lib.LIB_PATH):  # the driver may run the CPU suite before build()
        sys.path.insert(0, PKG)
        import build_engine
        build_engine.build(verbose=False)
    return C.CDLL(_lib.LIB_PATH)


def _header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(msw_\w+)\s*\(", text, flags=re.M)))


def test_abi_exports_every_header_symbol(libso):
    from mswegnn import _lib
    names = _header_functions()
    assert len(names) >= 12, names
    for n in names:
        assert hasattr(libso, n), f"{n} declared in include/mswegnn.h but not exported"
    bound = {s[0] for s in _lib.SYMBOLS}
    assert set(names) == bound, f"ctypes binding and header differ: {set(names) ^ bound}"


def test_abi_struct_layouts_and_version(libso):
    from mswegnn import _lib
    libso.msw_struct_size.restype = C.c_int64
    libso.msw_struct_size.argtypes = [C.c_char_p]
    for name, cls in _lib.STRUCTS.items():
        assert libso.msw_struct_size(name.encode()) == C.sizeof(cls), name
    assert libso.msw_struct_size(b"nope") == -1
    libso.msw_abi_version.restype = C.c_int
    assert libso.msw_abi_version() == 1
    libso.msw_last_error.restype = C.c_char_p
    assert isinstance(libso.msw_last_error(), bytes)


def test_abi_rejects_null_arguments_without_gpu(libso):
    """Argument validation happens before any HIP call: null plans / descriptors are
    reported through the error code + msw_last_error, never a crash."""
    libso.msw_plan_create.restype = C.c_int
    libso.msw_last_error.restype = C.c_char_p
    out = C.c_void_p()
    assert libso.msw_plan_create(None, None, 0, C.byref(out)) != 0
    assert b"null" in libso.msw_last_error()
    libso.msw_forward.restype = C.c_int
    assert libso.msw_forward(None, None, None, None) != 0
    assert libso.msw_plan_destroy(None) == 0


def test_mesh_generator_invariants():
    """Appendix B / SURVEY §8 sizes and the structural facts the engine relies on."""
    g = make_multiscale_mesh(**mesh_config("zenodo4"), T=4)
    npt = g.node_ptr.tolist()
    assert [npt[i + 1] - npt[i] for i in range(4)] == [10369, 2593, 649, 163]
    ept = g.edge_ptr.tolist()
    assert [ept[i + 1] - ept[i] for i in range(4)] == [30817, 7633, 1873, 451]
    ei = g.edge_index
    for s in range(4):
        e = ei[:, ept[s]:ept[s + 1]]
        assert ((e >= npt[s]) & (e < npt[s + 1])).all(), "edge leaves its scale"
        deg = torch.bincount(e[1] - npt[s], minlength=npt[s + 1] - npt[s])
        assert int(deg.max()) <= 16, "in-degree above the 16-edge tile bound"
    ii, ip = g.intra_mesh_edge_index, g.intra_edge_ptr.tolist()
    for l in range(3):
        e = ii[:, ip[l]:ip[l + 1]]
        assert ((e[0] >= npt[l + 1]) & (e[0] < npt[l + 2])).all()  # row = coarse
        assert ((e[1] >= npt[l]) & (e[1] < npt[l + 1])).all()      # col = fine
        parents = torch.bincount(e[1] - npt[l], minlength=npt[l + 1] - npt[l])
        assert int(parents.max()) <= 1
    assert int(g.node_BC.max()) < npt[1]
    assert g.x.shape == (npt[-1], 8) and g.BC.shape[1:] == (3, 5)


def test_drop_in_model_torch_path_matches_reference_fixture():
    """models.gnn.MSGNN (torch path: CPU tensors) reproduces the reference's output."""
    fx = golden("fx_tiny_K4_F32_step")
    g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), T=48), seed=1)
    m = build_msgnn(4, 32, 4, state=weights("K4_F32"))
    with torch.no_grad():
        y = m(g)
    assert rel_err(y, fx["y"]) <= 1e-5


def test_drop_in_model_rollout_torch_path():
    fx = golden("fx_small_K2_F16_rollout48")
    g = make_multiscale_mesh(**mesh_config("small"), T=48)
    m = build_msgnn(4, 16, 2, state=weights("K2_F16"))
    m.engine = "torch"
    r = m.rollout(g, 12)
    assert per_step_rel(r, torch.from_numpy(fx["rollout"][..., :12])) <= 1e-5


def test_gpu_engine_refuses_cpu_tensors():
    """engine='hip' never falls back silently."""
    g = make_multiscale_mesh(**mesh_config("tiny"), T=4)
    m = build_msgnn(4, 32, 4, state=weights("K4_F32"))
    m.engine = "hip"
    with pytest.raises(Exception):
        with torch.no_grad():
            m(g)


def test_collate_matches_individual_oracle():
    """Disjoint-union batch (update_batch_multiscale layout) == per-graph results."""
    from mswegnn.batch import collate
    ga = make_multiscale_mesh(n_coarse=2, num_scales=4, seed=1, T=3)
    gb = make_multiscale_mesh(n_coarse=3, num_scales=4, seed=2, T=3)
    from training.train import adapt_batch_training
    bt = adapt_batch_training(collate([ga, gb]))
    assert tuple(bt.node_ptr.shape) == (2, 5)
    cfg = manifest()["weights_K4_F32_cfg"]
    P = weights("K4_F32")
    r = orc.rollout(P, cfg, bt)
    ra, rb = orc.rollout(P, cfg, ga), orc.rollout(P, cfg, gb)
    na = ga.num_nodes
    # batched CPU matmuls block rows differently: equal to float rounding, not bit for bit
    assert rel_err(r[:na], ra) <= 1e-5 and rel_err(r[na:], rb) <= 1e-5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, T, q):
    import torch.distributed as dist
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    g, m, w, desc = bench.build_workload("tiny", seed=rank, T=T)
    m.engine = "torch"
    out = m.rollout(g, T)
    gather = bench.make_gatherer(dist, world, desc["fine_nodes"], T, torch.device("cpu"))
    parts = gather(out[:desc["fine_nodes"]].contiguous())
    if rank == 0:
        q.put([p.clone().numpy() for p in parts])
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_and_allgather_gloo():
    """bench.py's N>1 path on CPU: rank r simulates seed r, ONE all-gather at the end
    delivers every rank's fine-scale rollout to every rank."""
    T, world = 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    import bench
    for r in range(world):
        g, m, w, desc = bench.build_workload("tiny", seed=r, T=T)
        m.engine = "torch"
        ref = m.rollout(g, T)[:desc["fine_nodes"]]
        assert np.array_equal(parts[r], ref.numpy()), f"rank {r} slot"
    assert not np.array_equal(parts[0], parts[1]), "ranks must simulate different seeds"


def test_metrics_oracle_matches_reference_fixture():
    """oracle/metrics_ref.py reproduces the reference's own evaluation functions
    (fx_metrics.npz, made by oracle/gen_golden_metrics.py from utils/miscellaneous.py)."""
    import metrics_ref as mr
    fx = golden("fx_metrics")
    n0 = int(fx["n0"])
    real = torch.from_numpy(golden("fx_small_K4_F32_rollout48")["rollout"])[:n0]
    pred = torch.from_numpy(golden("fx_small_K2_F16_rollout48")["rollout"])[:n0]
    for tl in ("RMSE", "MAE"):
        assert torch.equal(mr.rollout_loss(pred, real, tl), torch.from_numpy(fx[f"loss_{tl}"]))
        assert torch.equal(mr.rollout_loss(pred, real, tl, True), torch.from_numpy(fx[f"loss_{tl}_water"]))
    for thr in (0.05, 0.3):
        np.testing.assert_array_equal(mr.csi(pred, real, thr).numpy(), fx[f"csi_{thr}"])
        np.testing.assert_array_equal(mr.f1(pred, real, thr).numpy(), fx[f"f1_{thr}"])
    p2, r2 = torch.stack([pred, real.flip(-1)]), torch.stack([real, pred])
    assert torch.equal(mr.rollout_loss(p2, r2, "RMSE"), torch.from_numpy(fx["loss_RMSE_stack"]))
    np.testing.assert_array_equal(mr.csi(p2, r2, 0.05).numpy(), fx["csi_0.05_stack"])
