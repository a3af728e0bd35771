"""CPU-side tests: the C ABI library (loads, exports every symbol include/mswegnn.h declares,
struct layouts agree with the ctypes binding), the synthetic mesh generator, the drop-in
model modules' torch path, batching, and the multi-rank (gloo, world size 2) rollout
sharding + end-of-rollout all-gather of bench.py.  No GPU is touched.
"""
import ctypes as C
import os
import re
import socket
import time
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


def test_training_abi_validation_and_workspace_without_gpu(libso):
    """The training entry points (msw_mlp_train_*, msw_swegnn_train_*, msw_pool_mean_*) size
    their workspaces and reject inconsistent descriptors / null buffers on the host, before
    any HIP call (no GPU here)."""
    from mswegnn import _lib as L
    lib = L.lib()
    d = L.MswMlpTrainDesc()
    d.rows, d.n_layers = 100, 3
    for i, w in enumerate((9, 32, 32, 2)):
        d.width[i] = w
    s, t = C.c_int64(), C.c_int64()
    assert lib.msw_mlp_train_workspace(C.byref(d), C.byref(s), C.byref(t)) != 0  # weights missing
    for i in range(3):
        d.weight[i] = 16  # any non-null address: the workspace call only validates
    assert lib.msw_mlp_train_workspace(C.byref(d), C.byref(s), C.byref(t)) == 0
    al = lambda n: (n + 63) // 64 * 64  # noqa: E731
    assert s.value == al(100 * 32) + al(100 * 32) + al(100 * 2) + al(100 * 32) + al(100 * 32)
    # scratch: two [rows][max width] buffers, fp64 split-K partials (splits = max(1, rows / 128)
    # slices of [max width][max width + 1] doubles), fp64 slope partials
    assert t.value == 2 * al(100 * 32) + al(2 * 1 * 32 * 33) + al(256 * 4)
    assert lib.msw_mlp_train_forward(C.byref(d), None, None, None, None) != 0
    assert b"null" in lib.msw_last_error()
    d.width[3] = 0
    assert lib.msw_mlp_train_workspace(C.byref(d), C.byref(s), C.byref(t)) != 0
    sd = L.MswSwegnnTrainDesc()
    sd.num_nodes, sd.num_edges, sd.F, sd.edge_features, sd.K, sd.n_layers = 10, 30, 32, 32, 4, 3
    for i, w in enumerate((160, 64, 64, 32)):
        sd.width[i] = w
    assert lib.msw_swegnn_train_workspace(C.byref(sd), C.byref(s), C.byref(t)) == 0 and s.value > 0
    sd.width[0] = 161  # != 4F + edge_features
    assert lib.msw_swegnn_train_workspace(C.byref(sd), C.byref(s), C.byref(t)) != 0
    assert lib.msw_pool_mean_forward(-1, 32, None, None, None, None, None, None) != 0
    assert lib.msw_pool_mean_forward(0, 32, None, None, None, None, None, None) == 0  # nothing to do
    assert lib.msw_pool_mean_backward(5, 32, None, None, None, None, None, None, None) != 0


def test_training_descriptor_cache_keys_follow_parameters():
    """mswegnn/autograd.py reuses a layer's descriptor template while the layer holds the same
    parameter objects: the validation list (_param_list) is the descriptor's own binding order
    for every SWEGNN layer and make_mlp stack of the model, and a replaced Parameter changes it."""
    from conftest import build_msgnn
    from mswegnn import autograd as ag
    m = build_msgnn(4, 32, 4)
    g = make_multiscale_mesh(**mesh_config("tiny"), T=2)
    csr = ag.GraphCSR(g.edge_index, g.num_nodes)
    for layer in list(m.gnn_processor) + list(m.intra_scale_gnn):
        ef = int(layer.edge_features) if layer.edge_features > 0 else 0
        meta = ag._Meta(layer, ag._mlp_layers(layer.edge_mlp), csr, 32, ef)
        assert [id(p) for p in meta.params] == [id(p) for p in ag._param_list(layer)]
    for seq in (m.edge_encoder, m.static_node_encoder, m.dynamic_node_encoder, m.node_decoder):
        meta = ag._MlpMeta(ag._mlp_layers(seq), 7)
        assert [id(p) for p in meta.params] == [id(p) for p in ag._param_list(seq=seq)]
    layer = m.gnn_processor[0]
    before = ag._param_list(layer)
    layer.filter_matrix[1].weight = torch.nn.Parameter(layer.filter_matrix[1].weight.detach().clone())
    after = ag._param_list(layer)
    assert len(before) == len(after) and any(a is not b for a, b in zip(before, after))


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
    from mswegnn.rollout import adapt_batch_training
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


def _rank_main(rank, world, port, T, q, workload, global_batch):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    torch.set_num_threads(2)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import argparse
    import bench
    args = argparse.Namespace(global_batch=global_batch, batch=1)
    ids, scaling = bench.simulations_of_rank(args, rank, world, workload)
    sims, gb, rows, fine = bench.rank_batch(workload, ids, T)
    m = sims[0][1]
    m.engine = "torch"
    out = m.rollout(gb, T)
    gather = bench.make_gatherer(dist, world, fine, T, torch.device("cpu"))
    parts = gather((out[:fine] if rows is None else out.index_select(0, rows)).contiguous())
    if rank == 0:
        q.put(([p.clone().numpy() for p in parts], scaling))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("workload,global_batch", [("tiny_mixed", 0), ("tiny_mixed", 3)])
def test_two_rank_sharding_and_allgather_gloo(workload, global_batch):
    """bench.py's N>1 path on CPU, world size 2.  Weak (global_batch 0): rank r simulates
    seed r.  Strong (--global-batch 3): the fixed set {0, 1, 2} (fine nodes 513, 1153, 513)
    split by size (longest processing time first): rank 0 runs {1}, rank 1 runs {0, 2} as
    one batch.  Ranks hold meshes of different sizes, so the all-gather pads; ONE all-gather
    at the end delivers every rank's fine-scale rollouts."""
    T, world = 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, T, q, workload, global_batch))
             for r in range(world)]
    for p in procs:
        p.start()
    parts, scaling = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    import bench
    assert scaling == ("strong" if global_batch else "weak")
    owners = [[1], [0, 2]] if global_batch else [[0], [1]]
    assert parts[0].shape[0] != parts[1].shape[0], "ranks must hold different mesh sizes (padding path)"
    for r in range(world):
        refs = []
        for i in owners[r]:
            g, m, w, desc = bench.build_workload(workload, seed=i, T=T)
            m.engine = "torch"
            refs.append(m.rollout(g, T)[:desc["fine_nodes"]])
        ref = torch.cat(refs).numpy()
        assert parts[r].shape == ref.shape, (r, parts[r].shape, ref.shape)
        assert np.abs(parts[r] - ref).max() <= 1e-5 * max(np.abs(ref).max(), 1e-30), f"rank {r} slot"


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
    # mass conservation (get_mass_conservation_loss), bit-exact in the reference's fp32 order
    npt = torch.tensor([0, n0])
    args = (torch.from_numpy(fx["mass_area"]), npt, torch.from_numpy(fx["mass_bc"]),
            torch.from_numpy(fx["mass_node_bc"]).long(), torch.from_numpy(fx["mass_edge_bc_length"]),
            torch.from_numpy(fx["mass_temporal_res"]))
    assert torch.equal(mr.mass_conservation_loss(pred, *args), torch.from_numpy(fx["mass_loss_pred"]))
    assert torch.equal(mr.mass_conservation_loss(real, *args), torch.from_numpy(fx["mass_loss_real"]))


# ------------------------------------------------------------------ single-mesh decomposition
def _hops_part(lp, xl, exchange, hops):
    """`hops` rounds of y[dst] += w_e * x[src] over the part's local edges, the halo refreshed
    by `exchange` before every round and poisoned (NaN) after it, as the engine's hop chain
    runs (mswegnn/partition.py): an owned row reached by a stale halo row turns NaN."""
    ei = lp.graph.edge_index.numpy()
    w = lp.graph.edge_attr.reshape(ei.shape[1], -1)[:, 0].double().numpy()
    halo = ~lp.owned
    for _ in range(hops):
        exchange(xl)
        y = np.zeros_like(xl)
        np.add.at(y, ei[1], w[:, None] * xl[ei[0]])
        y[halo] = np.nan
        xl[:] = y
    return xl


def _hops_global(g, x, hops):
    ei = g.edge_index.numpy()
    w = g.edge_attr.reshape(ei.shape[1], -1)[:, 0].double().numpy()
    for _ in range(hops):
        y = np.zeros_like(x)
        np.add.at(y, ei[1], w[:, None] * x[ei[0]])
        x = y
    return x


@pytest.mark.parametrize("parts", [2, 3, 5])
def test_partition_invariants_and_halo_exchange(parts):
    from mswegnn import partition as P
    g = make_multiscale_mesh(**mesh_config("small"), T=4)
    owner, lps, xp = P.decompose(g, parts)
    npt = g.node_ptr.numpy()
    N = int(npt[-1])
    ii = g.intra_mesh_edge_index.numpy()
    # every node owned once; nested (a fine node lives with its parent); finest balanced
    assert owner.min() == 0 and owner.max() == parts - 1
    assert np.array_equal(owner[ii[1]], owner[ii[0]])
    counts = np.bincount(owner[npt[0]:npt[1]], minlength=parts)
    grain = -(-(npt[1] - npt[0]) // (npt[-1] - npt[-2]))  # finest cells under one coarsest cell
    assert counts.max() - counts.min() <= 2 * grain, counts
    seen = np.zeros(N, np.int64)
    for lp in lps:
        seen[lp.nodes[lp.owned]] += 1
        # scales are contiguous and node_ptr agrees with scale_of
        lnp = lp.graph.node_ptr.numpy()
        for s in range(len(npt) - 1):
            assert np.all(lp.scale_of[lnp[s]:lnp[s + 1]] == s)
            assert np.all((lp.nodes[lnp[s]:lnp[s + 1]] >= npt[s]) & (lp.nodes[lnp[s]:lnp[s + 1]] < npt[s + 1]))
        # in-edges of owned nodes: all of them, in reference order
        ge = g.edge_index.numpy()
        le = lp.nodes[lp.graph.edge_index.numpy()]
        want = np.isin(ge[1], lp.nodes[lp.owned])
        assert np.array_equal(le, ge[:, want])
    assert np.all(seen == 1)
    # exchange lists agree pairwise (counts and global ids)
    for p in range(parts):
        for s, peers in xp[p].items():
            for q, (recv, send) in peers.items():
                back_recv, back_send = xp[q][s][p]
                assert np.array_equal(lps[p].nodes[recv], lps[q].nodes[back_send])
                assert np.array_equal(lps[p].nodes[send], lps[q].nodes[back_recv])
                assert np.all(owner[lps[p].nodes[recv]] == q) and np.all(lps[q].owned[back_send])
    # 4 hops of message passing with a loopback exchange == the undivided mesh
    rng = np.random.default_rng(0)
    x = rng.standard_normal((N, 3))
    ref = _hops_global(g, x.copy(), 4)
    xls = [x[lp.nodes].copy() for lp in lps]

    def loopback(p):
        def ex(xl):
            for s, peers in xp[p].items():
                for q, (recv, _) in peers.items():
                    if len(recv):
                        xl[recv] = xls[q][xp[q][s][p][1]]
        return ex
    for h in range(4):  # lockstep, as msw_group_rollout runs the parts
        for p, lp in enumerate(lps):
            loopback(p)(xls[p])
        for p, lp in enumerate(lps):
            xls[p] = _hops_part(lp, xls[p], lambda xl: None, 1)
    out = P.assemble(lps, [torch.from_numpy(a) for a in xls], N).numpy()
    assert np.isfinite(out).all()
    np.testing.assert_allclose(out, ref, rtol=1e-12, atol=1e-12)


def _exchange_worker(rank, world, port, q):
    import torch.distributed as dist
    from mswegnn import partition as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = make_multiscale_mesh(**mesh_config("small"), T=4)
        owner, lps, xp = P.decompose(g, world)
        N = g.num_nodes
        x = np.random.default_rng(0).standard_normal((N, 3))
        lp = lps[rank]

        def ex(xl):  # the RCCL exchange's pattern: per scale, grouped send/recv per peer
            for s in sorted(xp[rank]):
                reqs, bufs = [], []
                for q in sorted(xp[rank][s]):
                    recv, send = xp[rank][s][q]
                    if len(send):
                        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(xl[send])), q))
                    if len(recv):
                        b = torch.empty(len(recv), xl.shape[1], dtype=torch.float64)
                        reqs.append(dist.irecv(b, q))
                        bufs.append((recv, b))
                for r in reqs:
                    r.wait()
                for recv, b in bufs:
                    xl[recv] = b.numpy()
        out = _hops_part(lp, x[lp.nodes].copy(), ex, 4)
        # DistributedRollout.gather_owned: one padded tensor all-gather of the owned rows
        full = P.gather_parts(lps, rank, torch.from_numpy(out), N).numpy()
        q.put((rank, float(np.abs(full - _hops_global(g, x.copy(), 4)).max())))
    finally:
        dist.destroy_process_group()


def test_partition_halo_exchange_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    errs = sorted(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert [r for r, _ in errs] == [0, 1]
    assert all(e <= 1e-12 for _, e in errs), errs


def test_pmc_summary_attribution(tmp_path):
    """tools/pmc_summary.py (the `traffic` figures bench.py reports): gfx950 FETCH_SIZE
    correction (x2), per-launch averages, and the selection of the roofline kernels -- the
    middle hop moving the most bytes, and only the finest-scale dispatches of the grid-stride
    edge MLP (its launches of every scale share one grid)."""
    import csv
    import json
    import subprocess
    cols = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"]

    def write(d, counter, rows):
        d.mkdir()
        with open(d / "run_counter_collection.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=cols)
            w.writeheader()
            for i, (name, grid, val) in enumerate(rows):
                w.writerow(dict(Dispatch_Id=i, Kernel_Name=name, Grid_Size=grid, Counter_Name=counter,
                                Counter_Value=val))
    eh = "void msw::k_edge_hop<2, 1, true, 0>(msw::EdgeHopArgs)"
    mid = "void msw::k_hop<2, 1, false, true>(msw::HopArgs)"
    small = "void msw::k_hop<2, 1, false, false>(msw::HopArgs)"
    fetch = [(eh, 262144, 1000.0), (eh, 262144, 250.0), (eh, 262144, 1000.0), (mid, 262144, 400.0),
             (small, 2048, 10.0), (small, 2048, 10.0), (small, 2048, 10.0)]
    write_rows = [(n, g, v / 2) for n, g, v in fetch]
    write(tmp_path / "f", "FETCH_SIZE", fetch)
    write(tmp_path / "w", "WRITE_SIZE", write_rows)
    out = tmp_path / "s.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(out),
                    str(tmp_path / "f"), str(tmp_path / "w")], check=True, capture_output=True)
    s = json.load(open(out))
    big = s["k_edge_hop_large"]
    assert big["dispatches"] == 2  # the 250-KB (coarser-scale) launch is left out
    assert big["read_bytes_per_launch"] == 2 * 1024 * 1000.0
    assert big["write_bytes_per_launch"] == 1024 * 500.0
    assert s["k_hop_large"]["kernel"].startswith("k_hop<2, 1, false, true>")
    assert s["k_hop"]["kernel"].startswith("k_hop<2, 1, false, false>")  # most dispatches
    assert s["k_hop"]["hbm_bytes_per_launch"] == 2 * 1024 * 10.0 + 1024 * 5.0


def _subgroup_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from mswegnn.partition import group_root
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sub = dist.new_group([1, 2])
    if rank in (1, 2):
        box = [f"uid-from-{rank}".encode()] if dist.get_rank(sub) == 0 else [None]
        # DistributedRollout's unique-id broadcast within a group without global rank 0
        dist.broadcast_object_list(box, src=group_root(sub), group=sub)
        q.put((rank, group_root(sub), box[0]))
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_uid_broadcast_in_subgroup_gloo():
    """The partitioned rollout's unique id is broadcast from the group's rank 0, named by
    its GLOBAL rank (src=0 hangs for a group without global rank 0)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_subgroup_main, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == [(1, 1, b"uid-from-1"), (2, 1, b"uid-from-1")]


_PACK_DRIVER = r"""
#include <cstdio>
#include "tiling.h"
int main() {  // stdin: n deg_0 .. deg_{n-1}; stdout: the order
  int n;
  if (scanf("%d", &n) != 1) return 2;
  std::vector<int> d(n);
  for (int& x : d) if (scanf("%d", &x) != 1) return 2;
  for (int k : msw::pack_order(d)) printf("%d\n", k);
  return 0;
}
"""


def _greedy_tiles(deg):
    """plan.hip build_tiles: consecutive destinations, <= 16 in-edges and <= 16 per tile."""
    n = a = 0
    while a < len(deg):
        b, e = a, 0
        while b < len(deg) and b - a < 16 and e + deg[b] <= 16:
            e += deg[b]
            b += 1
        n, a = n + 1, max(b, a + 1)
    return n


def test_tile_pack_order(tmp_path):
    """csrc/tiling.h pack_order (the internal order of a scale's destinations): a permutation,
    never more edge tiles than the graph order, fewer on the Zenodo-size meshes (zenodo4's
    finest scale 2,050 -> 2,046: within the 2,048 tiles one round of the finest fused edge
    MLP holds), and it terminates on a destination with more than 16 in-edges."""
    import subprocess
    src = tmp_path / "pack.cpp"
    src.write_text(_PACK_DRIVER)
    exe = tmp_path / "pack"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(PKG, "csrc"), str(src), "-o", str(exe)],
                   check=True)

    def order(deg):
        out = subprocess.run([str(exe)], input=f"{len(deg)} " + " ".join(map(str, deg)), text=True,
                             capture_output=True, timeout=60, check=True).stdout.split()
        o = [int(v) for v in out]
        assert sorted(o) == list(range(len(deg)))
        return o

    counts = {}
    for name in ("zenodo4", "tiny"):
        g = make_multiscale_mesh(**mesh_config(name), T=1)
        ei, npt, ept = g.edge_index.numpy(), g.node_ptr.numpy(), g.edge_ptr.numpy()
        for s in range(len(npt) - 1):
            deg = np.bincount(ei[1, ept[s]:ept[s + 1]] - npt[s], minlength=npt[s + 1] - npt[s]).tolist()
            o = order(deg)
            before, after = _greedy_tiles(deg), _greedy_tiles([deg[k] for k in o])
            assert after <= before
            counts[(name, s)] = (before, after)
    assert counts[("zenodo4", 0)] == (2050, 2046)
    rng = np.random.default_rng(0)
    for _ in range(20):
        deg = rng.choice([0, 1, 2, 3, 4, 5, 8, 16], size=int(rng.integers(1, 400)),
                         p=[.02, .05, .1, .6, .1, .05, .05, .03]).tolist()
        assert _greedy_tiles([deg[k] for k in order(deg)]) <= _greedy_tiles(deg) + 0
    order([3, 17, 3, 40, 2])  # over-degree destinations: still a permutation, no hang


def test_plan_cache_rebuilds_after_in_place_graph_edit(monkeypatch):
    """a plan must not survive an in-place edit of the graph tensors it was built
    from (edge_attr / edge_index feed the edge terms and the tiles).  EnginePlan is replaced
    by a recorder, so no GPU is needed; the cache logic is the real one."""
    from mswegnn import engine as E
    built = []

    class FakePlan:
        def __init__(self, model, graph, device):
            self.ea = graph.edge_attr.clone()
            self.closed = False
            built.append(self)

        def close(self):
            self.closed = True

    monkeypatch.setattr(E, "EnginePlan", FakePlan)
    g = make_multiscale_mesh(**mesh_config("tiny"), T=2)
    m = build_msgnn(4, 32, 4, state=weights("K4_F32"))
    p1 = E.plan_for(m, g)
    assert E.plan_for(m, g) is p1 and len(built) == 1           # identity hit
    g2 = g.clone()
    assert E.plan_for(m, g2) is p1 and len(built) == 1          # equal content: adopted
    g2.edge_attr.mul_(2.0)                                      # in-place edit of the held tensor
    p2 = E.plan_for(m, g2)
    assert p2 is not p1 and len(built) == 2 and torch.equal(p2.ea, g2.edge_attr)
    assert p1.closed                                            # the stale plan is dropped
    # a clone of the edited graph reuses the new plan; the original graph (unedited) gets a
    # plan of its own content, never p2
    assert E.plan_for(m, g2.clone()) is p2
    p3 = E.plan_for(m, g)
    assert p3 is not p2 and torch.equal(p3.ea, g.edge_attr)
    # weights modified in place -> new plan; the cached parameter list follows registrations
    with torch.no_grad():
        next(m.parameters()).add_(1.0)
    assert E.plan_for(m, g) is not p3
    m.extra = torch.nn.Linear(2, 2)                              # registration bumps the list
    assert len(E._params(m)) == len(list(m.parameters()))


def test_lpt_split_balances_by_size():
    import bench
    sys.path.insert(0, ROOT)
    assert bench.lpt_split([5, 5, 5, 5], 2) == [[0, 2], [1, 3]]
    assert bench.lpt_split([1, 9, 4, 6], 2) == [[0, 1], [2, 3]]
    # BASELINE config 3 at G = 20 on 8 ranks: loads within one simulation of each other
    sizes = [bench.sim_fine_nodes("config3", i) for i in range(20)]
    assert sizes[:5] == [8193, 9249, 10369, 11553, 12801]
    split = bench.lpt_split(sizes, 8)
    loads = [sum(sizes[i] for i in s) for s in split]
    assert sorted(i for s in split for i in s) == list(range(20))
    assert max(loads) - min(loads) <= max(sizes)
    rr = [sum(sizes[i] for i in range(20) if i % 8 == r) for r in range(8)]
    assert max(loads) < max(rr)  # round-robin by count was the slower split


def _strong_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    torch.set_num_threads(2)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    rec = bench.strong_scaling_section(dist, rank, world, torch.device("cpu"), "torch", [3, 1], 2, 1, 0,
                                       dist.barrier, workload="tiny_mixed")
    if rank == 0:
        q.put(rec)
    dist.barrier()
    dist.destroy_process_group()


def test_strong_scaling_section_two_ranks_gloo():
    """bench.py's N > 1 strong_scaling record (verdict r2): rank 0 runs the whole fixed set
    alone, then both ranks their LPT share with the all-gather at the end; the gathered
    rollouts equal rank 0's single-device ones; the record carries t1 / tW / speed-up and
    the collective's world size."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strong_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rec = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert rec["rccl_world"] == 2 and rec["backend"] == "gloo"
    s3, s1 = rec["sets"]
    assert s1["G"] == 1 and "skipped" in s1
    assert s3["G"] == 3 and s3["sims_per_rank"] == [1, 2] and s3["fine_nodes_per_rank"] == [1153, 1026]
    for k in ("t1_ms", "tW_ms", "speedup", "rank_ms", "fine_node_steps_per_s_1gpu", "fine_node_steps_per_s_Wgpu"):
        assert k in s3, k
    assert len(s3["rank_ms"]) == 2 and s3["tW_ms"] >= max(s3["rank_ms"]) - 1e-9
    assert s3["gathered_vs_single_gpu_max_rel"] <= 1e-5


def test_speculative_forward_replans_on_weight_change(monkeypatch):
    """models.gnn _engine_forward launches the previous call's plan before consulting the plan
    cache (the reference's step loop syncs the host every step); when the cache names another
    plan -- weights modified in place, another graph -- the forward is redone with it and the
    speculative output is dropped.  EnginePlan is a recorder (no GPU)."""
    from mswegnn import engine as E
    calls = []

    class FakePlan:
        _h = 1

        def __init__(self, model, graph, device):
            self.tag = float(len(calls))
            calls.append(("build", self.tag))

        def accepts(self, x):
            return True

        def forward(self, x):
            calls.append(("fwd", self.tag))
            return torch.full((x.shape[0], 2), self.tag)

        def close(self):
            self._h = None

    monkeypatch.setattr(E, "EnginePlan", FakePlan)
    g = make_multiscale_mesh(**mesh_config("tiny"), T=2)
    m = build_msgnn(4, 32, 4, state=weights("K4_F32"))
    y0 = m._engine_forward(g)
    y1 = m._engine_forward(g)
    assert torch.equal(y0, y1) and [c[0] for c in calls] == ["build", "fwd", "fwd"]
    with torch.no_grad():
        m.node_decoder[0].weight.mul_(1.0)  # in-place: version bump -> new plan
    y2 = m._engine_forward(g)
    assert calls[-3:] == [("fwd", 0.0), ("build", 4.0), ("fwd", 4.0)]  # speculative, rebuild, redo
    assert float(y2[0, 0]) == 4.0
    y3 = m._engine_forward(g.clone())  # same content: cache adopts it, speculation stands
    assert float(y3[0, 0]) == 4.0 and calls[-1] == ("fwd", 4.0)


def test_flip_localisation_rules():
    """conftest.flip_localisation (the config-3 mask-flip exception, verdict r2): accepts a
    divergence that is a depth-mask flip at or after the reference's own flip, rejects one
    that is not a flip or that starts earlier."""
    from conftest import flip_localisation
    N, T = 50, 7
    g = torch.Generator().manual_seed(0)
    r64 = torch.rand(N, 2, T, generator=g, dtype=torch.float64) + 0.5
    r64[7, 0, 3] = 1.00002e-4          # fp64: just above the threshold -> kept
    ref = r64.clone().float().double()
    ref[7, :, 3] = 0.0                 # fp32 reference: masked (h and v) at step 3
    ref[:, :, 5:] += 0.01              # the flip propagates
    ours = ref.clone()                 # ours flips like the reference at step 3 ...
    ref[9, 0, 4] = 1.00001e-4          # ... and a second near-threshold cell at step 4:
    ours[9, :, 4] = 0.0                # ours masks it, the reference does not
    ours[:, :, 5:] += 0.02
    t, cells = flip_localisation(ours, ref, r64)
    assert (t, cells) == (4, [9])
    ours_fp64 = r64.clone()            # ours on the fp64 side of the first flip
    ours_fp64[:, :, 5:] += 0.5
    assert flip_localisation(ours_fp64, ref, r64) == (3, [7])
    bad = ours.clone()
    bad[11, 1, 4] += 0.5               # another cell diverging without a mask flip
    with pytest.raises(AssertionError):
        flip_localisation(bad, ref, r64)
    early = ours.clone()
    early[2, 0, 1] = 0.0               # divergence before the reference's flip
    with pytest.raises(AssertionError):
        flip_localisation(early, ref, r64)
    # the velocity mask v * (h != 0) on the unmasked depth (config-3 member 0, step 44): both
    # depths 0, the fp32 velocity 0, the fp64 one 0.011
    r64v = r64.clone()
    r64v[7, :, 3] = torch.tensor([0.0, 0.011], dtype=torch.float64)
    assert flip_localisation(r64v, ref, r64v) == (3, [7])


def _extras_main(rank, world, port, q, budget):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    torch.set_num_threads(2)
    import argparse
    import json as _json
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    args = argparse.Namespace(extras_budget=budget, strong_sets="3,40", strong_steps=1, T=2,
                              no_partition_check=False, no_partition_large=False)
    t0 = time.perf_counter()
    rec = bench.run_extras(dist, rank, world, torch.device("cpu"), args, dist.barrier, "gloo", engine="torch",
                           workload="tiny_mixed", gpus=0)
    if rank == 0:
        q.put((_json.dumps(rec), time.perf_counter() - t0))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("budget", [1.0, 600.0])
def test_extras_budget_two_ranks_gloo(budget):
    """bench.py's N > 1 records after the timed region run inside ONE budget (verdict r3 item 3):
    with 1 s every section is recorded as skipped and the call returns at once; with room, the
    small strong-scaling set runs (both ranks agree on every branch), the large one (G = 40,
    est. 26 s) is skipped for budget only when it does not fit, and the RCCL sections say why
    they are absent (gloo, no GPUs).  Every section carries wall_s; the record is JSON."""
    import json as _json
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_extras_main, args=(r, 2, port, q, budget)) for r in range(2)]
    for p in procs:
        p.start()
    line, wall = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rec = _json.loads(line)
    order = [o["section"] for o in rec["extras"]["order"]]
    assert order == ["strong_G3", "zenodo4_2_parts", "ddp", "strong_G40", "hbm1m_parts"]
    sets = {e["G"]: e for e in rec["strong_scaling"]["sets"]}
    assert all("wall_s" in e for e in sets.values())
    assert "skipped" in rec["ddp_training_rccl"] and "wall_s" in rec["ddp_training_rccl"]
    assert "skipped" in rec["partitioned_rollout_rccl"]["zenodo4_2_parts"]
    if budget < 2:
        assert all(e.get("skipped") == "budget" for e in sets.values())
        assert wall < 30
    else:
        assert "t1_ms" in sets[3] and "speedup" in sets[3] and sets[3]["gathered_vs_single_gpu_max_rel"] <= 1e-5
        assert "skipped" not in sets[40] or sets[40]["skipped"] == "budget"


def test_roofline_roles_match_kernel_kinds(tmp_path):
    """tools/roofline_check.py maps bench.py's timing runs (>= 20 back-to-back launches of one
    kernel in the rocprofv3 trace) to roles by kernel KIND, in bench.py's order: a role the
    run does not time (the pooling launch, fused away) is absent instead of shifting the
    large-mesh roles onto the wrong kernels (round-4 fix)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import roofline_check as rc
    seq = [("void msw::k_hop<2, 1, false, false>(msw::HopArgs)", 25, 5),
           ("void msw::k_edge_hop<2, 1, false, 0>(msw::EdgeHopArgs)", 25, 12),
           ("void at::native::vectorized_gather_kernel<16, long>(char*)", 30, 4),
           ("void msw::k_hop_rows<2>(msw::HopArgs)", 21, 144),
           ("void msw::k_edge_hop<2, 1, true, 0>(msw::EdgeHopArgs)", 20, 630)]
    path = tmp_path / "trace.csv"
    t = 0
    with open(path, "w") as f:
        f.write("Kernel_Name,Grid_Size,Start_Timestamp,End_Timestamp\n")
        for name, n, dur in seq:
            for _ in range(n):
                f.write(f"\"{name}\",1024,{t},{t + dur * 1000}\n")
                t += dur * 1000 + 500
    roles = rc.roles_of(rc.runs_of(str(path)))
    assert sorted(roles) == ["edge_hop", "edge_hop_large", "hop", "hop_large"]
    assert roles["hop"]["kernel"].startswith("k_hop<") and roles["edge_hop"]["kernel"].startswith("k_edge_hop<2, 1, false")
    assert roles["hop_large"]["kernel"] == "k_hop_rows<2>" and abs(roles["hop_large"]["avg_duration_us"] - 144) < 1e-9
    assert roles["edge_hop_large"]["kernel"].startswith("k_edge_hop<2, 1, true")


def test_step_breakdown_takes_the_rollout_period(tmp_path):
    """tools/step_breakdown.py finds the rollout step as the most common distance between
    encoder launches, not the rollout prologue's shorter one (round-4 fix: a 13-launch
    prologue was reported as the step)."""
    import subprocess
    rows = ["k_encode<2,1,true>"] + [f"k_rowmlp<{i}>" for i in range(12)]  # prologue: 13 launches
    step = ["k_encode<2,1,true>"] + [f"k_hop<{i}>" for i in range(29)]       # steps: 30 launches
    seq = rows + step * 5 + ["k_encode<2,1,true>"]
    path = tmp_path / "trace.csv"
    with open(path, "w") as f:
        f.write("Kernel_Name,Grid_Size_X,Workgroup_Size_X,Start_Timestamp,End_Timestamp\n")
        t = 0
        for n in seq:
            f.write(f"\"void msw::{n}(msw::Args)\",256,64,{t},{t + 4000}\n")
            t += 4500
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "step_breakdown.py"), str(path)],
                         capture_output=True, text=True, check=True).stdout
    assert out.splitlines()[0].endswith("steps of 30 launches"), out[:200]


def test_bench_gpus_flag_launches_ranks_without_a_launcher():
    """`python bench.py --gpus 2` with no launcher (verdict r4 item 2): bench.py starts the two
    ranks itself under torch.distributed.run before touching a GPU, and each rank sees
    WORLD_SIZE = 2 (gloo rehearsal backend; this container has no GPU, so each rank then stops
    with a clean non-zero exit naming its rank).  A launcher whose world size contradicts
    --gpus is refused, and without gloo an RCCL run on a node with too few GPUs is refused
    before any rank starts -- never a silent `n_gpus: 1` line."""
    import subprocess
    env = dict(os.environ, MSW_DIST_BACKEND="gloo", PYTHONDONTWRITEBYTECODE="1")
    env.pop("WORLD_SIZE", None)
    bench_py = os.path.join(ROOT, "bench.py")
    r = subprocess.run([sys.executable, bench_py, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and '"metric"' not in r.stdout, r.stdout
    assert "launching 2 ranks" in r.stderr
    for rank in (0, 1):
        assert f"rank {rank}/2: no GPU visible" in r.stderr, r.stderr[-2000:]
    env_w = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, bench_py, "--gpus", "8"], env=env_w, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr, r.stderr[-2000:]
    env_n = dict(env)
    env_n.pop("MSW_DIST_BACKEND")
    r = subprocess.run([sys.executable, bench_py, "--gpus", "2"], env=env_n, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 2 and "needs 2 GPUs" in r.stderr and "launching" not in r.stderr, r.stderr[-2000:]


def test_cpu_batch_baseline_one_process_per_simulation():
    """bench.cpu_batch_baseline: the batch's simulations run one per spawned
    process over the CPU share, started together behind a barrier; the rate counts every
    simulation's fine nodes x steps over the common wall time."""
    import bench
    rec = bench.cpu_batch_baseline("tiny", [0, 1], T=3, share=2, seconds=0.2, t1=0.05, t1_threads=2)
    assert rec["processes"] == 2 and rec["threads_per_process"] == 1 and rec["cores"] == 2
    assert rec["value"] > 0 and rec["unit"] == "fine-node-steps/s"
    host, share = bench.cpu_share()
    assert host == os.cpu_count() and 1 <= share <= 16
