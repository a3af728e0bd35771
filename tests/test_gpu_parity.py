"""HIP engine (through the C ABI) vs the reference's outputs.

Every test here runs the gfx950 kernels via libmswegnn.so -- ``engine='hip'`` forces the
native path and the plan statistics prove it ran.  References are the golden fixtures made
by the reference itself (oracle/gen_golden.py) or, for configurations without a fixture,
the oracle (bit-identical to the reference on CPU, pinned by test_oracle_golden.py).
Tolerance: max|ours - ref| / max|ref| <= 1e-4 at every step (BASELINE.json north star).
"""
import os

import numpy as np
import pytest
import torch

from conftest import (REL_TOL, build_gnn, build_msgnn, golden, manifest, per_step_rel, rel_err,
                      state_dict_of, weights)
import msgnn_torch as orc
from mswegnn.mesh import make_multiscale_mesh, make_single_scale_mesh, wet_state, mesh_config

pytestmark = pytest.mark.gpu


def _hip(model, dev):
    model = model.to(dev)
    model.engine = "hip"
    return model


def _stats(model, g):
    from mswegnn.engine import plan_for
    return plan_for(model, g).stats()


@pytest.mark.parametrize("ck,K,F", [("K4_F32", 4, 32), ("K2_F16", 2, 16)])
def test_single_step_vs_reference(cuda, ck, K, F):
    fx = golden(f"fx_tiny_{ck}_step")
    g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), T=48), seed=1).to(cuda)
    m = _hip(build_msgnn(4, F, K, state=weights(ck)), cuda)
    with torch.no_grad():
        y = m(g)
    torch.cuda.synchronize()
    assert _stats(m, g)["forward_calls"] >= 1
    # intermediates of the reference (forward hooks) localise any mismatch
    from mswegnn.engine import plan_for
    plan = plan_for(m, g)
    xs = plan.debug_buffer("x_s", F).cpu()
    xd = plan.debug_buffer("x_d", F).cpu()
    n0 = int(g.node_ptr[1])
    assert rel_err(xs, fx["mid__static_node_encoder"]) <= REL_TOL
    assert rel_err(xd[:n0], fx["mid__dynamic_node_encoder"][:n0]) <= REL_TOL
    assert rel_err(y.cpu(), fx["y"]) <= REL_TOL, rel_err(y.cpu(), fx["y"])


def test_f64_default_width_vs_reference(cuda):
    """config.yaml's default width F = 64 on the HIP engine against the REFERENCE's own outputs
    (oracle/gen_golden_f64.py: seeded init, no shipped F = 64 checkpoint): single step on the
    wet tiny mesh, the 48-step dry-start rollout and the 8-step wet-start rollout of the small
    mesh, 1e-4 relative per step."""
    m = _hip(build_msgnn(4, 64, 4), cuda)
    fx = golden("fx_tiny_F64_step")
    g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), T=48), seed=1).to(cuda)
    with torch.no_grad():
        y = m(g)
    assert rel_err(y.cpu(), fx["y"]) <= REL_TOL, rel_err(y.cpu(), fx["y"])
    for name, g in (("fx_small_F64_rollout48", make_multiscale_mesh(**mesh_config("small"), T=48)),
                    ("fx_small_F64_wet_rollout8", wet_state(make_multiscale_mesh(**mesh_config("small"), T=8), seed=4))):
        r = m.rollout(g.to(cuda)).cpu()
        err = per_step_rel(r, torch.from_numpy(golden(name)["rollout"]))
        print(f"{name}: per-step rel {err:.2e}")
        assert err <= REL_TOL, (name, err)


def test_single_step_msgnn3_and_gnn(cuda):
    fx = golden("fx_small3_msgnn3_wet")
    g = wet_state(make_multiscale_mesh(**mesh_config("small3"), T=6), seed=3).to(cuda)
    m = _hip(build_msgnn(3, 32, 4, state=weights("msgnn3_F32_seed666")), cuda)
    with torch.no_grad():
        y = m(g)
    assert rel_err(y.cpu(), fx["y"]) <= REL_TOL
    r = m.rollout(g, 6)
    assert per_step_rel(r.cpu(), torch.from_numpy(fx["rollout"])) <= REL_TOL

    fx = golden("fx_gnn_small_rollout10")
    g = wet_state(make_single_scale_mesh(n_coarse=3, refinements=3, T=10), seed=2).to(cuda)
    m = _hip(build_gnn(state=weights("gnn_F32_seed42")), cuda)
    with torch.no_grad():
        y = m(g)
    assert rel_err(y.cpu(), fx["y"]) <= REL_TOL
    r = m.rollout(g, 10)
    assert per_step_rel(r.cpu(), torch.from_numpy(fx["rollout"])) <= REL_TOL


@pytest.mark.parametrize("ck,K,F", [("K4_F32", 4, 32), ("K2_F16", 2, 16)])
def test_rollout48_vs_reference(cuda, ck, K, F):
    fx = golden(f"fx_small_{ck}_rollout48")
    g = make_multiscale_mesh(**mesh_config("small"), T=48).to(cuda)
    m = _hip(build_msgnn(4, F, K, state=weights(ck)), cuda)
    r = m.rollout(g)
    torch.cuda.synchronize()
    ref = torch.from_numpy(fx["rollout"])
    assert per_step_rel(r.cpu(), ref) <= REL_TOL, per_step_rel(r.cpu(), ref)
    st = _stats(m, g)
    assert st["rollout_steps"] >= 48


@pytest.mark.parametrize("model", ["msgnn_K4_F32", "msgnn_K2_F16", "gnn"])
def test_row_epilogue_split_matches_fused(cuda, model, monkeypatch):
    """Last hop + row epilogue launch (engine.h EpiArgs; forced on every scale with
    MSW_EPI_SPLIT_TILES=1) == the hop's fused epilogue, bit for bit, forward and rollout,
    and against the reference fixtures."""
    def build():
        if model == "gnn":
            return _hip(build_gnn(state=weights("gnn_F32_seed42")), cuda)
        ck, K, F = {"msgnn_K4_F32": ("K4_F32", 4, 32), "msgnn_K2_F16": ("K2_F16", 2, 16)}[model]
        return _hip(build_msgnn(4, F, K, state=weights(ck)), cuda)
    if model == "gnn":
        fx = golden("fx_gnn_small_rollout10")
        g = wet_state(make_single_scale_mesh(n_coarse=3, refinements=3, T=10), seed=2).to(cuda)
        T = 10
    else:
        fx = golden(f"fx_small_{model[6:]}_rollout48")
        g = make_multiscale_mesh(**mesh_config("small"), T=48).to(cuda)
        T = 48
    base = build()
    with torch.no_grad():
        y0 = base(g).cpu()
    r0 = base.rollout(g, T).cpu()
    n0 = _stats(base, g)["kernels_per_step"]
    monkeypatch.setenv("MSW_EPI_SPLIT_TILES", "1")
    m = build()
    with torch.no_grad():
        y = m(g).cpu()
    r = m.rollout(g, T).cpu()
    assert _stats(m, g)["kernels_per_step"] > n0  # the row epilogues were scheduled
    assert torch.equal(y, y0)
    assert torch.equal(r, r0)
    assert per_step_rel(r, torch.from_numpy(fx["rollout"])) <= REL_TOL


@pytest.mark.parametrize("F", [32, 64])
def test_coop_edge_hop_matches_single_wave(cuda, monkeypatch, F):
    """Two waves per tile in the fused edge MLP + hop (k_edge_coop) and in the edge-tile
    pooling (k_pool_edge<.., 2>), on by default while the tiles leave SIMDs idle, == one wave
    per tile (MSW_COOP_WAVES=0), bit for bit, incl. the unpooling layers' projection
    epilogue; and against the reference fixture."""
    fx = golden("fx_small_K4_F32_rollout48")
    g = make_multiscale_mesh(**mesh_config("small"), T=48).to(cuda)
    if F == 64:  # seeded init (no F = 64 checkpoint), wet start so that every scale is active
        g = wet_state(make_multiscale_mesh(**mesh_config("small"), T=12), seed=5).to(cuda)
    build = lambda: _hip(build_msgnn(4, F, 4, state=weights("K4_F32") if F == 32 else None), cuda)
    m1 = build()
    with torch.no_grad():
        y1 = m1(g).cpu()
    r1 = m1.rollout(g).cpu()
    monkeypatch.setenv("MSW_COOP_WAVES", "0")
    m0 = build()
    with torch.no_grad():
        y0 = m0(g).cpu()
    r0 = m0.rollout(g).cpu()
    assert torch.equal(y1, y0)
    assert torch.equal(r1, r0)
    if F == 32:
        assert per_step_rel(r1, torch.from_numpy(fx["rollout"])) <= REL_TOL


def test_rollout_zenodo_size_vs_reference(cuda):
    fx = golden("fx_zenodo4_K4_F32_rollout48")
    g = make_multiscale_mesh(**mesh_config("zenodo4"), T=48).to(cuda)
    m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)
    r = m.rollout(g)
    sel = r[..., fx["steps"]].cpu()
    assert per_step_rel(sel, torch.from_numpy(fx["rollout_sel"])) <= REL_TOL


def test_fused_rollout_matches_step_loop_and_graph_capture(cuda):
    """Fused msw_rollout (captured hipGraphs: one 16-step graph + single-step remainder at
    T = 20) == msw_rollout without graph == the reference-style Python loop over the HIP
    forward (training/train.py semantics)."""
    from mswegnn.engine import plan_for
    from mswegnn.rollout import apply_boundary_condition, use_prediction
    T = 20
    g = make_multiscale_mesh(**mesh_config("small"), T=T).to(cuda)
    m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)
    plan = plan_for(m, g)
    plan.set_graph_capture(True)
    r1 = m.rollout(g).clone()
    assert plan.stats()["graph_captured"] == 1
    plan.set_graph_capture(False)
    r2 = m.rollout(g).clone()
    assert torch.equal(r1, r2)
    temp = g.clone()
    preds = []
    with torch.no_grad():
        for t in range(T):
            temp.x[:, -6:] = apply_boundary_condition(temp.x[:, -6:], temp.BC[:, :, t], temp.node_BC, 2)
            p = m(temp)
            temp.x = use_prediction(temp.x, p, 3)
            preds.append(p)
    r3 = torch.stack(preds, -1)
    assert torch.equal(r1, r3)


@pytest.mark.parametrize("mesh,S,F,K,ck", [("small", 4, 32, 4, "K4_F32"), ("small", 4, 16, 2, "K2_F16"),
                                           ("small3", 3, 32, 4, None)])
def test_captured_forward_matches_eager_forward(cuda, mesh, S, F, K, ck):
    """msw_forward with graph capture (x copied into the plan's slot, one graph launch, y
    copied out) == the eager forward bit for bit, over the reference's own step loop
    (training/train.py:87-95: a new x tensor every step, predictions kept across steps) and
    == the fused rollout."""
    from mswegnn.engine import plan_for
    from mswegnn.rollout import apply_boundary_condition, use_prediction
    T = 12
    g = make_multiscale_mesh(**mesh_config(mesh), T=T).to(cuda)
    m = _hip(build_msgnn(S, F, K, state=weights(ck) if ck else None), cuda)
    plan = plan_for(m, g)

    def loop(capture):
        plan.set_graph_capture(capture)
        temp = g.clone()
        preds = []
        with torch.no_grad():
            for t in range(T):
                temp.x[:, -6:] = apply_boundary_condition(temp.x[:, -6:], temp.BC[:, :, t], temp.node_BC, 2)
                p = m(temp)
                temp.x = use_prediction(temp.x, p, 3)
                preds.append(p)
        return torch.stack(preds, -1)
    eager = loop(False)
    captured = loop(True)
    assert plan_for(m, g) is plan and plan.stats()["graph_captured"] == 1
    again = loop(True)  # replays the same captured forward
    assert torch.equal(captured, eager) and torch.equal(again, eager)
    plan.set_graph_capture(True)
    assert torch.equal(m.rollout(g, T), eager)


def test_rollout_test_dropin(cuda):
    from mswegnn.rollout import rollout_test
    fx = golden("fx_small_K4_F32_rollout48")
    g = make_multiscale_mesh(**mesh_config("small"), T=48).to(cuda)
    m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)
    r = rollout_test(m, g)
    assert r.shape == (g.num_nodes, 2, 48)
    assert per_step_rel(r.cpu(), torch.from_numpy(fx["rollout"])) <= REL_TOL


def test_hid64_random_init_vs_oracle(cuda):
    """F=64 (config.yaml default hid_features, checkpoint not shipped): seeded init,
    wet state, one step and a 4-step rollout vs the oracle."""
    m = build_msgnn(4, 64, 4)
    P = state_dict_of(m)
    cfg = orc.msgnn_config(num_scales=4, hid_features=64, K=4)
    g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), T=4), seed=5)
    ref_y = orc.forward(P, cfg, g)
    ref_r = orc.rollout(P, cfg, g)
    m = _hip(m, cuda)
    gd = g.to(cuda)
    with torch.no_grad():
        y = m(gd)
    assert rel_err(y.cpu(), ref_y) <= REL_TOL
    assert per_step_rel(m.rollout(gd).cpu(), ref_r) <= REL_TOL


def test_variants_vs_oracle(cuda):
    """Less common constructor options: mlp_layers=2 / 4, K per scale, no filter matrix,
    learned_residuals='all' / False, gnn_activation='prelu', K=1 GNN with 3 layers."""
    g = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=3, T=3), seed=7)
    cases = [
        dict(mlp_layers=2, K=[2, 3, 1]),
        # F = 32, 4-layer MLPs: the fused unpooling launch's region (two edge MLPs + the
        # projection) exceeds the cooperative kernel's LDS cap -> separate (un)pooling launches
        dict(mlp_layers=4, K=3),
        dict(with_filter_matrix=False, learned_residuals="all"),
        dict(gnn_activation="prelu", learned_residuals=False, skip_connections=False),
    ]
    for kw in cases:
        m = build_msgnn(3, 32, kw.pop("K", 2), mlp_layers=kw.pop("mlp_layers", 3), **kw)
        cfg = orc.msgnn_config(num_scales=3, hid_features=32, K=m.K[:3], mlp_layers=m.mlp_layers,
                               with_filter_matrix=m.gnn_processor[0].with_filter_matrix,
                               learned_residuals=m.learned_residuals,
                               gnn_activation="prelu" if isinstance(m.gnn_activation, torch.nn.PReLU) else "tanh",
                               skip_connections=m.skip_connections)
        P = state_dict_of(m)
        ref = orc.rollout(P, cfg, g)
        m = _hip(m, cuda)
        r = m.rollout(g.to(cuda))
        assert per_step_rel(r.cpu(), ref) <= REL_TOL, kw
    gs = wet_state(make_single_scale_mesh(n_coarse=2, refinements=2, T=3), seed=8)
    m = build_gnn(hid=32, K=1, n_layers=3, mlp_layers=2)
    cfg = orc.gnn_config(hid_features=32, K=1, n_GNN_layers=3, mlp_layers=2)
    ref = orc.rollout(state_dict_of(m), cfg, gs)
    m = _hip(m, cuda)
    assert per_step_rel(m.rollout(gs.to(cuda)).cpu(), ref) <= REL_TOL


def test_max_in_degree_and_unsupported_degree(cuda):
    """Limits of the edge tiles: a node with 16 in-edges (a whole tile of
    its own) matches the oracle; 17 in-edges is refused at plan creation with an error,
    never a fault."""
    def star(extra):
        gs = wet_state(make_single_scale_mesh(n_coarse=3, refinements=2, T=3), seed=9)
        ei = gs.edge_index
        have = set(ei[0, ei[1] == 0].tolist()) | {0}
        add = [u for u in range(1, gs.x.shape[0]) if u not in have][:extra]
        new = torch.tensor([add, [0] * len(add)], dtype=ei.dtype)
        gs.edge_index = torch.cat([ei, new], 1)
        gen = torch.Generator().manual_seed(3)
        gs.edge_attr = torch.cat([gs.edge_attr, torch.rand(len(add), gs.edge_attr.shape[1], generator=gen)], 0)
        return gs
    base = int((make_single_scale_mesh(n_coarse=3, refinements=2, T=3).edge_index[1] == 0).sum())
    g16 = star(16 - base)
    assert int((g16.edge_index[1] == 0).sum()) == 16
    m = build_gnn(hid=32, K=2, n_layers=2, mlp_layers=2)
    cfg = orc.gnn_config(hid_features=32, K=2, n_GNN_layers=2, mlp_layers=2)
    ref = orc.rollout(state_dict_of(m), cfg, g16)
    mh = _hip(m, cuda)
    assert per_step_rel(mh.rollout(g16.to(cuda)).cpu(), ref) <= REL_TOL
    g17 = star(17 - base)
    m2 = _hip(build_gnn(hid=32, K=2, n_layers=2, mlp_layers=2), cuda)
    with pytest.raises(RuntimeError, match="16 in-edges"):
        with torch.no_grad():
            m2(g17.to(cuda))


def test_batched_graphs_match_individual(cuda):
    """Two simulations as one disjoint-union batch (update_batch_multiscale layout,
    training/train.py:31-65) give the same rollouts as each alone."""
    from mswegnn.batch import collate
    ga = make_multiscale_mesh(n_coarse=2, num_scales=4, seed=1, T=8)
    gb = make_multiscale_mesh(n_coarse=3, num_scales=4, seed=2, T=8)
    m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)
    ra = m.rollout(ga.to(cuda)).cpu()
    rb = m.rollout(gb.to(cuda)).cpu()
    bt = collate([ga, gb])
    from mswegnn.rollout import rollout_test
    r = rollout_test(m, bt.to(cuda)).cpu()
    na = ga.num_nodes
    assert per_step_rel(r[:na], ra) <= REL_TOL
    assert per_step_rel(r[na:], rb) <= REL_TOL


def test_edge_cases(cuda):
    """T = 0, no BC node, and a dry graph (every active-edge predicate false)."""
    g = make_multiscale_mesh(**mesh_config("tiny"), T=4).to(cuda)
    m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)
    assert m.rollout(g, 0).shape == (g.num_nodes, 2, 0)
    g2 = g.clone()
    g2.node_BC = g2.node_BC[:0]
    g2.BC = g2.BC[:0]
    cfg = manifest()["weights_K4_F32_cfg"]
    ref = orc.rollout(weights("K4_F32"), cfg, g2.to("cpu"))
    assert per_step_rel(m.rollout(g2).cpu(), ref) <= REL_TOL


def test_water_depth_boundary_condition(cuda):
    """type_BC = 1: the BC series drives the ghost cell's water-depth columns instead of the
    discharge ones (apply_boundary_condition, utils/dataset.py:486-497), vs the oracle."""
    g = make_multiscale_mesh(**mesh_config("tiny"), T=6)
    g.type_BC = torch.tensor(1, dtype=torch.int)
    g.BC = g.BC * 0.25  # a depth series of plausible size
    cfg = manifest()["weights_K4_F32_cfg"]
    ref = orc.rollout(weights("K4_F32"), cfg, g)
    m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)
    r = m.rollout(g.to(cuda)).cpu()
    assert per_step_rel(r, ref) <= REL_TOL
    assert ref.abs().max() > 0  # the depth BC wets the mesh: a non-trivial comparison


def test_rollout_metrics_kernel_vs_reference(cuda):
    """the on-device metrics kernel against the reference's own evaluation
    functions (fx_metrics.npz): losses within fp32 rounding of the reference's fp32
    means, confusion counts exact (CSI / F1 equal where defined)."""
    from mswegnn.metrics import rollout_metrics
    fx = golden("fx_metrics")
    n0 = int(fx["n0"])
    real = torch.from_numpy(golden("fx_small_K4_F32_rollout48")["rollout"])
    pred = torch.from_numpy(golden("fx_small_K2_F16_rollout48")["rollout"])
    mass = dict(area=torch.from_numpy(fx["mass_area"]), node_bc=[fx["mass_node_bc"]], bc=[fx["mass_bc"]],
                edge_bc_length=[fx["mass_edge_bc_length"]], temporal_res=float(fx["mass_temporal_res"]))
    m = rollout_metrics(pred.to(cuda), real.to(cuda), [(0, n0)], thresholds=(0.05, 0.3), mass=mass)
    # mass conservation: fp64 volume sums vs the reference's fp32 sums (1e-4 of the largest)
    assert rel_err(m["mass_loss"][0].cpu(), fx["mass_loss_pred"]) <= 1e-4, m["mass_loss"][0][:4]
    for key, ref in (("rmse", "loss_RMSE"), ("mae", "loss_MAE"), ("rmse_water", "loss_RMSE_water"),
                     ("mae_water", "loss_MAE_water")):
        assert rel_err(m[key][0].cpu(), fx[ref]) <= 1e-5, key
    for thr in (0.05, 0.3):
        for key in ("csi", "f1"):
            np.testing.assert_allclose(m[key][thr][0].cpu().numpy(), fx[f"{key}_{thr}"], rtol=1e-6, equal_nan=True)
    # two simulations in one [N, 2, T] pair (batch layout: consecutive row ranges)
    p2 = torch.cat([pred[:n0], real[:n0].flip(-1)]).to(cuda)
    r2 = torch.cat([real[:n0], pred[:n0]]).to(cuda)
    m2 = rollout_metrics(p2, r2, [(0, n0), (n0, 2 * n0)], thresholds=(0.05,))
    assert rel_err(m2["rmse"].cpu(), fx["loss_RMSE_stack"]) <= 1e-5
    np.testing.assert_allclose(m2["csi"][0.05].cpu().numpy(), fx["csi_0.05_stack"], rtol=1e-6, equal_nan=True)
    # no floating-point atomics: bit-reproducible run to run
    m3 = rollout_metrics(p2, r2, [(0, n0), (n0, 2 * n0)], thresholds=(0.05,))
    for key in ("rmse", "mae", "rmse_water", "mae_water"):
        assert torch.equal(m2[key], m3[key]), key


@pytest.mark.parametrize("parts", [2, 3])
def test_partitioned_rollout_matches_whole_mesh(cuda, parts):
    """One mesh split over `parts` plans (mswegnn/partition.py) stepped in
    lockstep with halo exchanges (msw_group_rollout) == the undivided rollout (and the
    reference fixture), owned rows assembled back to graph numbering."""
    from mswegnn.partition import PartitionedRollout
    fx = golden("fx_small_K4_F32_rollout48")
    g = make_multiscale_mesh(**mesh_config("small"), T=48).to(cuda)
    m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)
    whole = m.rollout(g).cpu()
    pr = PartitionedRollout(m, g, parts, cuda)
    r = pr.rollout(g.x, g.BC, g.node_BC, g.type_BC, 48).cpu()
    torch.cuda.synchronize()
    assert per_step_rel(r, whole) <= REL_TOL, per_step_rel(r, whole)
    assert per_step_rel(r, torch.from_numpy(fx["rollout"])) <= REL_TOL
    for pl in pr.plans:
        assert pl.stats()["rollout_steps"] >= 48
    # wet start, single-scale GNN as well
    gw = wet_state(make_multiscale_mesh(**mesh_config("small3"), T=6), seed=3).to(cuda)
    m3 = _hip(build_msgnn(3, 32, 4, state=weights("msgnn3_F32_seed666")), cuda)
    r3 = PartitionedRollout(m3, gw, parts, cuda).rollout(gw.x, gw.BC, gw.node_BC, gw.type_BC, 6).cpu()
    assert per_step_rel(r3, torch.from_numpy(golden("fx_small3_msgnn3_wet")["rollout"])) <= REL_TOL
    gs = wet_state(make_single_scale_mesh(n_coarse=3, refinements=3, T=10), seed=2).to(cuda)
    mg = _hip(build_gnn(state=weights("gnn_F32_seed42")), cuda)
    rg = PartitionedRollout(mg, gs, parts, cuda).rollout(gs.x, gs.BC, gs.node_BC, gs.type_BC, 10).cpu()
    assert per_step_rel(rg, torch.from_numpy(golden("fx_gnn_small_rollout10")["rollout"])) <= REL_TOL


@pytest.mark.parametrize("parts", [2, 4])
def test_group_rollout_graph_matches_eager(cuda, parts):
    """msw_group_rollout replays its steps as hipGraphs (every part's launches + the halo copies
    between the parts' buffers, 16 steps per graph, held by plans[0]): the same rollout bit for
    bit as the eager group (msw_set_group_graph(plans[0], 0)) and as the undivided plan, on a
    replay (a second call) too, over T = 40 (two 16-step graph launches + eight single steps)."""
    from mswegnn import _lib as L
    from mswegnn.partition import PartitionedRollout
    T = 40
    g = make_multiscale_mesh(**mesh_config("small"), T=T).to(cuda)
    m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)
    whole = m.rollout(g, T).cpu()
    pr = PartitionedRollout(m, g, parts, cuda)
    graphed = pr.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).cpu()
    again = pr.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).cpu()
    L.check(L.lib().msw_set_group_graph(pr.plans[0]._h, 0))
    eager = pr.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).cpu()
    pr.close()
    assert torch.equal(graphed, eager) and torch.equal(graphed, again)
    assert torch.equal(graphed, whole)


def test_plan_cache_same_shape_graphs_in_sequence(cuda):
    """Two meshes of the same shape but different topology / edge_attr, one after the other,
    each freshly moved to the GPU (the allocator may hand the second the first's freed
    addresses): each rollout must match the oracle on its own graph, not a stale plan."""
    P = weights("K4_F32")
    cfg = orc.msgnn_config(num_scales=4, hid_features=32, K=4)
    m = _hip(build_msgnn(4, 32, 4, state=P), cuda)
    from mswegnn.rollout import rollout_test
    for seed in (3, 4, 3):
        g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), seed=seed, T=4), seed=seed)
        gd = g.to(cuda)
        r = rollout_test(m, gd).cpu()
        del gd
        assert per_step_rel(r, orc.rollout(P, cfg, g, 4)) <= REL_TOL, seed


def test_auto_engine_falls_back_for_unsupported_models(cuda):
    """engine='auto': a model the engine does not implement runs the torch path on the GPU
    (and gives the same result as engine='torch'); engine='hip' raises instead."""
    g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), T=3), seed=1).to(cuda)
    for kw in (dict(learned_pooling=True), dict(hid=24)):
        m = build_msgnn(4, kw.pop("hid", 32), 4, **kw).to(cuda)
        with torch.no_grad():
            y = m(g)
            m.engine = "torch"
            y_t = m(g)
        assert rel_err(y, y_t) <= 1e-5  # torch's GPU index_add_ is not bit-deterministic
        m.engine = "hip"
        with pytest.raises(RuntimeError):
            with torch.no_grad():
                m(g)


def test_broadcast_bc_column(cuda):
    """BC given as [n_BC, 1, T+1] broadcasts over the previous_t slots, as the reference's
    x_d[node_BC, (type_BC-1)::2] = BC does (utils/dataset.py:496)."""
    P = weights("K4_F32")
    cfg = orc.msgnn_config(num_scales=4, hid_features=32, K=4)
    g = make_multiscale_mesh(**mesh_config("tiny"), T=6)
    g.BC = g.BC[:, 2:3, :].contiguous()
    m = _hip(build_msgnn(4, 32, 4, state=P), cuda)
    r = m.rollout(g.to(cuda), 6).cpu()
    assert per_step_rel(r, orc.rollout(P, cfg, g, 6)) <= REL_TOL
    g.BC = torch.zeros(1, 2, 7)
    with pytest.raises(ValueError):
        m.rollout(g.to(cuda), 6)


@pytest.mark.parametrize("model", ["msgnn_K4_F32", "gnn"])
def test_deferred_decoder_matches_fused_decoder(cuda, model, monkeypatch):
    """Rollout mode runs the decoder of step t in the encoder launch of step t + 1 (plus a
    final decode launch) on latency-bound meshes, in the last hops' epilogues on large ones
    (MSW_DEFER_DECODE forces either): both orders give the same rollout bit for bit, and
    the reference's."""
    outs = {}
    for dv in ("0", "1"):
        monkeypatch.setenv("MSW_DEFER_DECODE", dv)
        if model == "gnn":
            fx = golden("fx_gnn_small_rollout10")
            g = wet_state(make_single_scale_mesh(n_coarse=3, refinements=3, T=10), seed=2).to(cuda)
            m = _hip(build_gnn(state=weights("gnn_F32_seed42")), cuda)
            outs[dv] = m.rollout(g, 10).cpu()
        else:
            fx = golden("fx_small_K4_F32_rollout48")
            g = make_multiscale_mesh(**mesh_config("small"), T=48).to(cuda)
            m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)
            outs[dv] = m.rollout(g).cpu()
        assert per_step_rel(outs[dv], torch.from_numpy(fx["rollout"])) <= REL_TOL
    assert torch.equal(outs["0"], outs["1"])


@pytest.mark.parametrize("model", ["msgnn_K4_F32", "gnn"])
def test_forward_deferred_decoder_matches_fused_decoder(cuda, model, monkeypatch):
    """Forward mode (msw_forward: the reference's own step loop, gnn.py:335-348 per call) runs
    the decoder as one row-local launch after the schedule (k_decode_fwd) on latency-bound
    meshes instead of in the four last hops' epilogues (MSW_DEFER_DECODE=0): the same output
    bit for bit, and the reference's single-step output."""
    from mswegnn.engine import EnginePlan
    outs, launches = {}, {}
    for dv in ("0", "1"):
        monkeypatch.setenv("MSW_DEFER_DECODE", dv)
        if model == "gnn":
            fx = golden("fx_gnn_small_rollout10")
            g = wet_state(make_single_scale_mesh(n_coarse=3, refinements=3, T=10), seed=2).to(cuda)
            m = build_gnn(state=weights("gnn_F32_seed42")).to(cuda)
        else:
            fx = golden("fx_tiny_K4_F32_step")
            g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), T=48), seed=1).to(cuda)
            m = build_msgnn(4, 32, 4, state=weights("K4_F32")).to(cuda)
        plan = EnginePlan(m, g, cuda)
        outs[dv] = plan.forward(g.x).clone().cpu()
        outs[dv + "_again"] = plan.forward(g.x).clone().cpu()  # the captured forward graph replayed
        plan.close()
        assert rel_err(outs[dv], torch.from_numpy(fx["y"])) <= REL_TOL
    assert torch.equal(outs["0"], outs["1"])
    assert torch.equal(outs["1"], outs["1_again"])


@pytest.mark.parametrize("act", ["relu", "leakyrelu", "elu", "swish", "sigmoid", "tanh"])
def test_mlp_activations_vs_oracle(cuda, act):
    """Every make_mlp activation of activation_functions (models/models.py:149-169) other
    than the shipped PReLU: the run-time activation path of the kernels (ACT = -1), a
    3-scale MSGNN rollout against the oracle; the GNN's gnn_activation too."""
    g = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=3, T=3), seed=9)
    m = build_msgnn(3, 32, 2, mlp_activation=act)
    cfg = orc.msgnn_config(num_scales=3, hid_features=32, K=2, mlp_activation=act)
    ref = orc.rollout(state_dict_of(m), cfg, g)
    m = _hip(m, cuda)
    assert per_step_rel(m.rollout(g.to(cuda)).cpu(), ref) <= REL_TOL, act
    gs = wet_state(make_single_scale_mesh(n_coarse=2, refinements=2, T=3), seed=10)
    m = build_gnn(hid=16, K=2, n_layers=2, mlp_layers=2, mlp_activation=act, gnn_activation=act)
    cfg = orc.gnn_config(hid_features=16, K=2, n_GNN_layers=2, mlp_layers=2, mlp_activation=act,
                         gnn_activation=act)
    ref = orc.rollout(state_dict_of(m), cfg, gs)
    m = _hip(m, cuda)
    assert per_step_rel(m.rollout(gs.to(cuda)).cpu(), ref) <= REL_TOL, act


def test_upwind_mode_vs_oracle(cuda):
    """SWEGNN(upwind_mode=True) (gnn.py:365,431-432: negative hydraulic gradients clamped to
    0) on every processor -- no shipped config sets it -- against the oracle, MSGNN and GNN."""
    g = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=3, T=4), seed=11)
    m = build_msgnn(3, 32, 2)
    for p in m.gnn_processor:
        p.upwind_mode = True
    cfg = orc.msgnn_config(num_scales=3, hid_features=32, K=2, upwind_mode=True)
    ref = torch.from_numpy(golden("fx_upwind_msgnn3_K2")["rollout"])  # the reference's own
    ref_plain = orc.rollout(state_dict_of(m), orc.msgnn_config(num_scales=3, hid_features=32, K=2), g)
    assert not torch.equal(ref, ref_plain)  # the clamp changes the result on this state
    m = _hip(m, cuda)
    assert per_step_rel(m.rollout(g.to(cuda)).cpu(), ref) <= REL_TOL
    gs = wet_state(make_single_scale_mesh(n_coarse=2, refinements=2, T=4), seed=12)
    m = build_gnn(hid=32, K=2, n_layers=2, mlp_layers=2)
    for p in m.gnn_processor:
        p.upwind_mode = True
    cfg = orc.gnn_config(hid_features=32, K=2, n_GNN_layers=2, mlp_layers=2, upwind_mode=True)
    ref = orc.rollout(state_dict_of(m), cfg, gs)
    m = _hip(m, cuda)
    assert per_step_rel(m.rollout(gs.to(cuda)).cpu(), ref) <= REL_TOL


@pytest.mark.parametrize("F", [64])
def test_split_edge_mlp_matches_fused(cuda, F, monkeypatch):
    """MSW_SPLIT_EDGE_MLP=1: each processor's edge MLP over dense 16-edge chunks (k_edge_mlp,
    padding slots skipped, the last chunk partly filled) + hop 1 as a k_hop launch -- the
    default for F = 64 scales with >= 1024 edge tiles -- gives the fused kernel's forward and
    rollout bit for bit, on one mesh and on a batch of two meshes of different sizes; and the
    oracle's rollout."""
    from mswegnn.batch import collate
    from mswegnn.rollout import rollout_test
    ga = wet_state(make_multiscale_mesh(**mesh_config("small"), T=6), seed=5)
    gb = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=4, seed=2, T=6), seed=6)
    outs = {}
    for sv in ("0", "1"):
        monkeypatch.setenv("MSW_SPLIT_EDGE_MLP", sv)
        m = _hip(build_msgnn(4, F, 4), cuda)
        gd = ga.to(cuda)
        with torch.no_grad():
            y = m(gd).cpu()
        outs[sv] = (y, m.rollout(gd).cpu(), _stats(m, gd)["kernels_per_step"],
                    rollout_test(m, collate([ga, gb]).to(cuda)).cpu())
    assert outs["1"][2] > outs["0"][2]  # the split launches were scheduled
    for i in (0, 1, 3):
        assert torch.equal(outs["0"][i], outs["1"][i])
    m = build_msgnn(4, F, 4)
    ref = orc.rollout(state_dict_of(m), orc.msgnn_config(num_scales=4, hid_features=F, K=4), ga)
    assert per_step_rel(outs["1"][1], ref) <= REL_TOL
    assert per_step_rel(outs["1"][3][:ga.num_nodes], ref) <= REL_TOL


@pytest.mark.parametrize("F", [32, 64])
def test_coop_encoder_matches_single_wave(cuda, F, monkeypatch):
    """k_encode_coop (F / 16 waves per 16-row tile, every MFMA layer's output tiles split over
    them; the F = 64 default while that leaves <= 4 waves per SIMD) == k_encode (MSW_ENC_COOP=0), bit
    for bit: forward (encoders, projection 0, unpool V) and rollout (the previous step's
    decoder in the encoder launch, the final decode-only launch); and vs the oracle."""
    g = wet_state(make_multiscale_mesh(**mesh_config("small"), T=6), seed=7)
    outs = {}
    for sv in ("0", "1"):
        monkeypatch.setenv("MSW_ENC_COOP", sv)
        m = _hip(build_msgnn(4, F, 4), cuda)
        gd = g.to(cuda)
        with torch.no_grad():
            y = m(gd).cpu()
        outs[sv] = (y, m.rollout(gd).cpu())
    assert torch.equal(outs["0"][0], outs["1"][0])
    assert torch.equal(outs["0"][1], outs["1"][1])
    m = build_msgnn(4, F, 4)
    ref = orc.rollout(state_dict_of(m), orc.msgnn_config(num_scales=4, hid_features=F, K=4), g)
    assert per_step_rel(outs["1"][1], ref) <= REL_TOL


@pytest.mark.parametrize("knob", ["MSW_XCD_MAX", "MSW_TILE_PACK"])
def test_launch_layout_knobs_are_bit_identical(cuda, knob, monkeypatch):
    """XCD packing of small grids (MSW_XCD_MAX=0: all eight XCDs) and the degree-aware
    destination order (MSW_TILE_PACK=0: graph order) change where rows and workgroups go,
    never a result bit: forward, rollout and a batch of two meshes, vs the default."""
    from mswegnn.batch import collate
    from mswegnn.rollout import rollout_test
    ga = wet_state(make_multiscale_mesh(**mesh_config("small"), T=6), seed=3)
    gb = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=4, seed=4, T=6), seed=4)
    outs = {}
    for sv in ("0", None):
        if sv is None:
            monkeypatch.delenv(knob, raising=False)
        else:
            monkeypatch.setenv(knob, sv)
        m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)
        gd = ga.to(cuda)
        with torch.no_grad():
            y = m(gd).cpu()
        outs[sv] = (y, m.rollout(gd).cpu(), rollout_test(m, collate([ga, gb]).to(cuda)).cpu())
    for a, b in zip(outs["0"], outs[None]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("F", [32, 64])
def test_feature_split_hop_matches_k_hop(cuda, F, monkeypatch):
    """k_hop_split (a middle hop's features split over two waves per tile, predicate partial
    sums and aggregated messages exchanged through LDS) == k_hop (MSW_HOP_SPLIT=0), bit for
    bit: forward, rollout, a batch of two meshes; and the oracle's rollout."""
    from mswegnn.batch import collate
    from mswegnn.rollout import rollout_test
    ga = wet_state(make_multiscale_mesh(**mesh_config("small"), T=6), seed=8)
    gb = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=4, seed=9, T=6), seed=9)
    outs = {}
    for sv in ("0", "1"):
        monkeypatch.setenv("MSW_HOP_SPLIT", sv)
        m = _hip(build_msgnn(4, F, 4), cuda)
        gd = ga.to(cuda)
        with torch.no_grad():
            y = m(gd).cpu()
        outs[sv] = (y, m.rollout(gd).cpu(), rollout_test(m, collate([ga, gb]).to(cuda)).cpu())
    for a, b in zip(outs["0"], outs["1"]):
        assert torch.equal(a, b)
    m = build_msgnn(4, F, 4)
    ref = orc.rollout(state_dict_of(m), orc.msgnn_config(num_scales=4, hid_features=F, K=4), ga)
    assert per_step_rel(outs["1"][1], ref) <= REL_TOL


def test_f64_two_wave_coop_edge_hop_matches_single_wave(cuda, monkeypatch):
    """F = 64 cooperative edge MLP + hop with two waves per tile, two tiles per workgroup
    (k_edge_coop4<.., P = 2>, forced by MSW_COOP2_F64=2) == one wave per tile
    (MSW_COOP_WAVES=0), bit for bit, incl. the unpooling layers' projection epilogue and a
    dead second tile group."""
    g = wet_state(make_multiscale_mesh(**mesh_config("small"), T=6), seed=11).to(cuda)
    outs = []
    for env in ({"MSW_COOP_WAVES": "0"}, {"MSW_COOP2_F64": "2"}):
        for k in ("MSW_COOP_WAVES", "MSW_COOP2_F64"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        m = _hip(build_msgnn(4, 64, 4), cuda)
        with torch.no_grad():
            y = m(g).cpu()
        outs.append((y, m.rollout(g).cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("F", [32, 64])
def test_wide_pool_matches_default(cuda, F, monkeypatch):
    """Pooling with 2F/16 waves per tile (k_pool_edge<NT, 2NT, 2NT>: one U and one V output
    tile per rank, ranks 0..NT-1 one O tile each; MSW_POOL_WIDE=1) == F/16 waves per tile
    (MSW_POOL_WIDE=0), bit for bit: forward, rollout, a batch of two meshes; and the oracle."""
    from mswegnn.batch import collate
    from mswegnn.rollout import rollout_test
    ga = wet_state(make_multiscale_mesh(**mesh_config("small"), T=6), seed=12)
    gb = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=4, seed=13, T=6), seed=13)
    outs = {}
    for sv in ("0", "1"):
        monkeypatch.setenv("MSW_POOL_WIDE", sv)
        m = _hip(build_msgnn(4, F, 4), cuda)
        gd = ga.to(cuda)
        with torch.no_grad():
            y = m(gd).cpu()
        outs[sv] = (y, m.rollout(gd).cpu(), rollout_test(m, collate([ga, gb]).to(cuda)).cpu())
    for a, b in zip(outs["0"], outs["1"]):
        assert torch.equal(a, b)
    m = build_msgnn(4, F, 4)
    ref = orc.rollout(state_dict_of(m), orc.msgnn_config(num_scales=4, hid_features=F, K=4), ga)
    assert per_step_rel(outs["1"][1], ref) <= REL_TOL


@pytest.mark.parametrize("S,F,K,ck", [(4, 32, 4, "K4_F32"), (4, 16, 2, "K2_F16"), (4, 64, 4, None), (3, 32, 4, None)])
def test_row_layout_hops_match_edge_tiles(cuda, monkeypatch, S, F, K, ck):
    """k_hop_rows (the row-layout middle hop of large meshes, forced on every scale here with
    MSW_HOP_ROWS=2) == the edge-tile k_hop bit for bit over a rollout (wet start: every
    branch of the activity predicate)."""
    from mswegnn.engine import EnginePlan
    T = 6
    g = wet_state(make_multiscale_mesh(**mesh_config("small" if S == 4 else "small3"), T=T), seed=4).to(cuda)
    m = build_msgnn(S, F, K, state=weights(ck) if ck else None).to(cuda)
    outs = []
    for v in ("0", "2"):
        monkeypatch.setenv("MSW_HOP_ROWS", v)
        plan = EnginePlan(m, g, cuda)
        outs.append(plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).clone())
        plan.close()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("S,F,K,ck", [(4, 32, 4, "K4_F32"), (3, 32, 4, None), (4, 64, 4, None)])
def test_grid_stride_edge_hops_match_one_tile_per_wave(cuda, monkeypatch, S, F, K, ck):
    """The grid-stride fused edge MLP + hop of large meshes (staged weights once per
    workgroup, the next tile's lane record prefetched; forced at any size with MSW_EH_LOOP=1)
    == the one-tile-per-wave kernels bit for bit over a wet-start rollout."""
    from mswegnn.engine import EnginePlan
    T = 6
    g = wet_state(make_multiscale_mesh(**mesh_config("small" if S == 4 else "small3"), T=T), seed=4).to(cuda)
    m = build_msgnn(S, F, K, state=weights(ck) if ck else None).to(cuda)
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("MSW_EH_LOOP", v)
        plan = EnginePlan(m, g, cuda)
        outs.append(plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).clone())
        plan.close()
    assert torch.equal(outs[0], outs[1])


def _built_variants():
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mswe-gnn_amd", "lib")
    names = sorted(f[len("libmswegnn_"):-3] for f in os.listdir(lib) if f.startswith("libmswegnn_") and
                   f.endswith(".so")) if os.path.isdir(lib) else []
    return [n for n in names if n != "trace"] or ["none-built"]


@pytest.mark.parametrize("variant", _built_variants())
def test_build_variant_matches_default_bitwise(variant):
    """A library build variant (build_engine.py --variant=<name>, loaded with MSW_LIB_VARIANT:
    workgroup sizes, wave counts, how the MLP operands are addressed -- speed knobs) == the
    default library bit for bit: a 3-step rollout of the dk15-size mesh with the grid-stride
    edge hops forced (MSW_EH_LOOP=1, ~4.3 k finest tiles), one of zenodo4 at F = 64 and a
    2-step rollout of config 5's 1.3 M-node mesh (the grid-stride encoder without the deferred
    decoder, the row-layout hops), one child process per library (a process loads one).  Round 4 ran it on the
    software-pipelined edge hop (ehpipe8, profiles/r04/ab_eh_pipe_hbm1m.txt, rejected).
    Skipped when no variant is built."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "mswe-gnn_amd", "lib", f"libmswegnn_{variant}.so")):
        pytest.skip(f"build variant {variant} not built")
    for args in (["--mesh", "dk15", "--T", "3", "--eh-loop"], ["--mesh", "zenodo4", "--T", "3", "--hid", "64"],
                 ["--mesh", "hbm1m", "--T", "2"]):
        res = []
        for v in ("", variant):
            env = {k: x for k, x in os.environ.items() if not k.startswith("MSW_")}
            if v:
                env["MSW_LIB_VARIANT"] = v
            r = subprocess.run([sys.executable, os.path.join(root, "tools", "rollout_digest.py")] + args,
                               capture_output=True, text=True, env=env, timeout=240)
            assert r.returncode == 0, r.stderr[-3000:]
            res.append(json.loads(r.stdout.strip().splitlines()[-1]))
        print(res)
        assert res[0]["sha256"] == res[1]["sha256"], res


@pytest.mark.parametrize("variant", ["coop2_direct"])
def test_f64_kernel_variants_match_default(cuda, monkeypatch, variant):
    """F = 64 kernel variants == the default bit for bit over a wet-start rollout (forced on the
    small mesh): the two-wave cooperative edge hop reading its MLP region from the blob
    (MSW_COOP2_DIRECT=2) against the LDS-staged one."""
    from mswegnn.engine import EnginePlan
    T = 6
    g = wet_state(make_multiscale_mesh(**mesh_config("small"), T=T), seed=4).to(cuda)
    m = build_msgnn(4, 64, 4).to(cuda)
    base = {"coop2_direct": {"MSW_COOP2_F64": "2"}}[variant]
    knob = {"coop2_direct": "MSW_COOP2_DIRECT"}[variant]
    for k, v in base.items():
        monkeypatch.setenv(k, v)
    outs = []
    for v in ("0", "2"):
        monkeypatch.setenv(knob, v)
        plan = EnginePlan(m, g, cuda)
        outs.append(plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).clone())
        plan.close()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("mode", ["fused", "stepped"])
def test_ingested_dataset_vs_reference(cuda, mode):
    """§8 f4 ingest: the reference's own dataset pipeline (get_scalers -> create_data_attr ->
    to_temporal_dataset, config.yaml settings; oracle/gen_golden_ingest.py) prepared
    simulations in its pickled-dataset layout; the HIP engine's rollout of those arrays -- each
    sample and the 2-graph batch, through rollout_test (fused) or the reference's step loop
    (one graph-replayed msw_forward per step) -- matches the reference's rollouts."""
    from conftest import ingest_samples
    from mswegnn.batch import collate
    from mswegnn.rollout import (adapt_batch_training, apply_boundary_condition, rollout_test, split_rollout,
                                 use_prediction)
    samples, rb = ingest_samples()
    m = _hip(build_msgnn(4, 32, 4, state=weights("K4_F32")), cuda)

    def run(graph):
        if mode == "fused":
            return rollout_test(m, graph)
        temp = adapt_batch_training(graph).clone() if hasattr(graph, "num_graphs") else graph.clone()
        preds = []
        with torch.no_grad():
            for t in range(graph.y.shape[-1]):
                temp.x[:, -6:] = apply_boundary_condition(temp.x[:, -6:], temp.BC[:, :, t], temp.node_BC,
                                                          type_BC=temp.type_BC)
                p = m(temp)
                temp.x = use_prediction(temp.x, p, 3)
                preds.append(p)
        return torch.stack(preds, -1)
    for g, T, ref in samples:
        r = run(g.to(cuda)).cpu()
        assert per_step_rel(r, ref) <= REL_TOL, per_step_rel(r, ref)
    b = collate([g for g, _, _ in samples])
    r = run(b.to(cuda)).cpu()
    for p, q in zip(split_rollout(r, b), split_rollout(rb, b)):
        assert per_step_rel(p, q) <= REL_TOL


def _reparent(g, level=0, moves=2):
    """A coarse node of `level` with more than kPoolInline (4) children: `moves` children of
    the second coarse node are re-assigned to the first (intra edges stay coarse-major), so
    the pooling's overflow path (children beyond the inline record) runs."""
    ie = g.intra_mesh_edge_index.clone()
    a, b = int(g.intra_edge_ptr[level]), int(g.intra_edge_ptr[level + 1])
    co = ie[0, a:b]
    first = int(co[0])
    second = int(co[co != first][0])
    idx = (co == second).nonzero().flatten()[:moves] + a
    ie[0, idx] = first
    seg = ie[:, a:b]
    order = torch.argsort(seg[0] * (int(seg[1].max()) + 1) + seg[1])
    ie[:, a:b] = seg[:, order]
    g.intra_mesh_edge_index = ie
    return g


@pytest.mark.parametrize("F,act,coop2", [(32, "prelu", None), (32, "relu", None), (64, "prelu", None),
                                         (64, "relu", "2")])
def test_fused_pooling_matches_pooling_launch(cuda, monkeypatch, F, act, coop2):
    """Mean pooling + projection fused into the coarse scale's first edge-MLP + hop launch
    (k_edge_coop<.., POOL> at F = 32, k_edge_coop4<.., POOL> at F = 64 -- four waves per
    tile, or two with MSW_COOP2_F64=2; MSW_POOL_FUSE=1, the default on small coarse scales)
    == the separate pooling launch (MSW_POOL_FUSE=0), bit for bit: forward, rollout, a batch
    of two meshes, on a mesh with a 6-child coarse node (the overflow path); 3 fewer launches
    per step on 4 scales; and the oracle on that mesh."""
    if coop2:
        monkeypatch.setenv("MSW_COOP2_F64", coop2)
    from mswegnn.batch import collate
    from mswegnn.rollout import rollout_test
    ga = _reparent(wet_state(make_multiscale_mesh(**mesh_config("small"), T=6), seed=21))
    gb = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=4, seed=22, T=6), seed=22)
    outs, kps = {}, {}
    for sv in ("0", "1"):
        monkeypatch.setenv("MSW_POOL_FUSE", sv)
        m = _hip(build_msgnn(4, F, 4, mlp_activation=act), cuda)
        gd = ga.to(cuda)
        with torch.no_grad():
            y = m(gd).cpu()
        kps[sv] = _stats(m, gd)["kernels_per_step"]
        outs[sv] = (y, m.rollout(gd).cpu(), rollout_test(m, collate([ga, gb]).to(cuda)).cpu())
    assert kps["1"] == kps["0"] - 3, kps
    for a, b in zip(outs["0"], outs["1"]):
        assert torch.equal(a, b)
    m = build_msgnn(4, F, 4, mlp_activation=act)
    ref = orc.rollout(state_dict_of(m), orc.msgnn_config(num_scales=4, hid_features=F, K=4,
                                                         mlp_activation=act), ga)
    assert per_step_rel(outs["1"][1], ref) <= REL_TOL


@pytest.mark.parametrize("F,kw", [(32, {}), (32, {"mlp_activation": "relu"}), (32, {"skip_connections": False})])
def test_fused_unpooling_matches_unpooling_launch(cuda, monkeypatch, F, kw):
    """The unpooling layer (intra-scale SWEGNN, own rows zero, + skip, + projection of the next
    processor) fused into the fine scale's first edge-MLP + hop launch (k_edge_coop<.., 2>;
    MSW_UNPOOL_FUSE=1, the default on small scales at F = 32) == the separate unpooling launch
    (MSW_UNPOOL_FUSE=0), bit for bit: forward, rollout, a batch of two meshes; fewer launches;
    and the oracle.  F = 64 keeps the unpooling launch (the fused F = 64 variant measured
    -2.5 %, profiles/r03/ab_unpool_fuse_f64.txt, and was removed)."""
    from mswegnn.batch import collate
    from mswegnn.rollout import rollout_test
    ga = _reparent(wet_state(make_multiscale_mesh(**mesh_config("small"), T=6), seed=23))
    gb = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=4, seed=24, T=6), seed=24)
    outs, kps = {}, {}
    for sv in ("0", "1"):
        monkeypatch.setenv("MSW_UNPOOL_FUSE", sv)
        m = _hip(build_msgnn(4, F, 4, **kw), cuda)
        gd = ga.to(cuda)
        with torch.no_grad():
            y = m(gd).cpu()
        kps[sv] = _stats(m, gd)["kernels_per_step"]
        outs[sv] = (y, m.rollout(gd).cpu(), rollout_test(m, collate([ga, gb]).to(cuda)).cpu())
    assert kps["1"] <= kps["0"] - 2, kps
    for a, b in zip(outs["0"], outs["1"]):
        assert torch.equal(a, b)
    m = build_msgnn(4, F, 4, **kw)
    cfg = orc.msgnn_config(num_scales=4, hid_features=F, K=4, **kw)
    assert per_step_rel(outs["1"][1], orc.rollout(state_dict_of(m), cfg, ga)) <= REL_TOL
