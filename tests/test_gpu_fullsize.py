"""Parity at BASELINE.json's full sizes (configs 3, 4 and 5), HIP engine vs the reference.

* config 3: a batch of 8 Zenodo-like meshes (8,193-12,801 fine nodes, mswegnn.mesh.
  config3_members), 3-scale (seeded init) and 4-scale (K4_F32), the full 48-step batched
  rollout, every member at every step against the oracle run on that member alone;
* config 4: dk15-like mesh, the full 200-step rollout against the reference's own outputs
  (fixture, 20 stored steps spread over the horizon) and the oracle at every step;
* config 5: the ~1M-node mesh, the full 100-step rollout with teacher-forced checks: the
  HIP state entering steps 0, 25, 50 and 99 (window of its own predictions + BC) goes
  through one oracle forward, compared with the HIP prediction of that step -- a
  late-horizon divergence of any single step shows up there.
The oracle (oracle/msgnn_torch.py, bit-identical to the reference on CPU, pinned by
test_oracle_golden.py) runs on the host cores.  Workloads are built as bench.py builds them.
Tolerance: the north star's fp32 bar, max|ours - ref| / max|ref| <= 1e-4 (per step).
"""
import os
import sys

import pytest
import torch

from conftest import REL_TOL, ROOT, assert_rollout_parity, per_step_rel, rel_err
import msgnn_torch as orc

pytestmark = pytest.mark.gpu

if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _oracle_threads():
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))


def _hip(model, g, dev):
    model = model.to(dev)
    model.engine = "hip"
    return model, g.to(dev)


def _state_at(g, r, t, p=3):
    """x entering step t (t >= p) of a rollout whose predictions are r [N, 2, T]: the static
    columns, the window [pred_{t-p} .. pred_{t-1}], and the BC of step t written into the BC
    nodes (use_prediction + apply_boundary_condition, utils/dataset.py:486-529)."""
    from mswegnn.rollout import apply_boundary_condition
    x = g.x.clone()
    ns = x.shape[1] - 2 * p
    x[:, ns:] = r[:, :, t - p:t].permute(0, 2, 1).reshape(x.shape[0], 2 * p)
    x[:, ns:] = apply_boundary_condition(x[:, ns:], g.BC[:, :, t], g.node_BC, type_BC=g.type_BC)
    return x


@pytest.mark.timeout(600)
def test_config5_million_node_rollout100_teacher_forced(cuda):
    """~1M fine nodes, 3 scales, fully wet (every edge active in every hop), T = 100."""
    import bench
    T = 100
    g, m, w, desc = bench.build_workload("hbm1m", seed=0, T=T)
    assert desc["fine_nodes"] > 1_000_000 and desc["edges"] > 3_900_000
    P = {k: v.detach().clone() for k, v in m.state_dict().items()}
    cfg = orc.msgnn_config(num_scales=3, hid_features=32, K=4)
    mh, gd = _hip(m, g, cuda)
    out = mh.rollout(gd, T)
    steps = [0, 25, 50, 99]
    r = out[:, :, :].cpu()
    del out
    assert torch.isfinite(r).all()
    _oracle_threads()
    for t in steps:
        gt = g.clone()
        if t > 0:
            gt.x = _state_at(g, r, t)
        else:
            from mswegnn.rollout import apply_boundary_condition
            gt.x[:, 2:] = apply_boundary_condition(gt.x[:, 2:], g.BC[:, :, 0], g.node_BC, type_BC=g.type_BC)
        ref = orc.forward(P, cfg, gt)
        err = rel_err(r[..., t], ref)
        print(f"config 5 step {t}: rel err {err:.2e}")
        assert err <= REL_TOL, (t, err)


@pytest.mark.timeout(600)
def test_config4_dk15_rollout200_vs_reference(cuda):
    """dk15-like mesh (21,633 fine nodes, 4 scales, K4_F32 weights), the full 200 steps."""
    import bench
    from conftest import golden
    T = 200
    g, m, w, desc = bench.build_workload("dk15", seed=0, T=T)
    P = {k: v.detach().clone() for k, v in m.state_dict().items()}
    cfg = orc.msgnn_config(num_scales=4, hid_features=32, K=4)
    mh, gd = _hip(m, g, cuda)
    r = mh.rollout(gd, T).cpu()
    fx = golden("fx_dk15_K4_F32_rollout200")
    err_fx = per_step_rel(r[..., fx["steps"]], torch.from_numpy(fx["rollout_sel"]))
    assert err_fx <= REL_TOL, err_fx
    _oracle_threads()
    ref = orc.rollout(P, cfg, g, T)
    err = per_step_rel(r, ref)
    print(f"dk15 T=200: rel err vs reference fixture {err_fx:.2e}, vs oracle (all steps) {err:.2e}")
    assert err <= REL_TOL, err


@pytest.mark.timeout(600)
@pytest.mark.parametrize("S", [3, 4])
def test_config3_batch_of_8_meshes_vs_oracle(cuda, S):
    """8 heterogeneous meshes as ONE disjoint-union batch (the reference's batch layout),
    48 steps; every member against the oracle run on it alone."""
    from conftest import build_msgnn, weights
    from mswegnn.batch import collate
    from mswegnn.mesh import config3_members, make_multiscale_mesh
    from mswegnn.rollout import rollout_test, split_rollout
    T = 48
    gs = [make_multiscale_mesh(**kw, T=T) for kw in config3_members(S)]
    n0 = [int(g.node_ptr[1]) for g in gs]
    assert min(n0) == 8193 and max(n0) == 12801
    P = weights("K4_F32" if S == 4 else "msgnn3_F32_seed666")
    m = build_msgnn(num_scales=S, state=P)
    cfg = orc.msgnn_config(num_scales=S, hid_features=32, K=4)
    b = collate(gs)
    mh, bd = _hip(m, b, cuda)
    parts = split_rollout(rollout_test(mh, bd).cpu(), b)
    _oracle_threads()
    worst, flips = 0.0, []
    for i, g in enumerate(gs):
        ref = orc.rollout(P, cfg, g, T)
        e, e_ref = assert_rollout_parity(parts[i], ref, P, cfg, g, T, label=f"config 3 member {i}")
        worst = max(worst, e)
        if e_ref is not None:
            flips.append(i)
    assert len(flips) <= 1, flips
    print(f"config 3 ({S} scales): worst member rel err {worst:.2e}; members with a mask-threshold "
          f"flip in the fp32 reference itself: {flips}")
