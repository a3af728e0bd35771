"""Shared test helpers.

Markers: ``gpu`` = needs an MI355X (runs the HIP engine through the C ABI).  Everything
else runs on CPU (oracle vs golden fixtures, drop-in modules, ABI loading, gloo).
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mswe-gnn_amd")
for p in (PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# fp32 parity bar of BASELINE.json's north star: max|ours - ref| / max|ref| <= 1e-4 per step
REL_TOL = 1e-4


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP engine via the C ABI)")


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def weights(name):
    return {k: torch.from_numpy(v) for k, v in golden("weights_" + name).items()}


def build_msgnn(num_scales=4, hid=32, K=4, mlp_layers=3, state=None, seed=666, **kw):
    from models.gnn import MSGNN
    args = dict(num_node_features=8, num_edge_features=1, num_scales=num_scales, hid_features=hid,
                K=K, mlp_layers=mlp_layers, seed=seed, learned_residuals=True, mlp_activation="prelu",
                gnn_activation="tanh", edge_mlp=True, normalize=True, with_filter_matrix=True,
                with_gradient=True, with_WL=True, learned_pooling=False, skip_connections=True,
                previous_t=3)
    args.update(kw)
    m = MSGNN(**args)
    if state is not None:
        m.load_state_dict(state, strict=True)
    return m.eval()


def build_gnn(hid=32, K=2, n_layers=2, mlp_layers=1, state=None, seed=42, **kw):
    from models.gnn import GNN
    args = dict(num_node_features=8, num_edge_features=1, hid_features=hid, K=K,
                n_GNN_layers=n_layers, mlp_layers=mlp_layers, previous_t=3,
                learned_residuals=True, seed=seed)
    args.update(kw)
    m = GNN(**args)
    if state is not None:
        m.load_state_dict(state, strict=True)
    return m.eval()


def state_dict_of(model):
    return {k: v.detach().clone() for k, v in model.state_dict().items()}


def rel_err(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    if b.numel() == 0:
        assert a.numel() == 0
        return 0.0
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)


def per_step_rel(ours, ref):
    """max over steps of max|ours-ref| / max|ref| at that step ([N, 2, T])."""
    worst = 0.0
    for t in range(ref.shape[-1]):
        worst = max(worst, rel_err(ours[..., t], ref[..., t]))
    return worst


@pytest.fixture(scope="session")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def graph_digest(g):
    """sha256 of a graph's input arrays (oracle/gen_golden.py graph_digest)."""
    import hashlib
    h = hashlib.sha256()
    for k in ("x", "edge_index", "edge_attr", "edge_ptr", "node_ptr", "intra_mesh_edge_index",
              "intra_edge_ptr", "BC", "node_BC"):
        if k in g.keys():
            h.update(np.ascontiguousarray(getattr(g, k).numpy()).tobytes())
    return np.frombuffer(bytes.fromhex(h.hexdigest()), np.uint8)


BATCH_FIXTURES = ["fx_batch_K4_F32", "fx_batch_msgnn3", "fx_batch_gnn"]


def batch_fixture(name):
    """-> (spec, member graphs, fixture arrays) of a batched-rollout fixture written by the
    reference's rollout_test on a PyG Batch (oracle/gen_golden.py BATCHES)."""
    from mswegnn.mesh import make_multiscale_mesh, make_single_scale_mesh, wet_state
    spec = manifest()[name + "_spec"]
    gs = []
    for m in spec["members"]:
        if spec["kind"] == "gnn":
            g = make_single_scale_mesh(n_coarse=m["n_coarse"], refinements=3, seed=m["seed"], T=spec["T"])
        else:
            g = make_multiscale_mesh(n_coarse=m["n_coarse"], num_scales=spec["S"], seed=m["seed"], T=spec["T"])
        gs.append(wet_state(g, seed=m["wet"]) if m["wet"] is not None else g)
    return spec, gs, golden(name)


def batch_model(spec):
    """-> (model, oracle weights, oracle cfg) of a batch fixture."""
    import msgnn_torch as orc
    if spec["kind"] == "gnn":
        P = weights("gnn_F32_seed42")
        return build_gnn(state=P), P, orc.gnn_config(hid_features=32, K=2, n_GNN_layers=2, mlp_layers=1)
    P = weights(spec["ckpt"] or "msgnn3_F32_seed666")
    return (build_msgnn(num_scales=spec["S"], hid=spec["F"], K=spec["K"], state=P), P,
            orc.msgnn_config(num_scales=spec["S"], hid_features=spec["F"], K=spec["K"]))


def ingest_samples():
    """The samples of fx_ingest (oracle/gen_golden_ingest.py): raw simulations in the pickled
    dataset layout, prepared by the REFERENCE's own get_scalers / create_data_attr /
    to_temporal_dataset -> [(Graph, T, reference rollout)], plus the reference's rollout of
    the 2-graph Batch."""
    from mswegnn.mesh import Graph
    fx = golden("fx_ingest")
    out = []
    for i in range(int(fx["num_samples"])):
        g = {k: torch.from_numpy(fx[f"s{i}_{k}"]) for k in ("x", "edge_index", "edge_attr", "edge_ptr", "node_ptr",
                                                             "intra_mesh_edge_index", "intra_edge_ptr", "BC",
                                                             "node_BC")}
        T = int(fx[f"s{i}_T"])
        gr = Graph(**g, type_BC=torch.tensor(int(fx[f"s{i}_type_BC"])), y=torch.zeros(g["x"].shape[0], 2, T),
                   temporal_res=torch.tensor(120), previous_t=torch.tensor(3))
        out.append((gr, T, torch.from_numpy(fx[f"s{i}_rollout"])))
    return out, torch.from_numpy(fx["batch_rollout"])


def oracle_fp64_rollout(P, cfg, g, T):
    """The oracle in float64 (weights, inputs and arithmetic): the exact-arithmetic yardstick
    for rollouts whose fp32 result is itself sensitive to rounding."""
    import msgnn_torch as orc
    P64 = {k: v.double() for k, v in P.items()}
    g64 = g.clone()
    for k in ("x", "edge_attr", "BC"):
        setattr(g64, k, getattr(g, k).double())
    return orc.rollout(P64, cfg, g64, T).float()


def assert_rollout_parity(ours, ref, P, cfg, g, T, label=""):
    """The north star's bar, 1e-4 relative per step against the fp32 reference, with one
    documented exception: a rollout the reference itself cannot resolve in fp32 -- its fp32
    result differs from exact (fp64) arithmetic by more than 1e-4, which happens when a
    cell's depth lands within rounding of the 1e-4 threshold of _mask_small_WD
    (models/models.py:79-91) and the mask flips.  There ours must be no further from the
    fp64 result than the fp32 reference is (x1.5), and the event is reported.
    Returns (error vs fp32 reference, error of the fp32 reference vs fp64 or None)."""
    e = per_step_rel(ours, ref)
    if e <= REL_TOL:
        return e, None
    r64 = oracle_fp64_rollout(P, cfg, g, T)
    e_ref = per_step_rel(ref, r64)
    e_ours = per_step_rel(ours, r64)
    print(f"{label}: rel err {e:.2e} vs the fp32 reference; fp32 reference vs fp64 {e_ref:.2e}, "
          f"ours vs fp64 {e_ours:.2e} (mask-threshold flip)")
    assert e_ref > REL_TOL, f"{label}: {e:.2e} > {REL_TOL} on a well-conditioned rollout"
    assert e_ours <= 1.5 * e_ref, f"{label}: ours {e_ours:.2e} vs fp64, reference {e_ref:.2e}"
    t, cells = flip_localisation(ours, ref, r64)
    print(f"{label}: divergence starts at step {t}, cells {cells} (the reference's own mask flip)")
    return e, e_ref


def flip_localisation(ours, ref, r64, thr=1e-4):
    """Proof that a rollout divergence from the fp32 reference comes from _mask_small_WD's
    threshold (models/models.py:79-91) and nothing else.  ours / ref / r64: [N, 2, T] (ours,
    the fp32 reference, exact fp64 arithmetic).  Asserts that
      * the fp32 reference itself leaves fp64 arithmetic (rel > REL_TOL) at some step t_ref,
        by a mask flip: at its first divergent step every cell where it differs from fp64 has
        one depth exactly 0 and the other within rounding above the 1e-4 threshold, or both
        depths 0 and one velocity exactly 0 (v * (h != 0) on the unmasked depth: ReLU gave
        exactly 0 on one side, a positive sub-threshold depth on the other);
      * ours does not leave the fp32 reference before t_ref;
      * at the first step where ours leaves the fp32 reference, every cell where they differ
        is such a flip between ours and the reference (their inputs still agree to 1e-4, so
        only the mask's discontinuity can produce it);
    returns (the step where ours leaves the reference, those cells)."""
    ours, ref, r64 = (torch.as_tensor(a).double().cpu() for a in (ours, ref, r64))
    T = ref.shape[-1]

    def first_step(a, b):
        for t in range(T):
            if rel_err(a[..., t], b[..., t]) > REL_TOL:
                return t
        return None

    def flipped_cells(a, b, t, what):
        den = b[..., t].abs().max().item()
        d = (a[..., t] - b[..., t]).abs().amax(1) > REL_TOL * den
        cells = torch.nonzero(d).flatten().tolist()
        assert cells, f"{what}: no cell diverges at step {t}"
        for n in cells:
            ha, hb = a[n, 0, t].item(), b[n, 0, t].item()
            va, vb = a[n, 1, t].item(), b[n, 1, t].item()
            lo, hi = sorted((abs(ha), abs(hb)))
            # (a) the depth mask h * (|h| > 1e-4) flipped: one depth exactly 0, the other within
            #     rounding above the threshold; (b) the velocity mask v * (h != 0) flipped on the
            #     UNMASKED depth: both depths come out 0 (ReLU gave exactly 0 on one side, a
            #     sub-threshold positive depth on the other), one velocity exactly 0
            depth_flip = lo == 0.0 and thr < hi <= thr * (1 + 1e-3)
            vel_flip = ha == 0.0 and hb == 0.0 and min(abs(va), abs(vb)) == 0.0 and max(abs(va), abs(vb)) > 0.0
            assert depth_flip or vel_flip, \
                f"{what}: cell {n} at step {t}: depths {ha!r} / {hb!r}, velocities {va!r} / {vb!r} " \
                f"are not a mask flip"
        return cells
    t_ref, t_ours = first_step(ref, r64), first_step(ours, ref)
    assert t_ref is not None, "the fp32 reference does not leave fp64 arithmetic"
    flipped_cells(ref, r64, t_ref, "fp32 reference vs fp64")
    assert t_ours is not None and t_ours >= t_ref, \
        f"ours leaves the fp32 reference at step {t_ours}, before the reference's own flip at {t_ref}"
    return t_ours, flipped_cells(ours, ref, t_ours, "ours vs fp32 reference")
