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
