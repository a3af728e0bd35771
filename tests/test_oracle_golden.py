"""The oracle (oracle/msgnn_torch.py) is pinned to outputs of the reference itself.

The fixtures were produced by running sdat2/mSWE-GNN's own MSGNN / GNN modules and
rollout_test on CPU (oracle/gen_golden.py); the oracle must reproduce them bit for bit
(same ATen CPU ops in the same order).  The synthetic meshes must also regenerate
identically (digest check), since fixtures store only the inputs that are not derivable.
"""
import hashlib

import numpy as np
import pytest
import torch

from conftest import golden, manifest, weights
import msgnn_torch as orc
from mswegnn.mesh import make_multiscale_mesh, make_single_scale_mesh, wet_state, mesh_config


def _digest(g):
    h = hashlib.sha256()
    for k in ("x", "edge_index", "edge_attr", "edge_ptr", "node_ptr", "intra_mesh_edge_index",
              "intra_edge_ptr", "BC", "node_BC"):
        if k in g.keys():
            h.update(np.ascontiguousarray(getattr(g, k).numpy()).tobytes())
    return np.frombuffer(bytes.fromhex(h.hexdigest()), np.uint8)


@pytest.fixture(autouse=True)
def _threads():
    torch.set_num_threads(min(8, torch.get_num_threads()))


@pytest.mark.parametrize("ck", ["K4_F32", "K2_F16"])
def test_oracle_single_step(ck):
    fx = golden(f"fx_tiny_{ck}_step")
    cfg = manifest()[f"weights_{ck}_cfg"]
    g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), T=48), seed=1)
    assert np.array_equal(_digest(g), fx["digest"]), "mesh generator drifted"
    y = orc.forward(weights(ck), cfg, g)
    assert torch.equal(y, torch.from_numpy(fx["y"]))


@pytest.mark.parametrize("ck", ["K4_F32", "K2_F16"])
def test_oracle_rollout48(ck):
    fx = golden(f"fx_small_{ck}_rollout48")
    cfg = manifest()[f"weights_{ck}_cfg"]
    g = make_multiscale_mesh(**mesh_config("small"), T=48)
    assert np.array_equal(_digest(g), fx["digest"])
    r = orc.rollout(weights(ck), cfg, g)
    assert torch.equal(r, torch.from_numpy(fx["rollout"]))


def test_oracle_msgnn3_wet():
    fx = golden("fx_small3_msgnn3_wet")
    cfg = manifest()["weights_msgnn3_F32_seed666_cfg"]
    g = wet_state(make_multiscale_mesh(**mesh_config("small3"), T=6), seed=3)
    assert np.array_equal(_digest(g), fx["digest"])
    P = weights("msgnn3_F32_seed666")
    assert torch.equal(orc.forward(P, cfg, g), torch.from_numpy(fx["y"]))
    assert torch.equal(orc.rollout(P, cfg, g), torch.from_numpy(fx["rollout"]))


def test_oracle_gnn_config1():
    fx = golden("fx_gnn_small_rollout10")
    cfg = manifest()["weights_gnn_F32_seed42_cfg"]
    g = wet_state(make_single_scale_mesh(n_coarse=3, refinements=3, T=10), seed=2)
    assert np.array_equal(_digest(g), fx["digest"])
    P = weights("gnn_F32_seed42")
    assert torch.equal(orc.forward(P, cfg, g), torch.from_numpy(fx["y"]))
    assert torch.equal(orc.rollout(P, cfg, g), torch.from_numpy(fx["rollout"]))


def test_oracle_zenodo_size_rollout():
    """Config-2-sized mesh (N0 = 10,369; 4 scales; K4_F32), 48 steps, selected steps."""
    fx = golden("fx_zenodo4_K4_F32_rollout48")
    cfg = manifest()["weights_K4_F32_cfg"]
    g = make_multiscale_mesh(**mesh_config("zenodo4"), T=48)
    assert np.array_equal(_digest(g), fx["digest"])
    r = orc.rollout(weights("K4_F32"), cfg, g)
    assert torch.equal(r[..., fx["steps"]], torch.from_numpy(fx["rollout_sel"]))
