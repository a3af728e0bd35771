"""Randomised configurations (fixed seeds, deterministic): HIP engine vs the oracle.

Each case draws a model (MSGNN with 2-4 scales or the 1-scale GNN; hid_features 16/32/64;
per-scale K 1-4; mlp_layers 1-3; an mlp / gnn activation; filter matrix on/off; learned
residuals True/'all'/False; skip connections on/off) and a batch of 1-3 synthetic meshes
of random sizes, dry or wet, and compares a 3-step rollout (rollout_test semantics) with
the oracle at the fp32 bar (per step 1e-4 relative; a mask-threshold flip of the fp32
reference itself is judged against fp64, conftest.assert_rollout_parity).  The shipped
configurations are covered elsewhere; this looks for combinations no fixed test names.
FUZZ_SEEDS="a:b" widens the seed range (default 0:16) for a longer sweep on the GPU box.
"""
import os

import numpy as np
import pytest
import torch

from conftest import assert_rollout_parity, build_gnn, build_msgnn, state_dict_of
import msgnn_torch as orc
from mswegnn.batch import collate
from mswegnn.mesh import make_multiscale_mesh, make_single_scale_mesh, wet_state
from mswegnn.rollout import adapt_batch_training, rollout_test

pytestmark = pytest.mark.gpu

ACTS = ["prelu", "relu", "tanh", "elu", "swish", "leakyrelu", "sigmoid"]


def draw(seed):
    rng = np.random.default_rng(seed)
    S = int(rng.choice([1, 2, 3, 4], p=[0.2, 0.2, 0.3, 0.3]))
    F = int(rng.choice([16, 32, 64], p=[0.3, 0.5, 0.2]))
    L = int(rng.integers(1, 4))
    act = str(rng.choice(ACTS))
    gact = str(rng.choice(["tanh", "prelu", "relu"]))
    filt = bool(rng.random() < 0.8)
    res = [True, "all", False][int(rng.integers(0, 3))]
    G = int(rng.integers(1, 4))
    meshes = []
    for i in range(G):
        n = int(rng.integers(2, 4))
        wet = bool(rng.random() < 0.6)
        meshes.append((n, int(rng.integers(0, 1000)), wet))
    if S == 1:
        K = int(rng.integers(1, 4))
        nl = int(rng.integers(1, 4))
        return dict(S=1, F=F, L=L, act=act, gact=gact, filt=filt, res=res, K=K, nl=nl, meshes=meshes)
    K = [int(k) for k in rng.integers(1, 5, size=S)]
    skip = bool(rng.random() < 0.7)
    return dict(S=S, F=F, L=L, act=act, gact=gact, filt=filt, res=res, K=K, skip=skip, meshes=meshes)


def build(c):
    T = 3
    if c["S"] == 1:
        m = build_gnn(hid=c["F"], K=c["K"], n_layers=c["nl"], mlp_layers=c["L"], mlp_activation=c["act"],
                      gnn_activation=c["gact"], with_filter_matrix=c["filt"], learned_residuals=c["res"])
        cfg = orc.gnn_config(hid_features=c["F"], K=c["K"], n_GNN_layers=c["nl"], mlp_layers=c["L"],
                             mlp_activation=c["act"], gnn_activation=c["gact"], with_filter_matrix=c["filt"],
                             learned_residuals=c["res"])
        gs = [make_single_scale_mesh(n_coarse=n, refinements=2, seed=sd, T=T) for n, sd, _ in c["meshes"]]
    else:
        m = build_msgnn(c["S"], c["F"], c["K"], mlp_layers=c["L"], mlp_activation=c["act"],
                        gnn_activation=c["gact"], with_filter_matrix=c["filt"], learned_residuals=c["res"],
                        skip_connections=c["skip"])
        cfg = orc.msgnn_config(num_scales=c["S"], hid_features=c["F"], K=c["K"], mlp_layers=c["L"],
                               mlp_activation=c["act"], gnn_activation=c["gact"], with_filter_matrix=c["filt"],
                               learned_residuals=c["res"], skip_connections=c["skip"])
        gs = [make_multiscale_mesh(n_coarse=n, num_scales=c["S"], seed=sd, T=T) for n, sd, _ in c["meshes"]]
    gs = [wet_state(g, seed=sd) if wet else g for g, (_, sd, wet) in zip(gs, c["meshes"])]
    return m, cfg, gs, T


def _seeds():
    a, b = (int(v) for v in os.environ.get("FUZZ_SEEDS", "0:16").split(":"))
    return range(a, b)


@pytest.mark.parametrize("seed", _seeds())
def test_random_configuration_vs_oracle(cuda, seed):
    c = draw(seed)
    m, cfg, gs, T = build(c)
    P = state_dict_of(m)
    b = collate(gs) if len(gs) > 1 else gs[0]
    ref_graph = adapt_batch_training(b) if len(gs) > 1 else b
    ref = orc.rollout(P, cfg, ref_graph, T)
    m = m.to(cuda)
    m.engine = "hip"
    r = rollout_test(m, b.to(cuda)).cpu()
    assert r.shape == ref.shape
    assert_rollout_parity(r, ref, P, cfg, ref_graph, T, label=f"fuzz {seed} {c}")
