"""Randomised engine schedules (fixed seeds, deterministic): every MSW_* switch is documented
as flipping between bit-identical variants (plan.hip Knobs), and each switch has its own test
that flips it alone.  This draws COMBINATIONS of switches — including the size thresholds
(MSW_COOP_WAVES, MSW_EPI_SPLIT_TILES) set low or high enough to put the large-mesh kernels on
small meshes and the small-mesh kernels on larger ones — on random models (MSGNN with 2-4
scales or the 1-scale GNN, F = 16/32/64, random K, MLP depth, activations, filter, residuals,
skips) and random meshes, and requires the forward, a rollout and a batched rollout_test to be
bit-identical to the default schedule.  One case per seed also checks the default schedule
against the oracle at the fp32 bar, so a combination cannot agree with a wrong default.
SCHED_FUZZ_SEEDS="a:b" widens the seed range (default 0:24) for a longer sweep on the box.
"""
import os

import numpy as np
import pytest
import torch

from conftest import assert_rollout_parity, build_gnn, build_msgnn, state_dict_of
import msgnn_torch as orc
from mswegnn.batch import collate
from mswegnn.mesh import make_multiscale_mesh, make_single_scale_mesh, wet_state
from mswegnn.rollout import rollout_test

pytestmark = pytest.mark.gpu

# the non-default values of each engine switch (plan.hip knobs_from_env)
KNOB_VALUES = {
    "MSW_SPLIT_EDGE_MLP": ["0", "1"],
    "MSW_POOL_FUSE": ["0"],
    "MSW_UNPOOL_FUSE": ["0", "2"],
    "MSW_DEFER_DECODE": ["0", "1"],
    "MSW_HOP_ROWS": ["0", "2"],
    "MSW_COOP2_DIRECT": ["0", "2"],
    "MSW_COOP2_F64": ["0", "2"],
    "MSW_ENC_COOP": ["0", "1"],
    "MSW_EH_LOOP": ["1"],
    "MSW_HOP_SPLIT": ["0", "1"],
    "MSW_POOL_WIDE": ["0"],
    "MSW_TILE_PACK": ["0"],
    "MSW_XCD_MAX": ["0"],
    "MSW_COOP_WAVES": ["0", "64", "100000"],
    "MSW_EPI_SPLIT_TILES": ["0", "4", "100000"],
}
ACTS = ["prelu", "relu", "tanh", "elu", "swish", "leakyrelu", "sigmoid"]
T = 4


def _seeds():
    a, b = (int(v) for v in os.environ.get("SCHED_FUZZ_SEEDS", "0:24").split(":"))
    return range(a, b)


def draw(seed):
    rng = np.random.default_rng(10_000 + seed)
    S = int(rng.choice([1, 2, 3, 4], p=[0.15, 0.15, 0.3, 0.4]))
    F = int(rng.choice([16, 32, 64], p=[0.15, 0.5, 0.35]))
    c = dict(S=S, F=F, L=int(rng.integers(1, 4)), act=str(rng.choice(ACTS)),
             gact=str(rng.choice(["tanh", "prelu", "relu"])), filt=bool(rng.random() < 0.8),
             res=[True, "all", False][int(rng.integers(0, 3))])
    if S == 1:
        c.update(K=int(rng.integers(1, 4)), nl=int(rng.integers(1, 4)))
    else:
        c.update(K=[int(k) for k in rng.integers(1, 5, size=S)], skip=bool(rng.random() < 0.7))
    # two meshes: the first up to ~4.6 k finest faces (S = 4, n = 6), the second small
    c["meshes"] = [(int(rng.integers(2, 7)), int(rng.integers(0, 1000)), bool(rng.random() < 0.7)),
                   (int(rng.integers(2, 4)), int(rng.integers(0, 1000)), bool(rng.random() < 0.5))]
    names = sorted(KNOB_VALUES)
    pick = rng.choice(len(names), size=int(rng.integers(2, 7)), replace=False)
    c["knobs"] = {names[i]: str(rng.choice(KNOB_VALUES[names[i]])) for i in sorted(pick)}
    return c


def build(c):
    if c["S"] == 1:
        kw = dict(hid=c["F"], K=c["K"], n_layers=c["nl"], mlp_layers=c["L"], mlp_activation=c["act"],
                  gnn_activation=c["gact"], with_filter_matrix=c["filt"], learned_residuals=c["res"])
        model = lambda: build_gnn(**kw)  # noqa: E731
        cfg = orc.gnn_config(hid_features=c["F"], K=c["K"], n_GNN_layers=c["nl"], mlp_layers=c["L"],
                             mlp_activation=c["act"], gnn_activation=c["gact"],
                             with_filter_matrix=c["filt"], learned_residuals=c["res"])
        gs = [make_single_scale_mesh(n_coarse=n, refinements=2, seed=sd, T=T) for n, sd, _ in c["meshes"]]
    else:
        kw = dict(mlp_layers=c["L"], mlp_activation=c["act"], gnn_activation=c["gact"],
                  with_filter_matrix=c["filt"], learned_residuals=c["res"], skip_connections=c["skip"])
        model = lambda: build_msgnn(c["S"], c["F"], c["K"], **kw)  # noqa: E731
        cfg = orc.msgnn_config(num_scales=c["S"], hid_features=c["F"], K=c["K"], mlp_layers=c["L"],
                               mlp_activation=c["act"], gnn_activation=c["gact"],
                               with_filter_matrix=c["filt"], learned_residuals=c["res"],
                               skip_connections=c["skip"])
        gs = [make_multiscale_mesh(n_coarse=n, num_scales=c["S"], seed=sd, T=T) for n, sd, _ in c["meshes"]]
    gs = [wet_state(g, seed=sd) if wet else g for g, (_, sd, wet) in zip(gs, c["meshes"])]
    return model, cfg, gs


def run(model, gs, cuda):
    from mswegnn.engine import plan_for
    m = model().to(cuda)
    m.engine = "hip"
    g = gs[0].to(cuda)
    with torch.no_grad():
        y = m(g).cpu()
    out = (y, m.rollout(g).cpu(), rollout_test(m, collate(gs).to(cuda)).cpu())
    return m, out, plan_for(m, g).stats()["kernels_per_step"]


_launch_counts = []  # (default, flipped) kernels per step of every case run in this session


@pytest.mark.parametrize("seed", _seeds())
def test_random_schedule_is_bit_identical(cuda, seed, monkeypatch):
    c = draw(seed)
    model, cfg, gs = build(c)
    for k in KNOB_VALUES:
        monkeypatch.delenv(k, raising=False)
    m, base, kps = run(model, gs, cuda)
    # the default schedule against the oracle (one mesh, rollout semantics of m.rollout)
    ref = orc.rollout(state_dict_of(m.cpu()), cfg, gs[0], T)
    assert_rollout_parity(base[1], ref, state_dict_of(m.cpu()), cfg, gs[0], T, label=f"sched {seed} {c}")
    for k, v in c["knobs"].items():
        monkeypatch.setenv(k, v)
    _, flipped, kps_flipped = run(model, gs, cuda)
    _launch_counts.append((kps, kps_flipped))
    for what, a, b in zip(("forward", "rollout", "rollout_test batch"), flipped, base):
        assert a.shape == b.shape
        assert torch.equal(a, b), f"{what} differs under {c['knobs']} ({c})"


def test_drawn_schedules_change_the_launch_sequence():
    """The switches took effect: among the cases above, the launches per step differ between
    the flipped and the default schedule in a good share of them (fused / unfused pooling and
    unpooling, deferred decoder, split edge MLP, row epilogue each add or remove launches)."""
    if len(_launch_counts) < 16:
        pytest.skip("needs the random-schedule cases of this module to have run first")
    changed = sum(a != b for a, b in _launch_counts)
    assert changed >= len(_launch_counts) // 5, _launch_counts
