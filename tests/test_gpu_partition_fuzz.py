"""Randomised single-mesh decompositions (fixed seeds, deterministic): a random model (MSGNN
with 2-4 scales or the 1-scale GNN, F = 16/32/64, random K, MLP depth, activations, filter,
residuals, skips) on a random mesh, dry or wet, split over 2-5 parts (mswegnn/partition.py,
SURVEY §8 f2) and stepped in lockstep by msw_group_rollout with its halo exchanges, must give
the undivided rollout BIT FOR BIT (the parts run the same per-row sums in the same order), with
the group's hipGraph replay and, for every other seed, eager as well.  The undivided rollout
itself is checked against the oracle at the fp32 bar.
PART_FUZZ_SEEDS="a:b" widens the seed range (default 0:16) for a longer sweep on the box.
"""
import os

import numpy as np
import pytest
import torch

from conftest import assert_rollout_parity, state_dict_of
import msgnn_torch as orc
from test_gpu_schedule_fuzz import T, build, draw

pytestmark = pytest.mark.gpu


def _seeds():
    a, b = (int(v) for v in os.environ.get("PART_FUZZ_SEEDS", "0:16").split(":"))
    return range(a, b)


@pytest.mark.parametrize("seed", _seeds())
def test_random_decomposition_matches_undivided(cuda, seed):
    from mswegnn import _lib as L
    from mswegnn.partition import PartitionedRollout, _scales
    c = draw(seed)
    c["meshes"] = c["meshes"][:1]
    model, cfg, gs = build(c)
    g = gs[0]
    rng = np.random.default_rng(20_000 + seed)
    npt, _ = _scales(g)
    top = int(npt[-1] - npt[-2])
    parts = int(rng.integers(2, max(3, min(6, top // 2 + 1))))
    m = model().to(cuda)
    m.engine = "hip"
    gd = g.to(cuda)
    whole = m.rollout(gd, T).cpu()
    P = state_dict_of(m)
    ref = orc.rollout({k: v.cpu() for k, v in P.items()}, cfg, g, T)
    assert_rollout_parity(whole, ref, {k: v.cpu() for k, v in P.items()}, cfg, g, T, label=f"part {seed} {c}")
    pr = PartitionedRollout(m, gd, parts, cuda)
    try:
        graphed = pr.rollout(gd.x, gd.BC, gd.node_BC, gd.type_BC, T).cpu()
        assert torch.equal(graphed, whole), (parts, c)
        if seed % 2:
            L.check(L.lib().msw_set_group_graph(pr.plans[0]._h, 0))
            eager = pr.rollout(gd.x, gd.BC, gd.node_BC, gd.type_BC, T).cpu()
            assert torch.equal(eager, whole), (parts, c)
    finally:
        pr.close()
