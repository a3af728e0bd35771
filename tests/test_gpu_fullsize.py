"""Parity at BASELINE.json's full sizes (configs 4 and 5), HIP engine vs the oracle.

The oracle (oracle/msgnn_torch.py, bit-identical to the reference on CPU, pinned by
test_oracle_golden.py) runs on the host cores: one forward of the ~1M-node mesh takes
~20-30 s there, so config 5 is checked on one forward step and config 4 on a 24-step
rollout; the bench workloads are built exactly as bench.py builds them.
Tolerance: the north star's fp32 bar, max|ours - ref| / max|ref| <= 1e-4 (per step).
"""
import os
import sys

import pytest
import torch

from conftest import REL_TOL, ROOT, per_step_rel, rel_err
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


@pytest.mark.timeout(300)
def test_config5_million_node_forward_vs_oracle(cuda):
    """~1M fine nodes, 3 scales, fully wet (every edge active in every hop)."""
    import bench
    g, m, w, desc = bench.build_workload("hbm1m", seed=0, T=2)
    assert desc["fine_nodes"] > 1_000_000 and desc["edges"] > 3_900_000
    P = {k: v.detach().clone() for k, v in m.state_dict().items()}
    cfg = orc.msgnn_config(num_scales=3, hid_features=32, K=4)
    mh, gd = _hip(m, g, cuda)
    with torch.no_grad():
        y = mh(gd).cpu()
    from mswegnn.engine import plan_for
    st = plan_for(mh, gd).stats()
    assert st["forward_calls"] >= 1
    _oracle_threads()
    ref = orc.forward(P, cfg, g)
    err = rel_err(y, ref)
    assert err <= REL_TOL, err


@pytest.mark.timeout(300)
def test_config4_dk15_rollout_vs_oracle(cuda):
    """dk15-like mesh (21,633 fine nodes, 4 scales, K4_F32 weights), 24 rollout steps."""
    import bench
    T = 24
    g, m, w, desc = bench.build_workload("dk15", seed=0, T=T)
    P = {k: v.detach().clone() for k, v in m.state_dict().items()}
    cfg = orc.msgnn_config(num_scales=4, hid_features=32, K=4)
    mh, gd = _hip(m, g, cuda)
    r = mh.rollout(gd, T).cpu()
    _oracle_threads()
    ref = orc.rollout(P, cfg, g, T)
    err = per_step_rel(r, ref)
    assert err <= REL_TOL, err
