"""The RCCL transport executed on a one-GPU box (SURVEY §8 rows e and f2).

RCCL refuses two ranks on one device, so the multi-GPU paths are driven here through ONE-rank
communicators:
  * halo exchange: a plan of the undivided mesh whose exchange list holds SELF entries (peer ==
    rank, msw_plan_create_part) runs every exchange point of msw_rollout through the real
    transport -- pack rows, grouped ncclSend / ncclRecv to self, unpack (plan.hip
    rccl_exchange).  Identity entries (send row k = receive row k) must leave the rollout bit
    for bit as the plain plan's; shifted entries (receive row k <- send row k+1) must move rows
    exactly as the in-process transport does (msw_group_rollout, device copies, no RCCL);
  * capture: the same exchanges recorded into the rollout's hipGraphs and replayed;
  * the torch.distributed side (tests/rccl_world1.py, a fresh process with an nccl process
    group of one rank): bench.make_gatherer's all-gather, DistributedRollout's communicator
    setup (ncclGetUniqueId broadcast, ncclCommInitRank) and gather_owned.
msw_plan_stats.rccl_calls / rccl_steps prove the RCCL calls were issued and the steps ran.
The reference's multi-device behaviour is Lightning's implicit DDP (main.py:107,
test_model.py:83); the north star replaces it with sharded simulations + one all-gather.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT, build_gnn, build_msgnn, golden, per_step_rel, weights, REL_TOL
from mswegnn.mesh import make_multiscale_mesh, make_single_scale_mesh, mesh_config, wet_state

pytestmark = pytest.mark.gpu


def _model(cuda, kind="msgnn32"):
    if kind == "msgnn32":
        m = build_msgnn(4, 32, 4, state=weights("K4_F32"))
    elif kind == "msgnn64":
        m = build_msgnn(4, 64, 4)
    else:
        m = build_gnn(state=weights("gnn_F32_seed42"))
    m = m.to(cuda)
    m.engine = "hip"
    return m


def _self_plan(g, stride, shift):
    """exchange_plan-style {scale: {0: (recv, send)}}: on every scale the rows k*stride (+1 per
    scale, so that scale 0 includes a BC-free interior row) received from rank 0 itself, send
    row i = recv row (i + shift) mod n."""
    from mswegnn.partition import _scales
    npt, _ = _scales(g)
    plan = {}
    for s in range(len(npt) - 1):
        rows = np.arange(int(npt[s]) + s % stride, int(npt[s + 1]), stride, dtype=np.int64)
        if rows.size == 0:
            continue
        plan[s] = {0: (rows.tolist(), np.roll(rows, -shift).tolist())}
    return plan


def _part_plan(model, g, cuda, xplan):
    from mswegnn.engine import EnginePlan
    from mswegnn.partition import exchange_desc
    d, keep = exchange_desc(xplan)
    pl = EnginePlan(model, g, cuda, exchange=d, rank=0)
    del keep
    return pl


def _set_comm(pl):
    from mswegnn import _lib as L
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")  # one rank: the bootstrap never leaves the host
    uid = C.create_string_buffer(128)
    L.check(L.lib().msw_comm_unique_id(uid))
    L.check(L.lib().msw_plan_set_comm(pl._h, uid.raw, 1, 0))


def _group_rollout(pl, g, T):
    """msw_group_rollout of the one-plan group: the in-process transport (device row copies)."""
    from mswegnn import _lib as L
    x0 = g.x.contiguous()
    out = torch.empty(g.num_nodes, 2, T, device=x0.device)
    nbc = np.ascontiguousarray(g.node_BC.cpu().to(torch.int32).reshape(-1).numpy())
    bc = g.BC.to(torch.float32).contiguous()
    vp = lambda t: (C.c_void_p * 1)(t.data_ptr())
    st = C.c_void_p(torch.cuda.current_stream(x0.device).cuda_stream)
    L.check(L.lib().msw_group_rollout((C.c_void_p * 1)(pl._h.value), 1, vp(x0), vp(bc),
                                      (C.c_int32 * 1)(int(bc.shape[-1])),
                                      (L.c_int32_p * 1)(nbc.ctypes.data_as(L.c_int32_p)),
                                      (C.c_int32 * 1)(int(nbc.size)), int(g.type_BC.reshape(-1)[0]), T,
                                      vp(out), st))
    return out


def test_rccl_one_rank_identity_exchange_matches_plain_plan(cuda):
    """Every exchange point of a 48-step 4-scale rollout through RCCL send / recv to self
    (identity rows): bit-identical to the undivided plan and to the reference fixture's bar;
    eager first, then the exchanges captured into the rollout graphs and replayed."""
    T = 48
    g = make_multiscale_mesh(**mesh_config("small"), T=T).to(cuda)
    m = _model(cuda)
    whole = m.rollout(g, T).clone()
    pl = _part_plan(m, g, cuda, _self_plan(g, stride=3, shift=0))
    _set_comm(pl)
    st0 = pl.stats()
    assert st0["rccl_calls"] == 0 and st0["graph_captured"] == 0
    eager = pl.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).clone()
    torch.cuda.synchronize()
    st1 = pl.stats()
    # 4 scales x 7 processors: every layer's first hop exchanges U and out_0, every further hop
    # out_k; one send + one recv per buffer and step
    assert st1["rccl_steps"] == T and st1["rccl_calls"] > 0 and st1["rccl_calls"] % (2 * T) == 0, st1
    per_step = st1["rccl_calls"] // T
    assert torch.equal(eager, whole), (eager - whole).abs().max().item()
    assert per_step_rel(eager.cpu(), torch.from_numpy(golden("fx_small_K4_F32_rollout48")["rollout"])) <= REL_TOL
    # captured: 16-step graphs hold the RCCL calls, replays issue none on the host
    pl.set_graph_capture(1)
    cap = pl.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).clone()
    torch.cuda.synchronize()
    st2 = pl.stats()
    assert st2["graph_captured"] == 1 and st2["rccl_steps"] == 2 * T
    captured_calls = st2["rccl_calls"] - st1["rccl_calls"]
    assert captured_calls == 16 * per_step, (captured_calls, per_step)  # one 16-step graph, T % 16 == 0
    again = pl.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).clone()
    torch.cuda.synchronize()
    st3 = pl.stats()
    assert st3["rccl_calls"] == st2["rccl_calls"] and st3["rccl_steps"] == 3 * T
    assert torch.equal(cap, whole) and torch.equal(again, whole)
    # forward mode (the reference's per-step loop, msw_forward): the exchange points of the
    # forward schedule through RCCL, captured into the forward graph, == the plain forward
    from mswegnn.engine import plan_for
    y_plain = plan_for(m, g).forward(g.x).clone()
    calls = pl.stats()["rccl_calls"]
    y = pl.forward(g.x).clone()
    torch.cuda.synchronize()
    assert pl.stats()["rccl_calls"] > calls  # the forward graph's capture issued them
    assert torch.equal(y, y_plain), (y - y_plain).abs().max().item()
    pl.close()


def test_rccl_self_exchange_on_a_batch(cuda):
    """A batch of two meshes (the reference's disjoint-union layout, graph-major rows inside a
    scale): shifted self entries whose rows span both graphs move rows exactly as the in-process
    transport does, eager and captured."""
    from mswegnn.batch import collate
    from mswegnn.rollout import adapt_batch_training
    T = 8
    ga = wet_state(make_multiscale_mesh(**mesh_config("tiny"), seed=1, T=T), seed=1)
    gb = wet_state(make_multiscale_mesh(**mesh_config("tiny"), seed=2, T=T), seed=2)
    g = adapt_batch_training(collate([ga, gb])).to(cuda)
    m = _model(cuda)
    npt = g.node_ptr.cpu().numpy()  # [graphs][scales + 1]
    xp = {}
    for s in range(npt.shape[1] - 1):  # on every scale: rows of graph 0 and graph 1 together
        rows = np.concatenate([np.arange(npt[0, s], npt[0, s + 1], 4), np.arange(npt[1, s] + 1, npt[1, s + 1], 4)])
        xp[s] = {0: (rows.tolist(), np.roll(rows, -3).tolist())}
    from mswegnn.engine import EnginePlan
    from mswegnn.partition import exchange_desc
    d, keep = exchange_desc(xp)
    loop_pl = EnginePlan(m, g, cuda, exchange=d, rank=0)
    rccl_pl = EnginePlan(m, g, cuda, exchange=d, rank=0)
    del keep
    loop = _group_rollout(loop_pl, g, T).clone()
    _set_comm(rccl_pl)
    eager = rccl_pl.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).clone()
    rccl_pl.set_graph_capture(1)
    cap = rccl_pl.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).clone()
    torch.cuda.synchronize()
    assert rccl_pl.stats()["rccl_steps"] == 2 * T
    assert torch.equal(eager, loop) and torch.equal(cap, loop)
    loop_pl.close()
    rccl_pl.close()


@pytest.mark.parametrize("kind", ["msgnn32", "msgnn64", "gnn"])
def test_rccl_self_exchange_moves_rows_like_loopback(cuda, kind):
    """Shifted self entries (receive row k <- send row k+1): the rollout is no longer the plain
    one, and the RCCL transport (eager and captured) gives the in-process transport's result
    bit for bit -- the bytes really went through ncclSend / ncclRecv and landed in the right rows
    (4-scale MSGNN at F = 32 / 64: U rows of 2F floats and out rows of F; the 1-scale GNN)."""
    T = 20
    if kind == "gnn":
        g = wet_state(make_single_scale_mesh(n_coarse=3, refinements=3, T=T), seed=2).to(cuda)
    else:
        g = wet_state(make_multiscale_mesh(**mesh_config("small"), T=T), seed=3).to(cuda)
    m = _model(cuda, kind)
    whole = m.rollout(g, T).clone()
    xp = _self_plan(g, stride=5, shift=1)
    loop_pl = _part_plan(m, g, cuda, xp)
    loop = _group_rollout(loop_pl, g, T).clone()
    rccl_pl = _part_plan(m, g, cuda, xp)
    _set_comm(rccl_pl)
    eager = rccl_pl.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).clone()
    rccl_pl.set_graph_capture(1)
    cap = rccl_pl.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).clone()
    torch.cuda.synchronize()
    st = rccl_pl.stats()
    assert st["rccl_steps"] == 2 * T and st["rccl_calls"] > 0
    assert torch.isfinite(loop).all()
    assert not torch.equal(loop, whole)  # the exchange changed the rollout
    assert torch.equal(eager, loop), (eager - loop).abs().max().item()
    assert torch.equal(cap, loop), (cap - loop).abs().max().item()
    loop_pl.close()
    rccl_pl.close()


def test_self_exchange_entry_validation(cuda):
    """A self entry must send as many rows as it receives (RCCL pairs them); other peers are
    validated against the group as before."""
    from mswegnn import _lib as L
    g = make_multiscale_mesh(**mesh_config("tiny"), T=2).to(cuda)
    m = _model(cuda)
    bad = {0: {0: ([0, 1, 2], [3, 4])}}
    with pytest.raises(L.EngineError, match="self exchange entry"):
        _part_plan(m, g, cuda, bad)
    # no communicator: the RCCL transport refuses to run rather than skip the exchange
    pl = _part_plan(m, g, cuda, _self_plan(g, stride=4, shift=0))
    with pytest.raises(L.EngineError, match="without a transport"):
        pl.rollout(g.x, g.BC, g.node_BC, g.type_BC, 2)
    pl.close()


def test_nccl_world1_process_group(cuda):
    """A fresh process with a one-rank nccl process group (tests/rccl_world1.py): bench.py's
    end-of-rollout all-gather, DistributedRollout (uid broadcast, ncclCommInitRank through the
    engine) and its gather_owned, against the plain rollout bit for bit."""
    env = dict(os.environ, NCCL_SOCKET_IFNAME=os.environ.get("NCCL_SOCKET_IFNAME", "lo"),
               NCCL_DEBUG=os.environ.get("NCCL_DEBUG", "WARN"))
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_world1.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    sys.stderr.write(p.stderr[-4000:])
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    print(rec)
    assert rec["backend"] == "nccl" and rec["world"] == 1
    assert rec["gather_equal"] and rec["gather_second_equal"]
    assert rec["distributed_rollout_equal"] and rec["gather_owned_equal"]
    assert rec["comm_set"]


def test_rccl_partition_checker_runs_at_world1(cuda):
    """tools/rccl_partition_check.py -- the single-mesh decomposition checker bench.py runs at
    N > 1 (eager RCCL exchanges, then captured) -- end to end on the one GPU at W = 1: spawned
    rank, nccl group, DistributedRollout, gather_owned, the captured pass; both records
    bit-identical to the undivided rollout."""
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "rccl_partition_check.py"), "1",
                        "--mesh", "small", "--steps", "2", "--T", "8", "--wait", "200"],
                       env=dict(os.environ, NCCL_SOCKET_IFNAME=os.environ.get("NCCL_SOCKET_IFNAME", "lo")),
                       capture_output=True, text=True, timeout=260)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    print(rec)
    assert rec["bit_identical"] and rec["world"] == 1
    assert rec["captured"]["bit_identical_to_eager"] and rec["captured"]["graph_captured"] == 1, rec["captured"]


def test_ddp_training_step_nccl_world1(cuda):
    """tools/ddp_train_check.py over nccl at W = 1 (the DDP training check bench.py runs at
    N > 1): DistributedDataParallel's gradient all-reduce through RCCL around the HIP training
    kernels, gradients against one process's own step."""
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "ddp_train_check.py"), "1",
                        "--backend", "nccl", "--wait", "200"],
                       env=dict(os.environ, NCCL_SOCKET_IFNAME=os.environ.get("NCCL_SOCKET_IFNAME", "lo")),
                       capture_output=True, text=True, timeout=260)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    print(rec)
    assert rec["backend"] == "nccl" and rec["world"] == 1
