"""Host-side plan construction under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5:
"optional ASan on host code"; verdict r3 item 8).

tests/asan/host_plan_check.cpp is compiled with g++ -fsanitize=address,undefined around
mswe-gnn_amd/csrc/graph_build.h -- the code msw_plan_create / msw_plan_create_part run on the
host: internal numbering with tiling.h's pack_order, per-scale CSR by destination, edge tiles
and lane records, dense edge chunks, the row-layout CSR, pooling / unpooling records and the
fused (un)pooling slot records, and the halo exchange lists of a partitioned mesh.  The
harness checks the invariants the kernels rely on (every edge in exactly one slot, reference
edge order per destination, records pointing at the right rows, exchange lists row-for-row
consistent between ranks) on the tiny, small, config-3, batched, degree-16 and partitioned
meshes; a node with 17 in-edges must be refused with MSW_ERR_UNSUPPORTED.  No GPU.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAGIC = 0x45534143
MSW_ERR_UNSUPPORTED = -3


def _graph_arrays(g):
    """The msw_graph_desc arrays of a graph, as mswegnn.engine.describe_graph fills them."""
    N, E = int(g.x.shape[0]), int(g.edge_index.shape[1])
    if "node_ptr" in g.keys():
        npt = g.node_ptr.reshape(-1, g.node_ptr.shape[-1]) if g.node_ptr.dim() == 2 else g.node_ptr.reshape(1, -1)
        S = int(npt.shape[1]) - 1
        iei = g.intra_mesh_edge_index
        return dict(S=S, G=int(npt.shape[0]), N=N, E=E, I=int(iei.shape[1]), node_ptr=npt.reshape(-1),
                    edge_index=g.edge_index.reshape(-1), edge_ptr=g.edge_ptr.reshape(-1),
                    intra_index=iei.reshape(-1), intra_ptr=g.intra_edge_ptr.reshape(-1)[:S] if S > 1 else torch.zeros(0))
    return dict(S=1, G=1, N=N, E=E, I=0, node_ptr=torch.tensor([0, N]), edge_index=g.edge_index.reshape(-1),
                edge_ptr=torch.tensor([0, E]), intra_index=torch.zeros(0), intra_ptr=torch.zeros(0))


def _write_case(f, name, g, expect_rc=0, group=-1, rank=-1, xch=None, l2g=None):
    a = _graph_arrays(g)
    if a["S"] > 1:
        assert len(a["intra_ptr"]) == a["S"]
    ints = lambda v: np.asarray(v, np.int64).reshape(-1)  # noqa: E731
    hdr = [MAGIC, len(name)] + [ord(ch) for ch in name] + [a["S"], a["G"], a["N"], a["E"], a["I"], expect_rc, group, rank]
    f.write(ints(hdr).tobytes())
    for k in ("node_ptr", "edge_index", "edge_ptr", "intra_index", "intra_ptr"):
        f.write(ints(torch.as_tensor(a[k]).to(torch.int64).numpy()).tobytes())
    if xch is None:
        f.write(ints([-1]).tobytes())
        return
    peers, scales, rptr, rrows, sptr, srows = xch
    f.write(ints([len(peers)]).tobytes())
    for v in (peers, scales, rptr, rrows, sptr, srows, l2g):
        f.write(ints(v).tobytes())


def _star(extra):
    """A single-scale mesh with `extra` added in-edges on node 0 (degree 16 fits one tile;
    17 is refused)."""
    from mswegnn.mesh import make_single_scale_mesh
    gs = make_single_scale_mesh(n_coarse=3, refinements=2, T=2)
    ei = gs.edge_index
    have = set(ei[0, ei[1] == 0].tolist()) | {0}
    deg0 = int((ei[1] == 0).sum())
    add = [u for u in range(1, gs.x.shape[0]) if u not in have][:extra - deg0]
    gs.edge_index = torch.cat([ei, torch.tensor([add, [0] * len(add)], dtype=ei.dtype)], 1)
    gs.edge_attr = torch.cat([gs.edge_attr, torch.zeros(len(add), gs.edge_attr.shape[1])], 0)
    assert int((gs.edge_index[1] == 0).sum()) == extra
    return gs


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("asan") / "host_plan_check")
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "mswe-gnn_amd", "csrc"), os.path.join(ROOT, "tests", "asan", "host_plan_check.cpp"),
           "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def test_host_plan_construction_under_asan_ubsan(harness, tmp_path):
    from mswegnn.batch import collate
    from mswegnn.mesh import config3_members, make_multiscale_mesh, mesh_config, make_single_scale_mesh, wet_state
    from mswegnn.partition import decompose
    from mswegnn.rollout import adapt_batch_training
    path = tmp_path / "cases.bin"
    names = []
    with open(path, "wb") as f:
        for nm in ("tiny", "small", "small3"):
            _write_case(f, nm, make_multiscale_mesh(**mesh_config(nm), T=2))
            names.append(nm)
        kw = config3_members(3, count=2)[1]
        _write_case(f, "config3_member1", make_multiscale_mesh(**kw, T=2))
        names.append("config3_member1")
        batch = adapt_batch_training(collate([make_multiscale_mesh(n_coarse=2, num_scales=4, seed=1, T=2),
                                              make_multiscale_mesh(n_coarse=3, num_scales=4, seed=2, T=2)]))
        _write_case(f, "batch_of_2", batch)
        names.append("batch_of_2")
        _write_case(f, "gnn_single_scale", make_single_scale_mesh(n_coarse=3, refinements=3, T=2))
        names.append("gnn_single_scale")
        _write_case(f, "degree16", _star(16))
        names.append("degree16")
        _write_case(f, "degree17", _star(17), expect_rc=MSW_ERR_UNSUPPORTED)
        names.append("degree17")
        for W in (2, 3):
            g = wet_state(make_multiscale_mesh(**mesh_config("small"), T=2), seed=3)
            owner, lps, plan = decompose(g, W)
            for p, lp in enumerate(lps):
                peers, scales, rptr, rrows, sptr, srows = [], [], [0], [], [0], []
                for s in sorted(plan[p]):
                    for q in sorted(plan[p][s]):
                        recv, send = plan[p][s][q]
                        peers.append(q)
                        scales.append(s)
                        rrows += list(recv)
                        srows += list(send)
                        rptr.append(len(rrows))
                        sptr.append(len(srows))
                _write_case(f, f"small_part{p}of{W}", lp.graph, group=W, rank=p,
                            xch=(peers, scales, rptr, rrows, sptr, srows), l2g=lp.nodes)
                names.append(f"small_part{p}of{W}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None) if "libasan" in env.get("LD_PRELOAD", "") else None
    r = subprocess.run([harness, str(path)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    recs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    by = {x["case"]: x for x in recs if "case" in x}
    assert sorted(by) == sorted(names)
    assert by["degree17"]["rc"] == MSW_ERR_UNSUPPORTED and "16 in-edges" in by["degree17"]["error"]
    assert by["degree16"]["rc"] == 0
    # the degree-aware destination order never needs more tiles than the graph order
    for x in recs:
        if x.get("rc") == 0 and "ntiles" in x:
            assert all(a <= b for a, b in zip(x["ntiles"], x["ntiles_graph_order"])), x
    # partitions: halo rows exist and both groups' exchange lists are consistent row for row
    groups = {x["group"]: x for x in recs if "group" in x}
    assert sorted(groups) == [2, 3] and all(x["exchange"] == "consistent" for x in groups.values())
    assert all(by[f"small_part{p}of3"]["halo_rows"] > 0 for p in range(3))
    print(f"{len(by)} host plans clean under ASan + UBSan: " +
          ", ".join(f"{k} {v.get('ntiles', v.get('rc'))}" for k, v in sorted(by.items())))
