"""Single-mesh domain decomposition: one multi-scale mesh split over W ranks.

Partitioning is nested across scales: the coarsest scale is cut into W parts (a BFS sweep
over its dual graph, cut into contiguous chunks balanced by the number of finest-scale
descendants) and every finer node follows its parent (each fine cell has exactly one
parent, train.py / dataset.py intra-mesh edges).  Consequences:
  * pooling (children -> parent) and unpooling (parent -> children) never cross ranks;
  * the only halo is the scale edges' one: the sources of the in-edges of a rank's owned
    nodes, per scale.  Those rows are refreshed before every launch that gathers from
    them: U and out_0 before a layer's first hop, out_k before every further hop.

A rank's local graph holds, per scale, its owned nodes then its halo nodes, the in-edges of
its owned nodes (reference edge order kept, so every segmented sum adds in the reference's
order), the intra-mesh edges of its owned fine nodes, and the BC nodes it holds.  Halo rows
are computed by the local engine like any other row (from incomplete neighbourhoods) and are
overwritten by the exchange before anything reads them, so owned rows come out exactly as
in the undivided rollout.
"""
from __future__ import annotations

from collections import deque

import numpy as np
import torch

from .mesh import Graph


def _scales(graph):
    if "node_ptr" in graph.keys() and graph.node_ptr.dim() == 1:
        npt = graph.node_ptr.cpu().numpy().astype(np.int64)
        ept = graph.edge_ptr.cpu().numpy().astype(np.int64)
    else:  # single-scale GNN graph
        npt = np.array([0, graph.num_nodes], np.int64)
        ept = np.array([0, graph.edge_index.shape[1]], np.int64)
    return npt, ept


def _bfs_sweep(nodes, src, dst):
    """BFS order of `nodes` over the undirected edges (src, dst), started from a peripheral
    node (the last one reached from an arbitrary start); disconnected pieces follow."""
    nodes = list(nodes)
    adj = {v: [] for v in nodes}
    for a, b in zip(src, dst):
        if a in adj and b in adj:
            adj[a].append(b)
            adj[b].append(a)

    def bfs(start, seen):
        order, q = [], deque([start])
        seen.add(start)
        while q:
            v = q.popleft()
            order.append(v)
            for u in sorted(adj[v]):
                if u not in seen:
                    seen.add(u)
                    q.append(u)
        return order

    if not nodes:
        return []
    far = bfs(nodes[0], set())[-1]
    seen, order = set(), []
    for start in [far] + nodes:
        if start not in seen:
            order += bfs(start, seen)
    return order


def partition_multiscale(graph, parts):
    """owner[node] in [0, parts) for every node of `graph` (nested across scales)."""
    npt, ept = _scales(graph)
    S = len(npt) - 1
    N = int(npt[-1])
    ei = graph.edge_index.cpu().numpy()
    parent = np.full(N, -1, np.int64)
    if S > 1:
        ii = graph.intra_mesh_edge_index.cpu().numpy()
        parent[ii[1]] = ii[0]  # (coarse, fine) pairs
    # finest-scale descendants of every node (balance weight)
    weight = np.zeros(N, np.int64)
    weight[npt[0]:npt[1]] = 1
    for s in range(S - 1):
        fine = np.arange(npt[s], npt[s + 1])
        np.add.at(weight, parent[fine][parent[fine] >= 0], weight[fine][parent[fine] >= 0])
    top = S - 1
    nodes = range(int(npt[top]), int(npt[top + 1]))
    e = ei[:, ept[top]:ept[top + 1]]
    order = _bfs_sweep(nodes, e[0].tolist(), e[1].tolist())
    owner = np.full(N, -1, np.int64)
    w = weight[order].astype(np.float64)
    cum = np.cumsum(w)
    total = cum[-1] if len(cum) else 0.0
    for v, c, wv in zip(order, cum, w):
        owner[v] = min(parts - 1, int((c - 0.5 * wv) * parts / max(total, 1.0)))
    for s in range(top - 1, -1, -1):  # finer scales follow their parent
        fine = np.arange(npt[s], npt[s + 1])
        has = parent[fine] >= 0
        owner[fine[has]] = owner[parent[fine[has]]]
        for v in fine[~has]:  # orphan (not produced by the reference's meshes): nearest owned
            owner[v] = 0
    return owner


class LocalPart:
    """Rank p's local graph + the bookkeeping to map it back and exchange its halo."""

    def __init__(self, graph, nodes, owned_mask, scale_of, halo, bc_keep):
        self.graph = graph          # Graph in local numbering (feed it to the engine)
        self.nodes = nodes          # [n_local] global id of every local row
        self.owned = owned_mask     # [n_local] bool
        self.scale_of = scale_of    # [n_local] scale of every local row
        self.halo = halo            # {scale: [local rows that are halo]}
        self.bc_keep = bc_keep      # indices into the global node_BC / BC rows held here


def local_graphs(graph, owner, parts):
    """LocalPart for every rank."""
    npt, ept = _scales(graph)
    S = len(npt) - 1
    N = int(npt[-1])
    ei = graph.edge_index.cpu().numpy()
    multiscale = S > 1 or ("node_ptr" in graph.keys())
    if S > 1:
        ii = graph.intra_mesh_edge_index.cpu().numpy()
        ipt = graph.intra_edge_ptr.cpu().numpy().astype(np.int64)
    node_bc = graph.node_BC.cpu().numpy().astype(np.int64)
    out = []
    for p in range(parts):
        nodes, scale_of, owned, halo = [], [], [], {}
        node_ptr = [0]
        edges, eattr_rows, edge_ptr = [], [], [0]
        for s in range(S):
            lo, hi = int(npt[s]), int(npt[s + 1])
            mine = np.arange(lo, hi)[owner[lo:hi] == p]
            es = ei[:, ept[s]:ept[s + 1]]
            sel = np.isin(es[1], mine)
            srcs = np.unique(es[0][sel])
            h = np.setdiff1d(srcs, mine)
            halo[s] = list(range(len(nodes) + len(mine), len(nodes) + len(mine) + len(h)))
            nodes += mine.tolist() + h.tolist()
            scale_of += [s] * (len(mine) + len(h))
            owned += [True] * len(mine) + [False] * len(h)
            node_ptr.append(len(nodes))
            idx = np.nonzero(sel)[0] + ept[s]
            edges.append(ei[:, idx])
            eattr_rows.append(idx)
            edge_ptr.append(edge_ptr[-1] + len(idx))
        nodes = np.asarray(nodes, np.int64)
        g2l = np.full(N, -1, np.int64)
        g2l[nodes] = np.arange(len(nodes))
        e_all = np.concatenate(edges, 1) if edges else np.zeros((2, 0), np.int64)
        attr_idx = np.concatenate(eattr_rows) if eattr_rows else np.zeros(0, np.int64)
        kw = dict(
            x=graph.x[torch.from_numpy(nodes)].clone(),
            edge_index=torch.from_numpy(g2l[e_all]),
            edge_attr=graph.edge_attr[torch.from_numpy(attr_idx)].clone(),
            y=graph.y[torch.from_numpy(nodes)].clone() if "y" in graph.keys() else None,
            type_BC=graph.type_BC.clone(),
        )
        bc_keep = [i for i, b in enumerate(node_bc) if g2l[b] >= 0]
        kw["node_BC"] = torch.tensor([int(g2l[node_bc[i]]) for i in bc_keep], dtype=torch.int32)
        kw["BC"] = graph.BC[bc_keep].clone() if len(bc_keep) else graph.BC[:0].clone()
        if multiscale:
            kw["node_ptr"] = torch.tensor(node_ptr, dtype=torch.int64)
            kw["edge_ptr"] = torch.tensor(edge_ptr, dtype=torch.int64)
            intra, iptr = [], [0]
            for l in range(S - 1):
                pe = ii[:, ipt[l]:ipt[l + 1]]
                keep = (owner[pe[1]] == p) & (g2l[pe[1]] >= 0) & (g2l[pe[0]] >= 0)
                intra.append(g2l[pe[:, keep]])
                iptr.append(iptr[-1] + int(keep.sum()))
            kw["intra_mesh_edge_index"] = torch.from_numpy(
                np.concatenate(intra, 1) if intra else np.zeros((2, 0), np.int64))
            kw["intra_edge_ptr"] = torch.tensor(iptr, dtype=torch.int64)
        for k in ("temporal_res", "previous_t"):
            if k in graph.keys():
                kw[k] = getattr(graph, k)
        g = Graph(**{k: v for k, v in kw.items() if v is not None})
        out.append(LocalPart(g, nodes, np.asarray(owned, bool), np.asarray(scale_of, np.int64), halo,
                             np.asarray(bc_keep, np.int64)))
    return out


def exchange_plan(parts_local, owner):
    """Per rank p and scale s: {peer q: (recv_rows, send_rows)} in local numbering.
    recv_rows: p's halo rows of scale s owned by q (ascending global id);
    send_rows: p's owned rows that q holds as halo, in q's recv order."""
    W = len(parts_local)
    g2l = []
    for lp in parts_local:
        m = {}
        for i, v in enumerate(lp.nodes.tolist()):
            m[v] = i
        g2l.append(m)
    plan = [dict() for _ in range(W)]
    for p, lp in enumerate(parts_local):
        for s, rows in lp.halo.items():
            by_peer = {}
            for r in rows:
                v = int(lp.nodes[r])
                by_peer.setdefault(int(owner[v]), []).append(r)
            for q, rr in sorted(by_peer.items()):
                send = [g2l[q][int(lp.nodes[r])] for r in rr]  # q's local rows of those nodes
                plan[p].setdefault(s, {}).setdefault(q, [None, None])[0] = rr
                plan[q].setdefault(s, {}).setdefault(p, [None, None])[1] = send
    for p in range(W):  # fill missing directions with empty lists
        for s in plan[p]:
            for q in plan[p][s]:
                a, b = plan[p][s][q]
                plan[p][s][q] = (a or [], b or [])
    return plan


def assemble(parts_local, outs, num_nodes):
    """Global [N, ...] from each rank's local output (owned rows only)."""
    o0 = outs[0]
    full = o0.new_zeros((num_nodes,) + tuple(o0.shape[1:]))
    for lp, o in zip(parts_local, outs):
        idx = torch.from_numpy(np.nonzero(lp.owned)[0]).to(o.device)
        full[torch.from_numpy(lp.nodes[lp.owned]).to(o.device)] = o[idx]
    return full


def exchange_desc(plan_p):
    """ctypes msw_exchange_desc of one rank from exchange_plan(...)[p]; returns (desc, keep)."""
    import ctypes as C

    from . import _lib as L
    peers, scales, rptr, sptr, rrows, srows = [], [], [0], [0], [], []
    for s in sorted(plan_p):
        for q in sorted(plan_p[s]):
            recv, send = plan_p[s][q]
            peers.append(q)
            scales.append(s)
            rrows += list(recv)
            srows += list(send)
            rptr.append(len(rrows))
            sptr.append(len(srows))
    keep = [np.asarray(peers, np.int32), np.asarray(scales, np.int32), np.asarray(rptr, np.int64),
            np.asarray(rrows, np.int32), np.asarray(sptr, np.int64), np.asarray(srows, np.int32)]
    d = L.MswExchangeDesc()
    d.num_entries = len(peers)
    d.peer, d.scale = (keep[0].ctypes.data_as(L.c_int32_p), keep[1].ctypes.data_as(L.c_int32_p))
    d.recv_ptr, d.recv_rows = (keep[2].ctypes.data_as(L.c_int64_p), keep[3].ctypes.data_as(L.c_int32_p))
    d.send_ptr, d.send_rows = (keep[4].ctypes.data_as(L.c_int64_p), keep[5].ctypes.data_as(L.c_int32_p))
    return d, keep


def decompose(graph, parts):
    """(owner, [LocalPart], exchange plan) of `graph` split over `parts` ranks."""
    owner = partition_multiscale(graph, parts)
    lps = local_graphs(graph, owner, parts)
    return owner, lps, exchange_plan(lps, owner)


def _bc_part(lp, BC, node_BC, device):
    nbc = torch.as_tensor(lp.graph.node_BC).to("cpu", torch.int32).reshape(-1).contiguous().numpy()
    if nbc.size == 0:
        return nbc, None, 0
    bc = torch.as_tensor(BC)[torch.from_numpy(lp.bc_keep)].to(device, torch.float32).contiguous()
    return nbc, bc, int(bc.shape[-1])


class PartitionedRollout:
    """All parts of a decomposed mesh on ONE GPU, stepped in lockstep by msw_group_rollout
    (halo exchange = device copies between the parts' plans).  Validates the decomposition
    and the exchange schedule that DistributedRollout runs over RCCL."""

    def __init__(self, model, graph, parts, device="cuda:0"):
        from .engine import EnginePlan
        self.device = torch.device(device)
        self.num_nodes = int(graph.x.shape[0])
        self.owner, self.parts, self.xplan = decompose(graph, parts)
        self.plans = []
        for p, lp in enumerate(self.parts):
            d, keep = exchange_desc(self.xplan[p])
            self.plans.append(EnginePlan(model, lp.graph, self.device, exchange=d, rank=p))
            del keep

    def rollout(self, x0, BC, node_BC, type_BC, T):
        """rollout_test of the whole mesh -> [N, 2, T] (training/train.py:67-95)."""
        import ctypes as C

        from . import _lib as L
        W, T = len(self.parts), int(T)
        x0 = x0.to(self.device, torch.float32)
        xs, outs, bcs, nbcs = [], [], [], []
        for lp in self.parts:
            xs.append(x0[torch.from_numpy(lp.nodes).to(self.device)].contiguous())
            outs.append(torch.empty(len(lp.nodes), 2, T, device=self.device))
            nbc, bc, _ = _bc_part(lp, BC, node_BC, self.device)
            nbcs.append(nbc)
            bcs.append(bc)
        vp = lambda ts: (C.c_void_p * W)(*[t.data_ptr() if t is not None else 0 for t in ts])
        nbc_p = (L.c_int32_p * W)(*[n.ctypes.data_as(L.c_int32_p) for n in nbcs])
        n_bc = (C.c_int32 * W)(*[int(n.size) for n in nbcs])
        tstr = (C.c_int32 * W)(*[int(b.shape[-1]) if b is not None else 0 for b in bcs])
        hs = (C.c_void_p * W)(*[pl._h.value for pl in self.plans])
        tb = int(torch.as_tensor(type_BC).reshape(-1)[0])
        st = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        L.check(L.lib().msw_group_rollout(hs, W, vp(xs), vp(bcs), tstr, nbc_p, n_bc, tb, T, vp(outs), st))
        return assemble(self.parts, outs, self.num_nodes)

    def close(self):
        for pl in self.plans:
            pl.close()


def group_root(group=None):
    """Global rank of `group`'s rank 0 (torch.distributed collectives take global ranks)."""
    import torch.distributed as dist
    if group is None:
        return 0
    return dist.get_global_rank(group, 0)


class DistributedRollout:
    """One part per process (torch.distributed initialised, one GPU per rank): the rank's
    plan exchanges its halo over RCCL inside msw_rollout.  rollout() returns this rank's
    local [n_local, 2, T]; gather_owned() assembles the whole mesh on every rank."""

    def __init__(self, model, graph, device=None, group=None):
        import ctypes as C
        import torch.distributed as dist

        from . import _lib as L
        from .engine import EnginePlan
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.group = group
        self.device = torch.device(device or f"cuda:{torch.cuda.current_device()}")
        self.num_nodes = int(graph.x.shape[0])
        self.owner, self.parts, self.xplan = decompose(graph, self.world)
        self.part = self.parts[self.rank]
        d, keep = exchange_desc(self.xplan[self.rank])
        self.plan = EnginePlan(model, self.part.graph, self.device, exchange=d, rank=self.rank)
        del keep
        uid = C.create_string_buffer(128)
        if self.rank == 0:
            L.check(L.lib().msw_comm_unique_id(uid))
        box = [bytes(uid.raw)]
        # src is a GLOBAL rank: the group's rank 0 (global rank 0 may not be in the group)
        dist.broadcast_object_list(box, src=group_root(group), group=group)
        L.check(L.lib().msw_plan_set_comm(self.plan._h, box[0], self.world, self.rank))

    def rollout(self, x0, BC, node_BC, type_BC, T):
        lp = self.part
        x0 = torch.as_tensor(x0)[torch.from_numpy(lp.nodes).to(torch.as_tensor(x0).device)]
        nbc = lp.graph.node_BC
        bc = torch.as_tensor(BC)[torch.from_numpy(lp.bc_keep)] if len(lp.bc_keep) else BC
        return self.plan.rollout(x0, bc, nbc, type_BC, T)

    def gather_owned(self, out_local):
        """The whole mesh's [N, ...] on every rank: ONE tensor all-gather of each rank's owned
        rows (RCCL over xGMI on an nccl group, device tensors; host tensors on gloo), padded
        to the largest part.  Every rank holds the decomposition, so no sizes are exchanged."""
        return gather_parts(self.parts, self.rank, out_local, self.num_nodes, self.group)

    def close(self):
        self.plan.close()


def gather_parts(parts, rank, out_local, num_nodes, group=None):
    """All-gather of owned rows (DistributedRollout.gather_owned): rank `rank` contributes
    out_local[owned rows of parts[rank]]; returns the assembled [num_nodes, ...]."""
    import torch.distributed as dist
    dev = out_local.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    counts = [int(lp.owned.sum()) for lp in parts]
    own_rows = torch.from_numpy(np.nonzero(parts[rank].owned)[0]).to(out_local.device)
    own = out_local.index_select(0, own_rows).to(dev)
    tail = tuple(out_local.shape[1:])
    buf = torch.zeros((max(counts),) + tail, dtype=out_local.dtype, device=dev)
    buf[:counts[rank]] = own
    slots = [torch.empty_like(buf) for _ in parts]
    dist.all_gather(slots, buf, group=group)
    full = torch.zeros((num_nodes,) + tail, dtype=out_local.dtype, device=dev)
    for q, lp in enumerate(parts):
        full[torch.from_numpy(lp.nodes[lp.owned]).to(dev)] = slots[q][:counts[q]]
    return full

