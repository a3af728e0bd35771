"""Synthetic multi-scale triangular flood meshes in the reference's graph layout.

The reference builds its graphs offline from D-Hydro meshes (database/graph_creation.py,
out of scope here); the Zenodo meshes are not available offline.  This
module emulates the *layout* those graphs have when they reach the hot path
(SURVEY Appendix B):

* graph nodes are mesh faces (dual graph); undirected dual edges appear in both
  directions, coalesced (sorted by (row, col)) like PyG ``to_undirected``;
* the hierarchy is a 1->4 midpoint refinement (graph_creation.py:498-518), scale 0 is the
  finest and comes first (graph_creation.py:1526-1530);
* every scale has ONE ghost cell appended after its faces with one *directed*
  ghost->BC-face dual edge appended after its dual edges (get_BC_edge_index,
  graph_creation.py:1239-1265, undirected_BC=False :1399);
* intra edges are (coarse, fine) pairs, one per fine face whose centre lies in the coarse
  face, in ``np.where`` order (connect_coarse_to_fine_mesh graph_creation.py:422-436,
  get_intra_edges :912-931);
* ``node_ptr = face_ptr``, ``edge_ptr = dual_edge_ptr`` (graph_creation.py:1542-1545);
* node features ``x = [area(std per scale), DEM(min-shifted), h,q x previous_t]``
  (dataset.py:74-131, 339-347), edge_attr = standardised face-centre distance;
* ``node_BC`` = the finest ghost cell (graph_creation.py:1577), ``BC[nBC, p, T+1]`` a
  sliding window over a hydrograph, ``type_BC = 2`` (discharge).

Deterministic for a given seed (numpy default_rng).
"""
from __future__ import annotations

import numpy as np
import torch

__all__ = ["Graph", "make_multiscale_mesh", "make_single_scale_mesh", "wet_state",
           "mesh_config", "config3_members"]


class Graph:
    """Attribute bag with the subset of the PyG ``Data`` API the hot path uses
    (``clone``, ``keys``, attribute access, ``to``)."""

    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    def keys(self):
        return list(self.__dict__.keys())

    def __contains__(self, key):
        return key in self.__dict__

    def clone(self):
        out = Graph()
        for k, v in self.__dict__.items():
            out.__dict__[k] = v.clone() if isinstance(v, torch.Tensor) else v
        return out

    def to(self, device):
        out = Graph()
        for k, v in self.__dict__.items():
            out.__dict__[k] = v.to(device) if isinstance(v, torch.Tensor) else v
        return out

    @property
    def num_nodes(self):
        return int(self.x.shape[0])


# ----------------------------------------------------------------------------- geometry
def _coarse_triangulation(n, rng, jitter=0.25, size=1000.0):
    """n x n squares, each split into two triangles, interior vertices jittered."""
    h = size / n
    ii, jj = np.meshgrid(np.arange(n + 1), np.arange(n + 1), indexing="ij")
    xy = np.stack([ii.ravel() * h, jj.ravel() * h], 1).astype(np.float64)
    interior = (ii.ravel() > 0) & (ii.ravel() < n) & (jj.ravel() > 0) & (jj.ravel() < n)
    xy[interior] += rng.uniform(-jitter, jitter, size=(interior.sum(), 2)) * h
    vid = lambda i, j: i * (n + 1) + j  # noqa: E731
    tris = []
    for i in range(n):
        for j in range(n):
            a, b, c, d = vid(i, j), vid(i + 1, j), vid(i + 1, j + 1), vid(i, j + 1)
            if (i + j) % 2 == 0:
                tris += [(a, b, c), (a, c, d)]
            else:
                tris += [(a, b, d), (b, c, d)]
    return xy, np.asarray(tris, dtype=np.int64)


def _refine(xy, tris):
    """1->4 midpoint subdivision. Returns (xy, tris, parent) with children of coarse
    face c at rows 4c..4c+3."""
    edge_mid = {}
    new_xy = [xy]
    nxt = xy.shape[0]
    extra = []

    def mid(a, b):
        nonlocal nxt
        key = (a, b) if a < b else (b, a)
        if key not in edge_mid:
            edge_mid[key] = nxt
            extra.append(0.5 * (xy[a] + xy[b]))
            nxt += 1
        return edge_mid[key]

    out = np.empty((tris.shape[0] * 4, 3), dtype=np.int64)
    for f, (a, b, c) in enumerate(tris):
        ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
        out[4 * f + 0] = (a, ab, ca)
        out[4 * f + 1] = (ab, b, bc)
        out[4 * f + 2] = (ca, bc, c)
        out[4 * f + 3] = (ab, bc, ca)
    new_xy.append(np.asarray(extra))
    parent = np.repeat(np.arange(tris.shape[0]), 4)
    return np.concatenate(new_xy, 0), out, parent


def _dual_graph(tris):
    """Undirected dual edges (both directions, sorted by (row, col)) and, for every
    boundary edge, the face it bounds."""
    e2f = {}
    for f, (a, b, c) in enumerate(tris):
        for u, v in ((a, b), (b, c), (c, a)):
            key = (u, v) if u < v else (v, u)
            e2f.setdefault(key, []).append(f)
    pairs = []
    boundary = {}
    for key, faces in e2f.items():
        if len(faces) == 2:
            f1, f2 = faces
            pairs.append((f1, f2))
            pairs.append((f2, f1))
        else:
            boundary[key] = faces[0]
    pairs = np.asarray(sorted(pairs), dtype=np.int64).T
    return pairs, boundary


def _smooth_dem(cx, cy, rng, size=1000.0, amp=2.0):
    z = 0.004 * cx + 0.002 * cy  # gentle regional slope
    for _ in range(6):
        kx, ky = rng.uniform(0.5, 4.0, 2) * 2 * np.pi / size
        ph = rng.uniform(0, 2 * np.pi)
        z = z + amp * rng.uniform(0.2, 1.0) * np.sin(kx * cx + ph) * np.cos(ky * cy + ph / 2)
    return z


def _standardize(v):
    s = v.std()
    return (v - v.mean()) / (s if s > 0 else 1.0)


def hydrograph_bc(T, previous_t=3, peak=3.0, seed=0):
    """BC[1, p, T+1]: sliding window (oldest first) over a smooth inflow hydrograph.
    BC[0, tau, t] = q(t + tau - (p - 1) + 1), q(k<=0)=0 (dataset.py:371-380 pads two
    dry steps before the first map)."""
    rng = np.random.default_rng(seed)
    k = np.arange(-previous_t, T + previous_t + 1, dtype=np.float64)
    rise = max(T * rng.uniform(0.3, 0.5), 1.0)
    q = np.where(k <= 0, 0.0, peak * np.sin(np.clip(k / rise, 0, 1) * np.pi / 2) ** 2
                 * np.exp(-np.clip(k - rise, 0, None) / (2.0 * T)))
    bc = np.zeros((1, previous_t, T + 1), dtype=np.float32)
    for t in range(T + 1):
        for tau in range(previous_t):
            kk = t + tau - (previous_t - 1) + 1
            bc[0, tau, t] = q[kk + previous_t]
    return bc


# ----------------------------------------------------------------------------- builder
def make_multiscale_mesh(n_coarse=3, num_scales=4, seed=0, T=48, previous_t=3,
                         jitter=0.25, size=1000.0, bc_peak=3.0):
    """Multi-scale graph (scale 0 finest).  The finest scale has 2*n^2*4^(S-1) faces
    (+1 ghost).  Returns a :class:`Graph` with the reference's attribute names."""
    rng = np.random.default_rng(seed)
    xy0, tris0 = _coarse_triangulation(n_coarse, rng, jitter, size)
    levels = [(xy0, tris0, None)]  # coarsest first
    for _ in range(num_scales - 1):
        xy, tris, _ = levels[-1]
        xy2, tris2, parent = _refine(xy, tris)
        levels.append((xy2, tris2, parent))
    levels = levels[::-1]  # finest first; levels[s][2] = parent of scale-s faces in scale s+1

    # BC point on the left boundary (x=0), mid-height of a finest boundary edge
    fxy, ftris, _ = levels[0]
    n_fine_side = n_coarse * 2 ** (num_scales - 1)
    y_bc = (n_fine_side // 2 + 0.5) * size / n_fine_side

    scales = []
    for s, (xy, tris, parent) in enumerate(levels):
        nf = tris.shape[0]
        c = xy[tris].mean(1)
        p0, p1, p2 = xy[tris[:, 0]], xy[tris[:, 1]], xy[tris[:, 2]]
        area = 0.5 * np.abs((p1[:, 0] - p0[:, 0]) * (p2[:, 1] - p0[:, 1])
                            - (p2[:, 0] - p0[:, 0]) * (p1[:, 1] - p0[:, 1]))
        dual, boundary = _dual_graph(tris)
        bc_face = None
        for (u, v), f in boundary.items():
            if abs(xy[u, 0]) < 1e-9 and abs(xy[v, 0]) < 1e-9:
                lo, hi = sorted((xy[u, 1], xy[v, 1]))
                if lo <= y_bc <= hi:
                    bc_face = f
                    bc_edge_len = hi - lo
                    break
        assert bc_face is not None
        ghost = nf
        ghost_c = np.array([-c[bc_face, 0], c[bc_face, 1]])
        cc = np.concatenate([c, ghost_c[None]], 0)
        edge_index = np.concatenate([dual, np.array([[ghost], [bc_face]])], 1)
        dist = np.linalg.norm(cc[edge_index[0]] - cc[edge_index[1]], axis=1)
        scales.append(dict(nf=nf, c=cc, area=np.append(area, area[bc_face]),
                           edge_index=edge_index, dist=dist, bc_face=bc_face,
                           parent=parent, bc_edge_len=bc_edge_len))

    # DEM on the finest scale, pooled (mean of children) to coarse scales
    sc0 = scales[0]
    dem = [_smooth_dem(sc0["c"][:-1, 0], sc0["c"][:-1, 1], rng, size)]
    for s in range(1, num_scales):
        par = scales[s - 1]["parent"]
        nf = scales[s]["nf"]
        sm = np.zeros(nf)
        np.add.at(sm, par, dem[-1])
        cnt = np.bincount(par, minlength=nf)
        dem.append(sm / np.maximum(cnt, 1))
    dem_min = min(d.min() for d in dem)
    for s in range(num_scales):
        d = dem[s] - dem_min
        scales[s]["dem"] = np.append(d, d[scales[s]["bc_face"]])  # ghost copies BC face

    face_ptr = np.cumsum([0] + [sc["nf"] + 1 for sc in scales])
    edge_ptr = np.cumsum([0] + [sc["edge_index"].shape[1] for sc in scales])
    N = int(face_ptr[-1])

    edge_index = np.concatenate([sc["edge_index"] + face_ptr[s] for s, sc in enumerate(scales)], 1)
    edge_attr = np.concatenate([_standardize(sc["dist"]) for sc in scales])[:, None]
    area = np.concatenate([_standardize(sc["area"]) for sc in scales])
    dem_all = np.concatenate([sc["dem"] for sc in scales])

    intra = []
    for s in range(num_scales - 1):
        fine, coarse = scales[s], scales[s + 1]
        pairs = [(p, f) for f, p in enumerate(fine["parent"])]
        pairs.append((coarse["nf"], fine["nf"]))  # ghost nests in the coarse ghost
        pairs = np.asarray(sorted(pairs), dtype=np.int64).T  # np.where order (coarse-major)
        pairs = pairs + np.array([[face_ptr[s + 1]], [face_ptr[s]]])
        intra.append(pairs)
    intra_edge_ptr = np.cumsum([0] + [p.shape[1] for p in intra])
    intra_edge_index = (np.concatenate(intra, 1) if intra else np.zeros((2, 0), np.int64))

    x = np.zeros((N, 2 + 2 * previous_t), dtype=np.float32)
    x[:, 0] = area
    x[:, 1] = dem_all
    bc = hydrograph_bc(T, previous_t, peak=bc_peak, seed=seed)  # unit discharge [m^2/s]
    node_BC = np.array([face_ptr[0] + scales[0]["nf"]], dtype=np.int32)

    return Graph(
        x=torch.from_numpy(x),
        edge_index=torch.from_numpy(edge_index.astype(np.int64)),
        edge_attr=torch.from_numpy(edge_attr.astype(np.float32)),
        edge_ptr=torch.from_numpy(edge_ptr.astype(np.int64)),
        node_ptr=torch.from_numpy(face_ptr.astype(np.int64)),
        intra_mesh_edge_index=torch.from_numpy(intra_edge_index.astype(np.int64)),
        intra_edge_ptr=torch.from_numpy(intra_edge_ptr.astype(np.int64)),
        BC=torch.from_numpy(bc.astype(np.float32)),
        node_BC=torch.from_numpy(node_BC),
        type_BC=torch.tensor(2, dtype=torch.int),
        y=torch.zeros(N, 2, T),
        temporal_res=torch.tensor(120),
        previous_t=torch.tensor(previous_t),
        # raw cell areas [m^2] and BC edge length [m] per scale (the reference's data.area /
        # data.edge_BC_length, used by the mass-conservation metric, loss.py:120-169)
        area=torch.from_numpy(np.concatenate([sc["area"] for sc in scales]).astype(np.float32)),
        edge_BC_length=torch.tensor([sc["bc_edge_len"] for sc in scales], dtype=torch.float32),
    )


def make_single_scale_mesh(n_coarse=3, refinements=3, seed=0, T=10, previous_t=3, **kw):
    """Single-scale graph (finest level of the hierarchy only) for the GNN model:
    keeps x / edge_index / edge_attr / BC / node_BC / type_BC / y."""
    g = make_multiscale_mesh(n_coarse, refinements + 1, seed, T, previous_t, **kw)
    n0 = int(g.node_ptr[1])
    e0 = int(g.edge_ptr[1])
    return Graph(x=g.x[:n0].clone(), edge_index=g.edge_index[:, :e0].clone(),
                 edge_attr=g.edge_attr[:e0].clone(), BC=g.BC.clone(), node_BC=g.node_BC.clone(),
                 type_BC=g.type_BC.clone(), y=torch.zeros(n0, 2, T),
                 temporal_res=g.temporal_res, previous_t=g.previous_t,
                 area=g.area[:n0].clone(), edge_BC_length=g.edge_BC_length[:1].clone())


def wet_state(graph, seed=0, depth=0.8, frac=0.35, previous_t=3, all_wet=False):
    """Return a copy of ``graph`` whose dynamic columns hold a smooth wet patch
    (h >= 0 with dry cells exactly 0, q = |v| h), coarse scales = mean of children.
    ``all_wet`` makes every cell wet (deterministic full work for the HBM stress)."""
    rng = np.random.default_rng(seed + 1000)
    g = graph.clone()
    x = g.x.numpy().copy()
    N = x.shape[0]
    dem = x[:, 1]
    u = rng.uniform(0.2, 1.0, size=(N, previous_t))
    thr = np.quantile(dem, frac) if not all_wet else np.inf
    wet = (dem <= thr) | all_wet
    for tau in range(previous_t):
        h = np.where(wet, depth * (0.3 + 0.7 * u[:, tau]) * (1 + 0.1 * tau), 0.0)
        q = h * rng.uniform(0.0, 0.6, size=N)
        x[:, 2 + 2 * tau] = h
        x[:, 3 + 2 * tau] = q
    g.x = torch.from_numpy(x.astype(np.float32))
    return g


def config3_members(num_scales=3, count=8):
    """BASELINE config 3: a batch of Zenodo-like test meshes whose fine-cell counts span the
    real test set's 8,191-12,989 (database/overview.csv:82-101): coarse sizes cycled so the
    members hold 8,193-12,801 fine nodes (incl. the ghost), seeds 0..count-1.
    Returns make_multiscale_mesh keyword dicts."""
    if num_scales == 4:
        sizes = [8, 9, 10]                    # 8,192 / 10,368 / 12,800 fine faces
    elif num_scales == 3:
        sizes = [16, 17, 18, 19, 20]          # 8,192 / 9,248 / 10,368 / 11,552 / 12,800
    else:
        raise ValueError("config 3 is defined for 3 or 4 scales")
    return [dict(n_coarse=sizes[i % len(sizes)], num_scales=num_scales, seed=i) for i in range(count)]


def mesh_config(name):
    """Named workloads of BASELINE.json configs."""
    table = {
        # unit-test sizes
        "tiny": dict(n_coarse=2, num_scales=4),       # N0 = 513
        "small": dict(n_coarse=3, num_scales=4),      # N0 = 1153
        "small3": dict(n_coarse=6, num_scales=3),     # N0 = 1153, 3 scales
        # config 2: single Zenodo-like mesh
        "zenodo4": dict(n_coarse=9, num_scales=4),    # N0 = 10369, N = 13774, E = 40774
        "zenodo3": dict(n_coarse=18, num_scales=3),   # N0 = 10369, 3 scales
        # config 4: dk15-like
        "dk15": dict(n_coarse=13, num_scales=4),      # N0 = 21633
        # config 5: ~1M fine nodes, 3 scales
        "hbm1m": dict(n_coarse=177, num_scales=3),    # N0 = 1,002,529
    }
    return table[name]
