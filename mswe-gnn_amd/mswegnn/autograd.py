"""Autograd through the HIP training kernels.

``swegnn_apply(layer, x_s, x_d, edge_index, edge_attr)`` runs one ``SWEGNN`` processor
(models/gnn.py:387-445) as a ``torch.autograd.Function`` whose forward and backward are the
gfx950 kernels of ``csrc/train.hip`` behind the C ABI (``msw_swegnn_train_*``,
include/mswegnn.h): every parameter and input gradient the reference's ``training_step``
(training/train.py:125-145) back-propagates through the layer is computed by HIP kernels --
MFMA GEMMs for the edge-MLP and filter layers (split-K weight gradients), CSR pulls by
destination and by source for the hop's transpose, no atomics.  torch only allocates the
buffers (saved state, scratch, gradients) and orders the work on its current stream.

``mlp_apply(seq, x)`` does the same for a make_mlp Sequential (models/models.py:121-146: the
edge / node encoders and the node decoder) over ``msw_mlp_train_*``.

``pool_apply(x, pool_edges)`` is MSGNN's mean pooling (models/gnn.py:242-257) over
``msw_pool_mean_*``: CSR pulls by coarse node (forward) and by fine node (backward), no
atomics, so the whole training forward / backward is deterministic.

``SWEGNN.forward``, the models' encoder / decoder calls and MSGNN's pooling (models/gnn.py of
this package) route here on a GPU with autograd enabled; the scale selections, skip sums and
the output mask stay elementwise torch ops.
"""
from __future__ import annotations

import ctypes as C
import weakref
from collections import OrderedDict

import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from . import _lib as L
from .engine import _act_code, _raw_stream

__all__ = ["swegnn_apply", "supported", "graph_csr", "mlp_apply", "mlp_supported", "pool_apply", "pool_supported",
           "clear_caches"]

_CSR_CACHE = OrderedDict()
_CSR_KEEP = 32
MLP_CALLS = [0]  # mlp_apply / pool_apply / swegnn_apply calls (tests check that the HIP path ran)
POOL_CALLS = [0]
SWEGNN_CALLS = [0]
# Diagnostics (tests/: the branch-following float64 yardstick).  A list here receives, per HIP
# training-forward call in call order, the discrete decisions the kernels took: the side of
# every activation kink (pre-activation > 0) of each MLP layer and, for SWEGNN, the hop
# predicate out.sum(1) != 0 of every hop (gnn.py:408) -- read back from the saved buffer.
RECORD = None


def _al(n):
    return (n + 63) // 64 * 64  # csrc/train.hip layout_of / mlp_layout_of: 64-float aligned slots


def _swegnn_decisions(d, saved):
    """The saved buffer of msw_swegnn_train_forward (csrc/train.hip layout_of): X0, pre[l],
    post[l], s, nrm, outk, agg, nz -> {pre: [E x w(l+1) bool], nz: [K x N bool]}."""
    E, N, F, K, nl = d.num_edges, d.num_nodes, d.F, d.K, d.n_layers
    w = [d.width[i] for i in range(nl + 1)]
    o = _al(E * w[0])
    pre = []
    for l in range(nl):
        pre.append(saved[o:o + E * w[l + 1]].view(E, w[l + 1]) > 0)
        o += _al(E * w[l + 1])
    for l in range(nl):
        o += _al(E * w[l + 1])
    o += _al(E * F) + _al(E) + _al((K + 1) * N * F) + _al(K * N * F)
    nz = saved[o:o + K * N].view(torch.int32).view(K, N) != 0
    return {"kind": "swegnn", "pre": pre, "nz": [nz[k] for k in range(K)]}


def _mlp_decisions(d, saved):
    """The saved buffer of msw_mlp_train_forward (mlp_layout_of): pre[l], post[l]."""
    R, nl = d.rows, d.n_layers
    o, pre = 0, []
    for l in range(nl):
        w = d.width[l + 1]
        pre.append(saved[o:o + R * w].view(R, w) > 0)
        o += _al(R * w)
    return {"kind": "mlp", "pre": pre}


class GraphCSR:
    """row / col (int32) and the CSRs by destination (col) and by source (row) of one
    edge_index on the GPU; each node's edges in reference (edge_index) order."""

    def __init__(self, edge_index, num_nodes):
        ei = edge_index.to(torch.int64)
        dev = ei.device
        self.num_nodes = int(num_nodes)
        self.num_edges = int(ei.shape[1])
        self.row = ei[0].to(torch.int32).contiguous()
        self.col = ei[1].to(torch.int32).contiguous()

        def csr(key):
            order = torch.sort(key, stable=True).indices.to(torch.int32).contiguous()
            cnt = torch.bincount(key, minlength=self.num_nodes)
            ptr = torch.zeros(self.num_nodes + 1, dtype=torch.int64, device=dev)
            ptr[1:] = torch.cumsum(cnt, 0)
            return ptr.to(torch.int32).contiguous(), order
        self.in_ptr, self.in_edge = csr(ei[1])
        self.out_ptr, self.out_edge = csr(ei[0])


def _drop_csr(key):
    """Forget one cached GraphCSR and every descriptor template bound to it; its owner's
    finalizer is detached (one finalizer per live entry: a graph re-cached every epoch does not
    pile them up, and a stale one can never drop a newer entry under the same key)."""
    ent = _CSR_CACHE.pop(key, None)
    if ent is not None:
        ent[2].detach()
        # a snapshot: a finalizer fired by the cyclic GC may call back into here
        for k in [k for k, m in list(_META_CACHE.items()) if getattr(m, "csr", None) is ent[1]]:
            _META_CACHE.pop(k, None)


def graph_csr(edge_index, num_nodes):
    """Cached GraphCSR, keyed by the index tensor's address, layout and in-place version.  The
    entry holds only a weak reference to the storage owner (the tensor, or the base of a
    slice such as MSGNN's per-scale ``edge_index[:, a:b]``) and is dropped, with the
    descriptors bound to it, when that owner is collected: a training loop over many batches
    keeps no previous batch's graph (or its GPU CSR) alive."""
    key = (edge_index.data_ptr(), tuple(edge_index.shape), tuple(edge_index.stride()), edge_index._version,
           int(num_nodes), str(edge_index.device))
    owner = edge_index._base if edge_index._base is not None else edge_index
    hit = _CSR_CACHE.get(key)
    if hit is not None and hit[0]() is owner:
        _CSR_CACHE.move_to_end(key)
        return hit[1]
    _drop_csr(key)
    g = GraphCSR(edge_index, num_nodes)
    _CSR_CACHE[key] = (weakref.ref(owner), g, weakref.finalize(owner, _drop_csr, key))
    while len(_CSR_CACHE) > _CSR_KEEP:
        _drop_csr(next(iter(_CSR_CACHE)))
    return g


def clear_caches():
    """Drop every cached CSR and descriptor template (their GPU arrays are freed)."""
    for ent in list(_CSR_CACHE.values()):
        ent[2].detach()
    _CSR_CACHE.clear()
    _META_CACHE.clear()


def _mlp_layers(seq):
    """make_mlp Sequential -> [(Linear, activation module or None)]; None if unsupported."""
    layers = []
    for m in seq:
        if isinstance(m, nn.Linear):
            layers.append([m, None])
        elif isinstance(m, nn.Dropout):
            if m.p > 0 and m.training:
                return None
        elif isinstance(m, nn.LayerNorm):
            return None
        elif layers:
            layers[-1][1] = m
        else:
            return None
    if not 1 <= len(layers) <= L.MAX_MLP_LAYERS:
        return None
    for lin, act in layers:
        try:
            _act_code(act)
        except NotImplementedError:
            return None
    return layers


def supported(layer, x_s, x_d, edge_attr):
    """The HIP training path implements this layer call (else the torch path runs): fp32 GPU
    tensors, static and dynamic node features of one width F over the same rows (the kernels'
    edge-MLP input is [x_s(row), x_s(col), x_d(row), x_d(col), e] = 4F + ef wide), no double
    backward (the kernels' backward is not itself differentiable)."""
    if not (x_d.is_cuda and x_s.is_cuda) or x_d.dtype != torch.float32 or x_s.dtype != torch.float32:
        return False
    if x_s.dim() != 2 or x_d.dim() != 2 or x_s.shape != x_d.shape:
        return False
    if layer.K < 1 or layer.K > L.MAX_HOPS or _mlp_layers(layer.edge_mlp) is None:
        return False
    ef = int(layer.edge_features) if layer.edge_features > 0 else 0
    if _mlp_layers(layer.edge_mlp)[0][0].in_features != 4 * x_d.shape[1] + ef:
        return False
    if layer.edge_features > 0 and (edge_attr is None or edge_attr.dtype != torch.float32):
        return False
    return all(p.dtype == torch.float32 and p.is_cuda for p in layer.parameters())


def _param_list(layer=None, seq=None):
    """The parameter objects a descriptor binds, in its order (cache validation)."""
    out = []
    for m in (layer.edge_mlp if layer is not None else seq):
        if isinstance(m, nn.Linear):
            out.append(m.weight)
            if m.bias is not None:
                out.append(m.bias)
        elif isinstance(m, nn.PReLU):
            out.append(m.weight)
    if layer is not None and layer.with_filter_matrix:
        out += [f.weight for f in layer.filter_matrix]
    return out


class _Meta:
    """Everything but the tensors autograd tracks: the descriptor template of one call."""

    def __init__(self, layer, layers, csr, F, ef):
        self.layer, self.layers, self.csr, self.F, self.ef = layer, layers, csr, F, ef
        self.ws = None
        d = L.MswSwegnnTrainDesc()
        d.num_nodes, d.num_edges = csr.num_nodes, csr.num_edges
        d.F, d.edge_features, d.K, d.n_layers = F, ef, layer.K, len(layers)
        d.width[0] = layers[0][0].in_features
        for i, (lin, act) in enumerate(layers):
            d.width[i + 1] = lin.out_features
            d.act[i] = _act_code(act)
        d.normalize = int(bool(layer.normalize))
        d.with_filter_matrix = int(bool(layer.with_filter_matrix))
        d.with_gradient = int(bool(layer.with_gradient))
        d.upwind_mode = int(bool(layer.upwind_mode))
        for name in ("row", "col", "in_ptr", "in_edge", "out_ptr", "out_edge"):
            setattr(d, name, getattr(csr, name).data_ptr())
        self.desc = d
        # parameter list order = the Function's *params
        self.params = []
        for lin, act in layers:
            self.params.append(lin.weight)
            if lin.bias is not None:
                self.params.append(lin.bias)
            if isinstance(act, nn.PReLU):
                self.params.append(act.weight)
        if layer.with_filter_matrix:
            self.params += [f.weight for f in layer.filter_matrix]

    def bind(self, params):
        """Point the descriptor at the (contiguous) parameter tensors of this call."""
        d, it = self.desc, iter(params)
        for i, (lin, act) in enumerate(self.layers):
            d.weight[i] = next(it).data_ptr()
            d.bias[i] = next(it).data_ptr() if lin.bias is not None else None
            d.slope[i] = next(it).data_ptr() if isinstance(act, nn.PReLU) else None
        if self.layer.with_filter_matrix:
            for k in range(self.layer.K + 1):
                d.filter[k] = next(it).data_ptr()
        return d


def _ws(meta):
    if meta.ws is None:  # depends on the descriptor's sizes only
        s, t = C.c_int64(), C.c_int64()
        L.check(L.lib().msw_swegnn_train_workspace(C.byref(meta.desc), C.byref(s), C.byref(t)))
        meta.ws = int(s.value), int(t.value)
    return meta.ws


_META_CACHE = OrderedDict()
_META_KEEP = 64


def _cached_meta(key, params_now, make):
    """Descriptor templates reused across calls (their ctypes structs cost more host time than
    the launches): keyed by the module and graph; valid while the module holds the same
    parameter objects (a replaced Parameter rebuilds it)."""
    hit = _META_CACHE.get(key)
    if hit is not None and len(hit.params) == len(params_now) and all(a is b for a, b in zip(hit.params, params_now)):
        _META_CACHE.move_to_end(key)
        return hit
    meta = make()
    _META_CACHE[key] = meta
    while len(_META_CACHE) > _META_KEEP:
        _META_CACHE.popitem(last=False)
    return meta


class _SwegnnFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, x_s, x_d, edge_attr, *params):
        dev = x_d.device
        x_s, x_d = x_s.contiguous(), x_d.contiguous()
        ea = edge_attr.contiguous() if meta.ef > 0 else None
        params = [p.contiguous() for p in params]
        d = meta.bind(params)
        n_saved, _ = _ws(meta)
        saved = torch.empty(n_saved, device=dev, dtype=torch.float32)
        out = torch.empty(meta.csr.num_nodes, meta.F, device=dev, dtype=torch.float32)
        with torch.cuda.device(dev):  # the kernels launch on the current device
            L.check(L.lib().msw_swegnn_train_forward(C.byref(d), x_s.data_ptr(), x_d.data_ptr(),
                                                     ea.data_ptr() if ea is not None else None,
                                                     saved.data_ptr(), out.data_ptr(),
                                                     C.c_void_p(_raw_stream(dev.index or 0))))
        if RECORD is not None:
            RECORD.append(_swegnn_decisions(d, saved))
        ctx.meta = meta
        ctx.has_ea = edge_attr is not None
        ctx.save_for_backward(x_s, x_d, ea if ea is not None else torch.empty(0, device=dev), saved, *params)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        meta = ctx.meta
        x_s, x_d, ea, saved, *params = ctx.saved_tensors
        dev = x_d.device
        gout = gout.contiguous().to(torch.float32)
        d = meta.bind(params)
        _, n_scratch = _ws(meta)
        scratch = torch.empty(n_scratch, device=dev, dtype=torch.float32)
        g = L.MswSwegnnGrads()
        dxs = torch.empty_like(x_s) if ctx.needs_input_grad[1] else None
        dxd = torch.empty_like(x_d)
        dea = torch.empty_like(ea) if meta.ef > 0 and ctx.needs_input_grad[3] else None
        g.d_x_s = dxs.data_ptr() if dxs is not None else None
        g.d_x_d = dxd.data_ptr()
        g.d_edge_attr = dea.data_ptr() if dea is not None else None
        dps = [torch.empty_like(p) if ctx.needs_input_grad[4 + i] else None for i, p in enumerate(params)]
        it = iter(dps)
        for i, (lin, act) in enumerate(meta.layers):
            w = next(it)
            g.d_weight[i] = w.data_ptr() if w is not None else None
            if lin.bias is not None:
                b = next(it)
                g.d_bias[i] = b.data_ptr() if b is not None else None
            if isinstance(act, nn.PReLU):
                a = next(it)
                g.d_slope[i] = a.data_ptr() if a is not None else None
        if meta.layer.with_filter_matrix:
            for k in range(meta.layer.K + 1):
                f = next(it)
                g.d_filter[k] = f.data_ptr() if f is not None else None
        with torch.cuda.device(dev):  # the kernels launch on the current device
            L.check(L.lib().msw_swegnn_train_backward(C.byref(d), x_s.data_ptr(), x_d.data_ptr(),
                                                      ea.data_ptr() if meta.ef > 0 else None, saved.data_ptr(),
                                                      gout.data_ptr(), C.byref(g), scratch.data_ptr(),
                                                      C.c_void_p(_raw_stream(dev.index or 0))))
        return (None, dxs, dxd, dea if ctx.has_ea else None, *dps)


def swegnn_apply(layer, x_s, x_d, edge_index, edge_attr=None):
    """SWEGNN.forward of `layer` on the HIP training kernels (differentiable)."""
    F = int(x_d.shape[1])
    ef = int(layer.edge_features) if layer.edge_features > 0 else 0
    csr = graph_csr(edge_index, x_d.shape[0])
    key = ("swegnn", id(layer), id(csr), F, ef, layer.K, bool(layer.normalize), bool(layer.with_filter_matrix),
           bool(layer.with_gradient), bool(layer.upwind_mode))
    meta = _cached_meta(key, _param_list(layer),
                        lambda: _Meta(layer, _mlp_layers(layer.edge_mlp), csr, F, ef))
    if ef > 0 and edge_attr.dim() == 1:
        edge_attr = edge_attr.unsqueeze(1)
    SWEGNN_CALLS[0] += 1
    return _SwegnnFunction.apply(meta, x_s, x_d, edge_attr if ef > 0 else None, *meta.params)


def mlp_supported(seq, x):
    """The HIP training path implements this make_mlp call (else the module runs)."""
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 2:
        return False
    layers = _mlp_layers(seq)
    if layers is None or layers[0][0].in_features != x.shape[1]:
        return False
    return all(p.dtype == torch.float32 and p.is_cuda for p in seq.parameters())


class _MlpMeta:
    def __init__(self, layers, rows):
        self.layers = layers
        self.ws = None
        d = L.MswMlpTrainDesc()
        d.rows, d.n_layers = rows, len(layers)
        d.width[0] = layers[0][0].in_features
        for i, (lin, act) in enumerate(layers):
            d.width[i + 1] = lin.out_features
            d.act[i] = _act_code(act)
        self.desc = d
        self.params = []
        for lin, act in layers:
            self.params.append(lin.weight)
            if lin.bias is not None:
                self.params.append(lin.bias)
            if isinstance(act, nn.PReLU):
                self.params.append(act.weight)

    def bind(self, params):
        d, it = self.desc, iter(params)
        for i, (lin, act) in enumerate(self.layers):
            d.weight[i] = next(it).data_ptr()
            d.bias[i] = next(it).data_ptr() if lin.bias is not None else None
            d.slope[i] = next(it).data_ptr() if isinstance(act, nn.PReLU) else None
        return d

    def workspace(self):
        if self.ws is None:
            s, t = C.c_int64(), C.c_int64()
            L.check(L.lib().msw_mlp_train_workspace(C.byref(self.desc), C.byref(s), C.byref(t)))
            self.ws = int(s.value), int(t.value)
        return self.ws


class _MlpFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, x, *params):
        dev = x.device
        x = x.contiguous()
        params = [p.contiguous() for p in params]
        d = meta.bind(params)
        n_saved, _ = meta.workspace()
        saved = torch.empty(max(n_saved, 1), device=dev, dtype=torch.float32)
        out = torch.empty(x.shape[0], meta.layers[-1][0].out_features, device=dev, dtype=torch.float32)
        with torch.cuda.device(dev):  # the kernels launch on the current device
            L.check(L.lib().msw_mlp_train_forward(C.byref(d), x.data_ptr(), saved.data_ptr(), out.data_ptr(),
                                                  C.c_void_p(_raw_stream(dev.index or 0))))
        if RECORD is not None:
            RECORD.append(_mlp_decisions(d, saved))
        ctx.meta = meta
        ctx.save_for_backward(x, saved, *params)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        meta = ctx.meta
        x, saved, *params = ctx.saved_tensors
        dev = x.device
        gout = gout.contiguous().to(torch.float32)
        d = meta.bind(params)
        _, n_scratch = meta.workspace()
        scratch = torch.empty(max(n_scratch, 1), device=dev, dtype=torch.float32)
        g = L.MswMlpGrads()
        dx = torch.empty_like(x) if ctx.needs_input_grad[1] else None
        g.d_x = dx.data_ptr() if dx is not None else None
        dps = [torch.empty_like(p) if ctx.needs_input_grad[2 + i] else None for i, p in enumerate(params)]
        it = iter(dps)
        for i, (lin, act) in enumerate(meta.layers):
            w = next(it)
            g.d_weight[i] = w.data_ptr() if w is not None else None
            if lin.bias is not None:
                b = next(it)
                g.d_bias[i] = b.data_ptr() if b is not None else None
            if isinstance(act, nn.PReLU):
                a = next(it)
                g.d_slope[i] = a.data_ptr() if a is not None else None
        with torch.cuda.device(dev):  # the kernels launch on the current device
            L.check(L.lib().msw_mlp_train_backward(C.byref(d), x.data_ptr(), saved.data_ptr(), gout.data_ptr(),
                                                   C.byref(g), scratch.data_ptr(),
                                                   C.c_void_p(_raw_stream(dev.index or 0))))
        if dx is not None and x.shape[0] == 0:
            dx.zero_()
        return (None, dx, *dps)


def mlp_apply(seq, x):
    """make_mlp `seq` applied to x [rows][in] on the HIP training kernels (differentiable)."""
    rows = int(x.shape[0])
    meta = _cached_meta(("mlp", id(seq), rows), _param_list(seq=seq), lambda: _MlpMeta(_mlp_layers(seq), rows))
    MLP_CALLS[0] += 1
    return _MlpFunction.apply(meta, x, *meta.params)


class _PoolFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, csr, x):
        x = x.contiguous()
        out = torch.empty_like(x)
        dev = x.device
        with torch.cuda.device(dev):  # the kernels launch on the current device
            L.check(L.lib().msw_pool_mean_forward(csr.num_nodes, int(x.shape[1]), csr.col.data_ptr(),
                                                  csr.out_ptr.data_ptr(), csr.out_edge.data_ptr(), x.data_ptr(),
                                                  out.data_ptr(), C.c_void_p(_raw_stream(dev.index or 0))))
        ctx.csr = csr
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        csr = ctx.csr
        gout = gout.contiguous().to(torch.float32)
        dx = torch.empty_like(gout)
        dev = gout.device
        with torch.cuda.device(dev):  # the kernels launch on the current device
            L.check(L.lib().msw_pool_mean_backward(csr.num_nodes, int(gout.shape[1]), csr.row.data_ptr(),
                                                   csr.out_ptr.data_ptr(), csr.in_ptr.data_ptr(),
                                                   csr.in_edge.data_ptr(), gout.data_ptr(), dx.data_ptr(),
                                                   C.c_void_p(_raw_stream(dev.index or 0))))
        return None, dx


def pool_supported(x, pool_edges):
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and pool_edges.is_cuda
            and pool_edges.dim() == 2 and pool_edges.shape[0] == 2)


def pool_apply(x, pool_edges):
    """Mean pooling of x [N][F] over pool_edges [2][E] = (coarse, fine) rows (a slice of
    intra_mesh_edge_index, gnn.py:310) on the HIP kernels (differentiable)."""
    POOL_CALLS[0] += 1
    return _PoolFunction.apply(graph_csr(pool_edges, x.shape[0]), x)
