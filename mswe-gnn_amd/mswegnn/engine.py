"""Host side of the HIP engine: model/graph descriptors -> msw_plan, forward and rollout.

This is the Python mirror of the reference's operator interface for the hot path
(``MSGNN.forward`` / ``GNN.forward``, models/gnn.py:102-152, 267-350, and ``rollout_test``,
training/train.py:67-95).  All numerical work runs in libmswegnn.so (gfx950 kernels);
this module only describes the model and the graph to it, and passes device pointers of
torch tensors plus the current HIP stream.
"""
from __future__ import annotations

import ctypes as C
import operator
import weakref

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L

__all__ = ["EnginePlan", "plan_for", "describe_model"]

_raw_stream = torch._C._cuda_getCurrentRawStream if hasattr(torch._C, "_cuda_getCurrentRawStream") \
    else (lambda i: torch.cuda.current_stream(i).cuda_stream)


# ------------------------------------------------------------------ model description
def _f32(keep, t):
    a = np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy())
    keep.append(a)
    return a.ctypes.data_as(L.c_float_p)


def _act_code(mod):
    """enum msw_activation code of an activation module (no device read)."""
    if mod is None:
        return 0
    if isinstance(mod, nn.PReLU):
        if mod.weight.numel() != 1:
            raise NotImplementedError("PReLU with more than one parameter")
        return L.ACT["prelu"]
    for name, cls in (("relu", nn.ReLU), ("elu", nn.ELU), ("swish", nn.SiLU),
                      ("sigmoid", nn.Sigmoid), ("tanh", nn.Tanh)):
        if isinstance(mod, cls):
            return L.ACT[name]
    if isinstance(mod, nn.LeakyReLU):
        if abs(mod.negative_slope - 0.1) > 1e-12:
            raise NotImplementedError("LeakyReLU slope other than 0.1")
        return L.ACT["leakyrelu"]
    raise NotImplementedError(f"activation {type(mod).__name__}")


def _act_of(mod):
    """(code, param) of an activation module (reads a PReLU slope from the device)."""
    code = _act_code(mod)
    if isinstance(mod, nn.PReLU):
        return code, float(mod.weight.detach().reshape(-1)[0])
    return code, 0.0


def _mlp(keep, seq):
    """make_mlp Sequential -> MswMlp (Linear, [Dropout (eval: identity)], activation)."""
    layers = []
    for m in seq:
        if isinstance(m, nn.Linear):
            layers.append([m, None])
        elif isinstance(m, nn.Dropout):
            continue
        elif isinstance(m, nn.LayerNorm):
            raise NotImplementedError("layer_norm MLPs are not used by any shipped config")
        else:
            layers[-1][1] = m
    if not 1 <= len(layers) <= L.MAX_MLP_LAYERS:
        raise NotImplementedError(f"MLP with {len(layers)} layers")
    d = L.MswMlp()
    d.n_layers = len(layers)
    for i, (lin, act) in enumerate(layers):
        e = d.layer[i]
        e.in_features, e.out_features = lin.in_features, lin.out_features
        e.weight = _f32(keep, lin.weight)
        e.bias = _f32(keep, lin.bias) if lin.bias is not None else None
        e.act, e.act_param = _act_of(act)
    return d


def _swegnn(keep, g):
    d = L.MswSwegnn()
    d.K = g.K
    d.normalize = int(bool(g.normalize))
    d.with_filter_matrix = int(bool(g.with_filter_matrix))
    d.with_gradient = int(bool(g.with_gradient))
    d.upwind_mode = int(bool(g.upwind_mode))
    d.edge_features = g.edge_features
    d.edge_mlp = _mlp(keep, g.edge_mlp)
    if g.with_filter_matrix:
        arr = (L.c_float_p * (g.K + 1))(*[_f32(keep, f.weight) for f in g.filter_matrix])
        keep.append(arr)
        d.filter = C.cast(arr, C.POINTER(L.c_float_p))
    else:
        d.filter = None
    return d


def describe_model(model):
    """nn.Module (our models.gnn.GNN / MSGNN) -> (MswModelDesc, keepalive list)."""
    keep = []
    d = L.MswModelDesc()
    is_ms = model.type_model == "MSGNN"
    d.model_type = 0 if is_ms else 1
    d.hid_features = model.hid_features
    d.num_scales = model.num_scales if is_ms else 1
    d.previous_t = model.previous_t
    d.num_node_features = model.num_node_features
    d.with_WL = int(bool(model.with_WL))
    d.skip_connections = int(bool(getattr(model, "skip_connections", False)))
    d.learned_pooling = int(bool(getattr(model, "learned_pooling", False)))
    d.gnn_act, d.gnn_act_param = _act_of(model.gnn_activation)
    M = model._residual_matrix()
    d.residual_weights = _f32(keep, M) if M is not None else None
    d.edge_mlp = int(bool(model.edge_mlp))
    if model.edge_mlp:
        d.edge_encoder = _mlp(keep, model.edge_encoder)
    d.static_encoder = _mlp(keep, model.static_node_encoder)
    d.dynamic_encoder = _mlp(keep, model.dynamic_node_encoder)
    d.decoder = _mlp(keep, model.node_decoder)
    procs = (L.MswSwegnn * len(model.gnn_processor))(*[_swegnn(keep, g) for g in model.gnn_processor])
    keep.append(procs)
    d.num_processors = len(model.gnn_processor)
    d.processors = C.cast(procs, C.POINTER(L.MswSwegnn))
    if is_ms and len(model.intra_scale_gnn):
        ups = (L.MswSwegnn * len(model.intra_scale_gnn))(*[_swegnn(keep, g) for g in model.intra_scale_gnn])
        keep.append(ups)
        d.num_unpool = len(model.intra_scale_gnn)
        d.unpool = C.cast(ups, C.POINTER(L.MswSwegnn))
    else:
        d.num_unpool = 0
        d.unpool = None
    return d, keep


# ------------------------------------------------------------------ graph description
def _i64(keep, t):
    a = np.ascontiguousarray(t.detach().to("cpu", torch.int64).numpy())
    keep.append(a)
    return a.ctypes.data_as(L.c_int64_p)


def describe_graph(model, graph):
    keep = []
    g = L.MswGraphDesc()
    N = int(graph.x.shape[0])
    E = int(graph.edge_index.shape[1])
    g.num_nodes = N
    g.num_edges = E
    g.edge_index = _i64(keep, graph.edge_index.reshape(2, E))
    ea = graph.edge_attr
    if ea.dim() == 1:
        ea = ea.unsqueeze(1)
    g.num_edge_features = int(ea.shape[1])
    g.edge_attr = _f32(keep, ea)
    if model.type_model == "MSGNN":
        S = model.num_scales
        node_ptr = graph.node_ptr
        if node_ptr.dim() == 1:
            node_ptr = node_ptr.reshape(1, -1)
        g.num_scales = S
        g.num_graphs = int(node_ptr.shape[0])
        g.node_ptr = _i64(keep, node_ptr)
        g.edge_ptr = _i64(keep, graph.edge_ptr.reshape(-1))
        iei = graph.intra_mesh_edge_index
        g.num_intra_edges = int(iei.shape[1])
        g.intra_edge_index = _i64(keep, iei)
        g.intra_edge_ptr = _i64(keep, graph.intra_edge_ptr.reshape(-1))
    else:
        g.num_scales = 1
        g.num_graphs = 1
        g.node_ptr = _i64(keep, torch.tensor([0, N]))
        g.edge_ptr = _i64(keep, torch.tensor([0, E]))
        g.num_intra_edges = 0
        g.intra_edge_index = None
        g.intra_edge_ptr = None
    return g, keep


# ------------------------------------------------------------------ plan
class EnginePlan:
    """An msw_plan: the graph (CSR per scale, pooling maps) and packed weights on one GPU."""

    def __init__(self, model, graph, device, exchange=None, rank=-1):
        """exchange: an L.MswExchangeDesc (mswegnn/partition.py) -> the plan of part `rank`
        of a partitioned mesh (msw_plan_create_part)."""
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("the HIP engine needs a GPU device")
        self.num_nodes = int(graph.x.shape[0])
        self.nnf = int(graph.x.shape[1])
        self.previous_t = int(model.previous_t)
        md, k1 = describe_model(model)
        gd, k2 = describe_graph(model, graph)
        h = C.c_void_p()
        lib = L.lib()
        dev = self.device.index or 0
        if exchange is None:
            L.check(lib.msw_plan_create(C.byref(gd), C.byref(md), dev, C.byref(h)))
        else:
            L.check(lib.msw_plan_create_part(C.byref(gd), C.byref(md), dev, C.byref(exchange), int(rank),
                                             C.byref(h)))
        self._h = h
        del k1, k2

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            L.lib().msw_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        # the raw handle of torch's current stream on the plan's device (no Stream object)
        return C.c_void_p(_raw_stream(self.device.index or 0))

    def _x(self, x):
        if x.device != self.device or x.dtype != torch.float32:
            x = x.to(self.device, torch.float32)
        if x.shape != (self.num_nodes, self.nnf):
            raise ValueError(f"x has shape {tuple(x.shape)}, plan expects {(self.num_nodes, self.nnf)}")
        return x.contiguous()

    def accepts(self, x):
        """x can be fed to forward() as is (right device, dtype, shape, contiguous)."""
        return (x.is_cuda and x.device == self.device and x.dtype == torch.float32
                and x.shape == (self.num_nodes, self.nnf) and x.is_contiguous())

    def forward(self, x):
        """MSGNN.forward / GNN.forward on the GPU: x [N, nnf] -> y [N, 2].  The plan replays
        its captured forward graph (msw_forward): two device copies + one graph launch."""
        x = self._x(x)
        y = torch.empty((self.num_nodes, 2), device=self.device, dtype=torch.float32)
        rc = self._fwd(self._h, x.data_ptr(), y.data_ptr(), _raw_stream(self.device.index or 0))
        if rc:
            L.check(rc)
        return y

    @property
    def _fwd(self):
        return L.lib().msw_forward

    def rollout(self, x0, BC, node_BC, type_BC, T, out=None):
        """rollout_test on the GPU -> [N, 2, T] (training/train.py:67-95)."""
        x0 = self._x(x0)
        T = int(T)
        if out is None:
            out = torch.empty(self.num_nodes, 2, T, device=self.device, dtype=torch.float32)
        nbc = np.ascontiguousarray(torch.as_tensor(node_BC).detach().to("cpu", torch.int32).reshape(-1).numpy())
        bc = None
        tstride = 0
        if nbc.size:
            if nbc.min() < 0 or nbc.max() >= self.num_nodes:
                raise ValueError("node_BC holds a node index outside the graph")
            bc = BC.to(self.device, torch.float32)
            if bc.dim() != 3 or bc.shape[0] != nbc.size:
                raise ValueError("BC must be [n_BC, previous_t, T+1]")
            if bc.shape[1] == 1 and self.previous_t > 1:
                # x_d[node_BC, (type_BC-1)::2] = BC broadcasts a single column over the
                # previous_t slots (utils/dataset.py:496); the kernels read [n_BC, p, T+1]
                bc = bc.expand(-1, self.previous_t, -1)
            if bc.shape[1] != self.previous_t:
                raise ValueError(f"BC has {bc.shape[1]} time columns, the model expects previous_t="
                                 f"{self.previous_t} (or 1, broadcast)")
            if bc.shape[2] < T:
                raise ValueError(f"BC holds {bc.shape[2]} time steps, the rollout needs {T}")
            bc = bc.contiguous()
            tstride = int(bc.shape[-1])
        tb = int(torch.as_tensor(type_BC).reshape(-1)[0])
        L.check(L.lib().msw_rollout(self._h, C.c_void_p(x0.data_ptr()),
                                    C.c_void_p(bc.data_ptr() if bc is not None else 0), tstride,
                                    nbc.ctypes.data_as(L.c_int32_p), int(nbc.size), tb, T,
                                    C.c_void_p(out.data_ptr()), self._stream()))
        return out

    def debug_buffer(self, name, F):
        dst = torch.empty(self.num_nodes, F, device=self.device)
        L.check(L.lib().msw_debug_buffer(self._h, name.encode(), C.c_void_p(dst.data_ptr()),
                                         self._stream()))
        return dst

    KERNELS = {"hop": 0, "edge_hop": 1, "pool": 2, "encode": 3, "unpool": 4}  # plan.hip bench_kernel

    def bench_kernel(self, kernel, scale, iters):
        """Enqueue `iters` launches of one kernel on the current stream -> units (rows, edges)
        of one launch.  Bracket with events on torch.cuda.current_stream() to time it."""
        units = (C.c_int64 * 2)()
        L.check(L.lib().msw_bench_kernel(self._h, self.KERNELS[kernel], int(scale), int(iters),
                                         units, self._stream()))
        return int(units[0]), int(units[1])

    def set_graph_capture(self, enable):
        L.check(L.lib().msw_set_graph_capture(self._h, int(bool(enable))))

    def stats(self):
        s = L.MswPlanStats()
        L.check(L.lib().msw_plan_get_stats(self._h, C.byref(s)))
        out = {k: getattr(s, k) for k, _ in L.MswPlanStats._fields_}
        return out


# ------------------------------------------------------------------ cache
_TOPOLOGY = {"GNN": ("edge_index", "edge_attr"),
             "MSGNN": ("edge_index", "edge_attr", "node_ptr", "edge_ptr", "intra_mesh_edge_index",
                       "intra_edge_ptr")}


class _GraphRef:
    """The tensors a plan was built from, held by STRONG reference and compared by identity
    plus in-place version: a freed tensor's address can be reused by a new same-shaped
    tensor (caching allocator), so addresses alone cannot tell two graphs apart."""

    def __init__(self, model, graph):
        self.tensors = tuple(getattr(graph, n) for n in _TOPOLOGY[model.type_model])
        self.versions = tuple(t._version for t in self.tensors)
        self.shape = (tuple(graph.x.shape), str(graph.x.device))

    def matches(self, model, graph):
        ts = tuple(getattr(graph, n) for n in _TOPOLOGY[model.type_model])
        return (self.shape == (tuple(graph.x.shape), str(graph.x.device))
                and all(a is b for a, b in zip(ts, self.tensors))
                and self.versions == tuple(t._version for t in ts))

    def still_valid(self):
        """The held tensors still hold the plan's content: none was modified in place since
        the plan was built from them (or adopted them)."""
        return all(t._version == v for t, v in zip(self.tensors, self.versions))

    def same_content(self, model, graph):
        """Equal values in other tensors (e.g. ``graph.clone()``, which the reference's
        rollout_test makes once per rollout, train.py:80): one device compare per tensor.
        Only meaningful while the held tensors are unmodified (``still_valid``): a held
        tensor edited in place no longer shows the content the plan was built from."""
        ts = tuple(getattr(graph, n) for n in _TOPOLOGY[model.type_model])
        if self.shape != (tuple(graph.x.shape), str(graph.x.device)) or not self.still_valid():
            return False
        for a, b in zip(ts, self.tensors):
            if a.shape != b.shape or a.dtype != b.dtype:
                return False
        return all(torch.equal(a, b.to(a.device)) for a, b in zip(ts, self.tensors))

    def adopt(self, model, graph):
        """Hold the new (equal) tensors so the next calls with them hit by identity."""
        self.tensors = tuple(getattr(graph, n) for n in _TOPOLOGY[model.type_model])
        self.versions = tuple(t._version for t in self.tensors)


# Parameter lists per model, cached: ``model.parameters()`` walks the module tree (~0.35 ms
# for a 150-parameter MSGNN, more than a whole HIP forward).  Any parameter or submodule
# registration anywhere bumps _STRUCT_GEN and invalidates every cached list.
_STRUCT_GEN = [0]
_param_lists = weakref.WeakKeyDictionary()


def _bump_struct_gen(*_args):
    _STRUCT_GEN[0] += 1


try:
    from torch.nn.modules import module as _tm
    _tm.register_module_parameter_registration_hook(_bump_struct_gen)
    _tm.register_module_module_registration_hook(_bump_struct_gen)
    _HOOKED = True
except AttributeError:  # older torch: no global registration hooks -> walk every call
    _HOOKED = False


def _params(model):
    ent = _param_lists.get(model)
    if not _HOOKED or ent is None or ent[0] != _STRUCT_GEN[0]:
        ent = (_STRUCT_GEN[0], list(model.parameters()))
        _param_lists[model] = ent
    return ent[1]


_ver = operator.attrgetter("_version")


def _weights_key(model):
    """(storage addresses, in-place versions) of every parameter: a plan holds a copy of the
    weights, so a moved or modified parameter needs a new plan."""
    ps = _params(model)
    return tuple(map(torch.Tensor.data_ptr, ps)), tuple(map(_ver, ps))


_plans = weakref.WeakKeyDictionary()
CACHE_PLANS = 4  # plans kept per model (most recently used first)


def plan_for(model, graph, unsupported_ok=False):
    """Cached EnginePlan for (model weights, graph topology).

    unsupported_ok: a model or graph the engine does not implement (MSW_ERR_UNSUPPORTED or
    NotImplementedError while describing it) returns None instead of raising, and that
    answer is cached like a plan (the caller takes its torch path)."""
    entries = _plans.setdefault(model, [])
    wk = _weights_key(model)
    for i, (ref, w, plan) in enumerate(entries):
        if ref.matches(model, graph):
            if w == wk:
                entries.insert(0, entries.pop(i))
                if plan is None and not unsupported_ok:
                    break  # rebuild to raise the engine's own error
                return plan
            entries.pop(i)
            if plan is not None:
                plan.close()
            break
    else:
        # plans whose graph tensors were modified in place since: their content is gone
        for ent in [e for e in entries if not e[0].still_valid()]:
            entries.remove(ent)
            if ent[2] is not None:
                ent[2].close()
        for i, (ref, w, plan) in enumerate(entries):
            if w == wk and ref.same_content(model, graph):
                ref.adopt(model, graph)
                entries.insert(0, entries.pop(i))
                if plan is None and not unsupported_ok:
                    break
                return plan
    try:
        plan = EnginePlan(model, graph, graph.x.device)
    except (NotImplementedError, L.EngineError) as e:
        if not unsupported_ok or (isinstance(e, L.EngineError) and e.code != L.MSW_ERR_UNSUPPORTED):
            raise
        plan = None
    entries.insert(0, (_GraphRef(model, graph), wk, plan))
    while len(entries) > CACHE_PLANS:
        old = entries.pop()[2]
        if old is not None:
            old.close()
    return plan
