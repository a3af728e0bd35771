"""ORACLE -- test infrastructure only.  CPU restatement of the reference hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline -- never as the product path.

It restates, op for op and in the same order, the reference's multi-scale rollout
(sdat2/mSWE-GNN @ /root/reference):

  rollout_test            training/train.py:67-95
  apply_boundary_condition utils/dataset.py:486-497
  use_prediction          utils/dataset.py:508-529
  create_scale_mask       utils/dataset.py:615-638
  MSGNN.forward           models/gnn.py:267-350 (+ _pooling :242-257)
  GNN.forward             models/gnn.py:102-152
  SWEGNN.forward          models/gnn.py:387-445
  make_mlp / activations  models/models.py:121-169
  residual / WD mask      models/models.py:50-91

It uses the same ATen CPU ops as the reference (F.linear, F.prelu, torch.cat, boolean
indexing, vector_norm, scatter_add_) so on CPU it is bit-identical to the reference; this
is pinned by tests/test_oracle_golden.py against fixtures produced by the reference itself
(oracle/gen_golden.py).  The only third-party arithmetic, PyG 2.4.0 ``scatter``, is
restated in :func:`scatter` (sum / mean over dim 0).

Weights are a plain ``{name: tensor}`` dict with the reference's state-dict key names.
"""
from __future__ import annotations

import torch
import torch.nn.functional as Fn
from torch.linalg import vector_norm

NUM_WATER_VARS = 2

# ------------------------------------------------------------------ branch following
# Off by default (then every function below is the op-for-op restatement).  Set through
# `following(tape)`: a list of the discrete decisions a fp32 run took, in call order --
# {"kind": "mlp", "pre": [bool per layer]} per make_mlp call, {"kind": "swegnn", "pre": [...],
# "nz": [bool per hop]} per SWEGNN call (mswegnn.autograd.RECORD reads them back from the HIP
# kernels), {"kind": "out", "x": relu'd output} per forward.  The restatement then takes those
# sides of every discontinuity the reference's arithmetic has (activation kinks, the hop
# predicate out.sum(1) != 0, the ReLU and _mask_small_WD of the output) and exact arithmetic
# everywhere else: run in float64 it is the yardstick of that fp32 run's ROUNDING, separated from
# its branch decisions (tests/test_gpu_train.py).
_TAPE = None


class following:
    """Context manager: the restatement follows `tape` (see above); `.flips` collects, per
    decision, where the yardstick's own arithmetic would have taken the other side.
    `following(None)` RECORDS instead: the run's own decisions are appended to `.tape` (the
    tape of a restatement run, e.g. the reference's arithmetic in fp32)."""

    def __init__(self, tape):
        self.recording = tape is None
        self.tape, self.pos, self.flips = ([] if tape is None else list(tape)), 0, []

    def next(self, kind):
        rec = self.tape[self.pos]
        assert rec["kind"] == kind, (self.pos, rec["kind"], kind)
        self.pos += 1
        return rec

    def __enter__(self):
        global _TAPE
        _TAPE = self
        return self

    def __exit__(self, *exc):
        global _TAPE
        _TAPE = None


def _mlp_sides(P, prefix, x, n_layers, act, dropout=False):
    """The kink sides (pre-activation > 0) of every layer of a natural make_mlp pass."""
    per = 1 + (1 if dropout else 0) + (1 if act is not None else 0)
    sides = []
    for i in range(n_layers):
        li = i * per
        x = Fn.linear(x, P[f"{prefix}.{li}.weight"], P.get(f"{prefix}.{li}.bias"))
        sides.append((x > 0).detach())
        if act is not None:
            x = activation(act, x, P.get(f"{prefix}.{li + per - 1}.weight"))
    return sides


def _forced(name, x, w, side, where):
    """activation(name, x, w) taking the recorded side of the kink (side: x > 0 in the run
    followed); `where` labels the decision for the flip log."""
    if name not in ("prelu", "relu", "leakyrelu"):
        return activation(name, x, w)
    side = side.to(x.device)
    flip = side != (x > 0)
    if bool(flip.any()):  # (decision, how many, largest distance of the own value to the kink)
        _TAPE.flips.append((where, int(flip.sum()), float(x.detach()[flip].abs().max())))
    neg = w * x if name == "prelu" else (0.1 * x if name == "leakyrelu" else torch.zeros_like(x))
    return torch.where(side, x, neg)


# ------------------------------------------------------------------ PyG scatter (2.4.0)
def scatter(src, index, dim_size, reduce="sum"):
    """torch_geometric.utils.scatter over dim 0 (gnn.py:7; call sites :254,256,437)."""
    size = (dim_size,) + tuple(src.shape[1:])
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    out = src.new_zeros(size).scatter_add_(0, idx, src)
    if reduce in ("sum", "add"):
        return out
    if reduce == "mean":
        count = src.new_zeros(dim_size)
        count.scatter_add_(0, index, src.new_ones(src.shape[0]))
        count = count.clamp(min=1)
        return out / count.view(-1, *([1] * (src.dim() - 1)))
    raise NotImplementedError(reduce)


# ------------------------------------------------------------------ MLPs (models.py)
def activation(name, x, w=None):
    """activation_functions (models/models.py:149-169)."""
    if name is None:
        return x
    if name == "prelu":
        return Fn.prelu(x, w)
    if name == "relu":
        return torch.relu(x)
    if name == "leakyrelu":
        return Fn.leaky_relu(x, 0.1)
    if name == "elu":
        return Fn.elu(x)
    if name == "swish":
        return Fn.silu(x)
    if name == "sigmoid":
        return torch.sigmoid(x)
    if name == "tanh":
        return torch.tanh(x)
    raise AttributeError(name)


def mlp(P, prefix, x, n_layers, act, dropout=False, sides=None):
    """make_mlp Sequential (models/models.py:121-146): Linear -> [Dropout] -> act after
    EVERY layer (also the last).  Module indices follow the Sequential layout.  `sides`
    (branch following only): the recorded kink sides per layer."""
    if _TAPE is not None and _TAPE.recording:
        if sides is None:  # a make_mlp call of its own (not a SWEGNN's edge MLP)
            _TAPE.tape.append({"kind": "mlp", "pre": _mlp_sides(P, prefix, x, n_layers, act, dropout)})
        sides = None
    elif _TAPE is not None and sides is None:
        sides = _TAPE.next("mlp")["pre"]
    per = 1 + (1 if dropout else 0) + (1 if act is not None else 0)
    for i in range(n_layers):
        li = i * per
        W = P[f"{prefix}.{li}.weight"]
        b = P.get(f"{prefix}.{li}.bias")
        x = Fn.linear(x, W, b)
        if act is not None:
            ai = li + per - 1
            if sides is not None:
                x = _forced(act, x, P.get(f"{prefix}.{ai}.weight"), sides[i], f"{prefix}.{li}")
            else:
                x = activation(act, x, P.get(f"{prefix}.{ai}.weight"))
    return x


# ------------------------------------------------------------------ SWEGNN
def swegnn(P, prefix, x_s, x_d, edge_index, edge_attr, K, n_layers, act,
           normalize=True, with_filter_matrix=True, with_gradient=True, upwind_mode=False,
           edge_features=1):
    """SWEGNN.forward, models/gnn.py:387-445."""
    row = edge_index[0]
    col = edge_index[1]
    num_nodes = x_d.size(0)
    rec = _TAPE.next("swegnn") if _TAPE is not None and not _TAPE.recording else None
    if _TAPE is not None and _TAPE.recording:  # every edge's MLP sides + each hop's predicate
        e_all = torch.cat([x_s[row], x_s[col], x_d[row], x_d[col]] + ([edge_attr] if edge_features > 0 else []), 1)
        rec_out = {"kind": "swegnn", "pre": _mlp_sides(P, f"{prefix}.edge_mlp", e_all, n_layers, act), "nz": []}
        _TAPE.tape.append(rec_out)
    if with_filter_matrix:
        out = Fn.linear(x_d.clone(), P[f"{prefix}.filter_matrix.0.weight"])      # :402
    else:
        out = x_d.clone()                                                          # :404
    for k in range(K):
        mask = out.sum(1) != 0                                                     # :408
        if _TAPE is not None and _TAPE.recording:
            rec_out["nz"].append(mask.detach())
        if rec is not None:
            side = rec["nz"][k].to(mask.device)
            if bool((side != mask).any()):
                _TAPE.flips.append((f"{prefix}.hop{k}", int((side != mask).sum()),
                                    float(out.detach().sum(1)[side != mask].abs().max())))
            mask = side
        mask_row = mask[row]
        mask_col = mask[col]
        edge_index_mask = mask_row + mask_col                                      # :411
        e_ij = torch.cat([x_s[row][edge_index_mask], x_s[col][edge_index_mask],
                          x_d[row][edge_index_mask], x_d[col][edge_index_mask]], 1)  # :414
        if edge_features > 0:
            e_ij = torch.cat([e_ij, edge_attr[edge_index_mask]], 1)                # :420
        sides = [p[edge_index_mask.to(p.device)] for p in rec["pre"]] if rec is not None else None
        if _TAPE is not None and _TAPE.recording:
            sides = []  # the edge MLP's sides were recorded above, over every edge
        s_ij = mlp(P, f"{prefix}.edge_mlp", e_ij, n_layers, act, sides=sides)     # :422
        if normalize:
            s_ij = s_ij / vector_norm(s_ij, dim=1, keepdim=True)                   # :425
            s_ij.masked_fill_(torch.isnan(s_ij), 0)                                # :426
        if with_gradient:
            hydraulic_gradient = out[col][edge_index_mask] - out[row][edge_index_mask]  # :430
            if upwind_mode:
                hydraulic_gradient[hydraulic_gradient < 0] = 0
            shift_sum = hydraulic_gradient * s_ij
        else:
            shift_sum = s_ij * out[row][edge_index_mask]                           # :435
        scattered = scatter(shift_sum, col[edge_index_mask], num_nodes, "sum")     # :437
        if with_filter_matrix:
            scattered = Fn.linear(scattered, P[f"{prefix}.filter_matrix.{k + 1}.weight"])  # :441
        out = out + scattered                                                      # :443
    return out


# ------------------------------------------------------------------ BaseFloodModel
def residual(P, cfg, x):
    """BaseFloodModel._add_residual_connection, models/models.py:50-77."""
    p = cfg["previous_t"]
    lr = cfg.get("learned_residuals", None)
    res = torch.zeros(x.shape[0], NUM_WATER_VARS)
    if lr is True:
        x0 = x[:, -p * NUM_WATER_VARS:].reshape(-1, p, NUM_WATER_VARS)
        res = torch.stack([(x0[:, :, i] @ P["residual_weights"][:, 0])
                           for i in range(NUM_WATER_VARS)], -1)
    elif lr == "all":
        x0 = x[:, -p * NUM_WATER_VARS:].reshape(-1, p, NUM_WATER_VARS)
        res = torch.stack([(x0[:, :, i] @ P["residual_weights"][:, i])
                           for i in range(NUM_WATER_VARS)], -1)
    elif lr is False:
        res = x[:, -NUM_WATER_VARS:]
    return res


def mask_small_wd(x, epsilon=0.0001):
    """BaseFloodModel._mask_small_WD, models/models.py:79-91."""
    wd = x[:, 0::NUM_WATER_VARS] * (x[:, 0::NUM_WATER_VARS].abs() > epsilon)
    v = x[:, 1::NUM_WATER_VARS] * (x[:, 0::NUM_WATER_VARS] != 0)
    return torch.cat((wd, v), dim=-1)


def relu_mask(x, epsilon=0.0001):
    """torch.relu then mask_small_wd (gnn.py:345-348) -- or, following a tape, the recorded
    sides of the ReLU and of both masks (the run's relu'd output x_run: x_run > 0, |h| > eps,
    h != 0)."""
    if _TAPE is None or _TAPE.recording:
        y = torch.relu(x)
        if _TAPE is not None:
            _TAPE.tape.append({"kind": "out", "x": y.detach()})
        return mask_small_wd(y, epsilon)
    xr = _TAPE.next("out")["x"].to(x.device)
    pos = xr > 0
    flip = pos != (x > 0)
    if bool(flip.any()):
        _TAPE.flips.append(("relu", int(flip.sum()), float(x.detach()[flip].abs().max())))
    x = torch.where(pos, x, torch.zeros_like(x))
    h = x[:, 0::NUM_WATER_VARS]
    hr = xr[:, 0::NUM_WATER_VARS]
    keep, wet = hr.abs() > epsilon, hr != 0
    for name, a, b, dist in (("depth_mask", keep, h.abs() > epsilon, (h.abs() - epsilon).abs()),
                             ("velocity_mask", wet, h != 0, h.abs())):
        if bool((a != b).any()):
            _TAPE.flips.append((name, int((a != b).sum()), float(dist.detach()[a != b].max())))
    return torch.cat((h * keep, x[:, 1::NUM_WATER_VARS] * wet), dim=-1)


def create_scale_mask(num_nodes, num_scales, node_ptr):
    """utils/dataset.py:615-638 (single graph, or 2-D node_ptr for a batch)."""
    mask = torch.zeros(num_nodes, dtype=torch.int)
    for i in range(num_scales):
        if node_ptr.dim() == 2:
            for j in node_ptr[:, i:i + 2]:
                mask[j[0]:j[1]] = i
        else:
            mask[node_ptr[i]:node_ptr[i + 1]] = i
    return mask


# ------------------------------------------------------------------ models
def msgnn_forward(P, cfg, graph):
    """MSGNN.forward, models/gnn.py:267-350."""
    S = cfg["num_scales"]
    L = cfg["mlp_layers"]
    act = cfg["mlp_activation"]
    with_WL = cfg["with_WL"]
    p = cfg["previous_t"]
    Kl = cfg["K_list"]
    dyn = p * NUM_WATER_VARS
    nstat = cfg["num_node_features"] - dyn + with_WL
    x = graph.x.clone()
    edge_index, edge_attr = graph.edge_index, graph.edge_attr
    edge_ptr, iei, iptr = graph.edge_ptr, graph.intra_mesh_edge_index, graph.intra_edge_ptr
    mask = create_scale_mask(x.size(0), S, graph.node_ptr)
    if cfg["edge_mlp"]:
        edge_attr = mlp(P, "edge_encoder", edge_attr, L, act)
    x0 = x
    x_s = x[:, :nstat - with_WL]
    x_d = x[:, nstat - with_WL:]
    if with_WL:
        WL = x_s[:, -1] + x_d[:, -NUM_WATER_VARS]
        x_s = torch.cat((x_s, WL.unsqueeze(-1)), 1)
    x_s = mlp(P, "static_node_encoder", x_s, L, act)
    x_d = mlp(P, "dynamic_node_encoder", x_d, L, act)
    x_down = torch.zeros_like(x_d)
    x_up = torch.zeros_like(x_d)
    ef = edge_attr.shape[1]
    kw = dict(normalize=cfg["normalize"], with_filter_matrix=cfg["with_filter_matrix"],
              with_gradient=cfg["with_gradient"], edge_features=ef,
              upwind_mode=cfg.get("upwind_mode", False))  # SWEGNN(upwind_mode=...), gnn.py:365
    for i in range(S - 1):
        x_d = swegnn(P, f"gnn_processor.{i}", x_s, x_d, edge_index[:, edge_ptr[i]:edge_ptr[i + 1]],
                     edge_attr[edge_ptr[i]:edge_ptr[i + 1]], Kl[i], L, act, **kw)
        x_down = x_down + x_d * (mask == i)[:, None]
        col_coarse, row_fine = iei[:, iptr[i]:iptr[i + 1]]
        x_d = scatter(x_d[row_fine], col_coarse, x_d.shape[0], "mean")            # :256
    x_down = x_down + x_d
    for i in range(S):
        gid = S - 1 + i
        x_d = swegnn(P, f"gnn_processor.{gid}", x_s, x_d, edge_index[:, edge_ptr[-i - 2]:edge_ptr[-i - 1]],
                     edge_attr[edge_ptr[-i - 2]:edge_ptr[-i - 1]], Kl[gid], L, act, **kw)
        x_up = x_up + x_d * (mask == S - i - 1)[:, None]
        if i < S - 1:
            ie = iei[:, iptr[-i - 2]:iptr[-i - 1]]
            x_d = swegnn(P, f"intra_scale_gnn.{i}", x_s, x_d, ie, None, 1, L, act,
                         normalize=True, with_filter_matrix=False, with_gradient=False,
                         edge_features=0)
            if cfg["skip_connections"]:
                x_d = x_d + x_down * (mask == S - i - 2)[:, None]
    x = x_up
    x = activation(cfg["gnn_activation"], x, P.get("gnn_activation.weight"))
    x = mlp(P, "node_decoder", x, L, act)
    x = x + residual(P, cfg, x0)
    return relu_mask(x, 0.0001)


def gnn_forward(P, cfg, graph):
    """GNN.forward (type_GNN='SWEGNN'), models/gnn.py:102-152."""
    L = cfg["mlp_layers"]
    act = cfg["mlp_activation"]
    with_WL = cfg["with_WL"]
    p = cfg["previous_t"]
    dyn = p * NUM_WATER_VARS
    nstat = cfg["num_node_features"] - dyn + with_WL
    x = graph.x.clone()
    edge_index, edge_attr = graph.edge_index, graph.edge_attr
    if cfg["edge_mlp"]:
        edge_attr = mlp(P, "edge_encoder", edge_attr, L, act)
    x0 = x
    x_s = x[:, :nstat - with_WL]
    x_d = x[:, nstat - with_WL:]
    if with_WL:
        WL = x_s[:, -1] + x_d[:, -NUM_WATER_VARS]
        x_s = torch.cat((x_s, WL.unsqueeze(-1)), 1)
    x_s = mlp(P, "static_node_encoder", x_s, 2, act)
    x = x_d = mlp(P, "dynamic_node_encoder", x_d, L, act)
    for i in range(cfg["n_GNN_layers"]):
        x = swegnn(P, f"gnn_processor.{i}", x_s, x_d, edge_index, edge_attr, cfg["K"], L, act,
                   normalize=cfg["normalize"], with_filter_matrix=cfg["with_filter_matrix"],
                   with_gradient=cfg["with_gradient"], edge_features=edge_attr.shape[1],
                   upwind_mode=cfg.get("upwind_mode", False))
        x = activation(cfg["gnn_activation"], x, P.get("gnn_activation.weight"))
        x_d = x
    x = mlp(P, "node_decoder", x, L, act, dropout=bool(cfg.get("dropout", 0)))
    x = x + residual(P, cfg, x0)
    return relu_mask(x, 0.0001)


def forward(P, cfg, graph):
    return msgnn_forward(P, cfg, graph) if cfg["type_model"] == "MSGNN" else gnn_forward(P, cfg, graph)


# ------------------------------------------------------------------ rollout
def apply_boundary_condition(x_d, BC, node_BC, type_BC=2):
    """utils/dataset.py:486-497."""
    x_d[node_BC.long(), (int(type_BC) - 1)::NUM_WATER_VARS] = BC
    return x_d


def use_prediction(x, pred, previous_t):
    """utils/dataset.py:508-529."""
    dyn = previous_t * NUM_WATER_VARS
    static_vars = x.shape[1] - dyn
    if previous_t == 1:
        return torch.cat((x[:, :static_vars], pred), 1)
    return torch.cat((x[:, :static_vars], x[:, -dyn + NUM_WATER_VARS:], pred), 1)


@torch.no_grad()
def rollout(P, cfg, graph, steps=None):
    """rollout_test, training/train.py:67-95 (single graph)."""
    temp = graph.clone()
    p = cfg["previous_t"]
    dyn = p * NUM_WATER_VARS
    T = graph.y.shape[-1] if steps is None else steps
    preds = []
    for t in range(T):
        temp.x[:, -dyn:] = apply_boundary_condition(temp.x[:, -dyn:], temp.BC[:, :, t],
                                                    temp.node_BC, type_BC=temp.type_BC)
        pred = forward(P, cfg, temp)
        temp.x = use_prediction(temp.x, pred, p)
        preds.append(pred)
    return torch.stack(preds, -1)


# ------------------------------------------------------------------ config helpers
def msgnn_config(num_scales=4, hid_features=32, K=4, mlp_layers=3, previous_t=3,
                 num_node_features=8, **over):
    """config.yaml:42-58 model block (the shipped K*_F* checkpoints' architecture)."""
    Kl = [K] * num_scales if isinstance(K, int) else list(K)
    Kl = Kl + Kl[::-1][1:]
    cfg = dict(type_model="MSGNN", num_scales=num_scales, hid_features=hid_features, K_list=Kl,
               mlp_layers=mlp_layers, previous_t=previous_t, num_node_features=num_node_features,
               mlp_activation="prelu", gnn_activation="tanh", edge_mlp=True, normalize=True,
               with_filter_matrix=True, with_gradient=True, with_WL=True, learned_residuals=True,
               skip_connections=True)
    cfg.update(over)
    return cfg


def gnn_config(hid_features=32, K=2, n_GNN_layers=2, mlp_layers=1, previous_t=3,
               num_node_features=8, **over):
    """GNN defaults (models/gnn.py:39-42)."""
    cfg = dict(type_model="GNN", hid_features=hid_features, K=K, n_GNN_layers=n_GNN_layers,
               mlp_layers=mlp_layers, previous_t=previous_t, num_node_features=num_node_features,
               mlp_activation="prelu", gnn_activation="prelu", edge_mlp=True, normalize=True,
               with_filter_matrix=True, with_gradient=True, with_WL=True, learned_residuals=True,
               dropout=0)
    cfg.update(over)
    return cfg
