"""Rollout-path operators of the reference, restated without PyG, plus the fused rollout.

  apply_boundary_condition  utils/dataset.py:486-497
  check_type_BC             utils/dataset.py:499-506
  use_prediction            utils/dataset.py:508-529
  create_scale_mask         utils/dataset.py:615-638
  adapt_batch_training      training/train.py:14-29
  update_batch_multiscale   training/train.py:31-65
  rollout_test              training/train.py:67-95
  split_rollout             training/train.py:182-185 (LightningTrainer.predict_step)

These live in the engine package, not in packages named ``training`` / ``utils``: the
drop-in replaces only the reference's ``models`` package, so the
reference's own ``training.train`` / ``utils.dataset`` stay importable for its callers
(main.py, test_model.py).  ``rollout_test`` here is the fused variant: for our GNN / MSGNN
on a GPU it is ONE engine call (msw_rollout; the T steps replay a captured hipGraph, the BC
write and the window shift fused into the decoder kernel).  ``MSWEGNN_FUSED_ROLLOUT=1`` in
the environment (read by ``models/__init__.py``, :mod:`mswegnn.hooks`) installs it in place
of the reference's ``training.train.rollout_test``.  If ``training.train`` is itself being
imported at that moment, the swap happens at the first model call, so that first
``rollout_test`` call still steps the reference's loop (one graph-replayed ``msw_forward``
per step); every later call is fused.
"""
import weakref

import numpy as np
import torch

NUM_WATER_VARS = 2

__all__ = ["apply_boundary_condition", "check_type_BC", "use_prediction", "create_scale_mask",
           "is_batch", "adapt_batch_training", "update_batch_multiscale", "rollout_test",
           "split_rollout"]


def is_batch(data):
    """A PyG ``Batch`` (or mswegnn.batch.Batch): has ``num_graphs`` and ``ptr``."""
    return hasattr(data, "num_graphs") and hasattr(data, "ptr")


def check_type_BC(type_BC, num_water_vars):
    if type_BC == 1 or type_BC == 2:
        assert type_BC <= num_water_vars, \
            "The boundary conditions are not compatible with the data format you are using."
    elif type_BC == 3:
        raise ValueError("Vector boundary conditions are not implemented.")
    else:
        raise ValueError(f"BC_type={type_BC} is not a valid input. Please select either:\n"
                         "1: Inflow water depth\n2: Inflow discharge")


def apply_boundary_condition(x_d, BC, node_BC, type_BC=2):
    """Write the inflow BC into the dynamic columns of the BC nodes:
    x_d[node_BC, (type_BC-1)::2] = BC (type 1: depth h, type 2: discharge |q|)."""
    type_BC = int(type_BC)
    check_type_BC(type_BC, NUM_WATER_VARS)
    x_d[node_BC.long(), (type_BC - 1)::NUM_WATER_VARS] = BC
    return x_d


def use_prediction(x, pred, previous_t):
    """Slide the dynamic window by one step and append the prediction."""
    assert pred.shape[-1] == NUM_WATER_VARS, \
        "The number of predictions is not consistent with the number of future time steps"
    dyn = previous_t * NUM_WATER_VARS
    n_static = x.shape[1] - dyn
    keep = x[:, n_static + NUM_WATER_VARS:] if previous_t > 1 else x[:, :0]
    out = torch.cat((x[:, :n_static], keep, pred), 1)
    assert out.shape == x.shape, f'The shape of the input has changed from {x.shape} to {out.shape}'
    return out


_PTR_LISTS = {}


def ptr_list(t):
    """A small index tensor (node_ptr / edge_ptr / intra_edge_ptr) as Python ints, read from
    the device once per tensor and in-place version: slicing with its 0-d elements (as the
    reference does) synchronises the host on every slice, which on a GPU drains the queue
    ~50 times per forward (the training step's autograd path)."""
    if not t.is_cuda:
        return t.tolist()
    hit = _PTR_LISTS.get(id(t))
    if hit is not None and hit[0]() is t and hit[1] == t._version:
        return hit[2]
    lst = t.tolist()
    if len(_PTR_LISTS) > 256:
        _PTR_LISTS.clear()
    _PTR_LISTS[id(t)] = (weakref.ref(t), t._version, lst)
    return lst


def create_scale_mask(num_nodes, num_scales, node_ptr, data_type=None, device='cpu'):
    """Scale id per node from node_ptr ([S+1], or [G, S+1] for a batch)."""
    mask = torch.zeros(num_nodes, dtype=torch.int, device=device)
    rows = ptr_list(node_ptr) if node_ptr.dim() == 2 else [ptr_list(node_ptr)]
    for i in range(num_scales):
        for j in rows:
            mask[j[i]:j[i + 1]] = i
    return mask


def update_batch_multiscale(batch):
    """Regroup a batch of multi-scale graphs scale-major and make node_ptr [G, S+1]."""
    G = batch.num_graphs
    edge_ptr = batch.edge_ptr.reshape(G, -1)
    intra_ptr = batch.intra_edge_ptr.reshape(G, -1)
    node_ptr = batch.node_ptr.reshape(G, -1)
    S = intra_ptr.shape[1]

    def cumulate(ptr):
        rows = [ptr[0]]
        for line in ptr[1:]:
            rows.append(line + rows[-1].max())
        return torch.stack(rows)

    edge_ptr, intra_ptr, node_ptr = cumulate(edge_ptr), cumulate(intra_ptr), cumulate(node_ptr)
    ie = [torch.cat([batch.intra_mesh_edge_index[:, a:b] for a, b in intra_ptr[:, i:i + 2]], 1)
          for i in range(S - 1)]
    ei = [torch.cat([batch.edge_index[:, a:b] for a, b in edge_ptr[:, i:i + 2]], 1) for i in range(S)]
    ea = [torch.cat([batch.edge_attr[a:b] for a, b in edge_ptr[:, i:i + 2]]) for i in range(S)]
    batch.node_ptr = node_ptr
    batch.edge_index = torch.cat(ei, 1)
    batch.edge_attr = torch.cat(ea)
    batch.edge_ptr = torch.LongTensor(np.cumsum([0] + [e.shape[1] for e in ei]))
    batch.intra_edge_ptr = torch.LongTensor(np.cumsum([0] + [e.shape[1] for e in ie]))
    batch.intra_mesh_edge_index = torch.cat(ie, 1)


def _graph_of_node(node_BC, lo, hi):
    """Index of the graph whose [lo, hi] node range holds each BC node (train.py:24-28; the
    reference's closed interval, first match)."""
    nb = node_BC.detach().cpu().reshape(-1, 1)
    hit = (lo.detach().cpu().reshape(1, -1) <= nb) & (nb <= hi.detach().cpu().reshape(1, -1))
    if not bool(hit.any(1).all()):
        raise ValueError("a BC node lies outside every graph of the batch")
    return hit.int().argmax(1)


def adapt_batch_training(batch):
    """Offset node_BC per graph, take scalar BC metadata, regroup multi-scale batches and
    record the graph of each BC node (``node_BC_ptr``)."""
    assert is_batch(batch), "This function requires a batched graph (num_graphs, ptr)"
    temp = batch.clone()
    temp.node_BC = torch.cat([temp.ptr[i] + temp[i].node_BC for i in range(temp.num_graphs)])
    temp.temporal_res = temp.temporal_res[0]
    temp.type_BC = temp.type_BC[0]
    temp.previous_t = temp.previous_t[0]
    if 'edge_ptr' in temp.keys():
        update_batch_multiscale(temp)
        temp.node_BC_ptr = _graph_of_node(temp.node_BC, temp.node_ptr[:, 0], temp.node_ptr[:, -1])
    else:
        # the reference compares with the scalars ptr[0] / ptr[-1] here (train.py:27-28), so
        # every BC node maps to graph 0
        temp.node_BC_ptr = _graph_of_node(temp.node_BC, temp.ptr[:1], temp.ptr[-1:])
    return temp


def _fused_ok(model, temp):
    from models.gnn import GNN, MSGNN
    return (isinstance(model, (GNN, MSGNN)) and temp.x.is_cuda
            and getattr(model, "engine", "auto") != "torch")


@torch.no_grad()
def rollout_test(model, batch):
    """Autoregressive rollout over T = batch.y.shape[-1] steps -> [N, 2, T]."""
    temp = adapt_batch_training(batch) if is_batch(batch) else batch
    dynamic_vars = model.previous_t * model.NUM_WATER_VARS
    assert temp.x.shape[-1] >= dynamic_vars, \
        "The number of dynamic variables is greater than the number of node features"
    final_step = batch.y.shape[-1]
    if _fused_ok(model, temp):
        return model.rollout(temp, final_step)
    temp = temp.clone()
    preds = []
    for t in range(final_step):
        temp.x[:, -dynamic_vars:] = apply_boundary_condition(temp.x[:, -dynamic_vars:], temp.BC[:, :, t],
                                                             temp.node_BC, type_BC=temp.type_BC)
        pred = model(temp)
        temp.x = use_prediction(temp.x, pred, model.previous_t)
        preds.append(pred)
    return torch.stack(preds, -1)


def split_rollout(rollout, batch):
    """Per-graph pieces of a batched rollout, as LightningTrainer.predict_step returns them
    (training/train.py:182-185): rollout[ptr[i]:ptr[i+1]] for each graph i."""
    return [rollout[int(batch.ptr[i]):int(batch.ptr[i + 1])] for i in range(batch.num_graphs)]
