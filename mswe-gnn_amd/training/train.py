"""Drop-in for the rollout part of the reference's ``training.train``.

  adapt_batch_training     training/train.py:14-29
  update_batch_multiscale  training/train.py:31-65
  rollout_test             training/train.py:67-95

``rollout_test`` keeps the reference's semantics (BC injection -> forward -> window shift,
T = batch.y.shape[-1], output ``stack(preds, -1)`` = [N, 2, T]).  For our GNN / MSGNN on a
GPU it runs as ONE fused engine call (msw_rollout): the T steps are replays of a captured
hipGraph, with the BC write and the window shift fused into the decoder kernel.  For any
other model (or CPU tensors) it runs the step loop with the same operators.

The Lightning module / data module / curriculum of the reference are training
orchestration outside the MI355X hot path.
"""
import numpy as np
import torch

from utils.dataset import use_prediction, apply_boundary_condition, _is_batch


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


def adapt_batch_training(batch):
    """Offset node_BC per graph, take scalar BC metadata, regroup multi-scale batches."""
    assert _is_batch(batch), "This function requires a batched graph (num_graphs, ptr)"
    temp = batch.clone()
    temp.node_BC = torch.cat([temp.ptr[i] + temp[i].node_BC for i in range(temp.num_graphs)])
    temp.temporal_res = temp.temporal_res[0]
    temp.type_BC = temp.type_BC[0]
    temp.previous_t = temp.previous_t[0]
    if 'edge_ptr' in temp.keys():
        update_batch_multiscale(temp)
    return temp


def _fused_ok(model, temp):
    from models.gnn import GNN, MSGNN
    return (isinstance(model, (GNN, MSGNN)) and temp.x.is_cuda
            and getattr(model, "engine", "auto") != "torch")


@torch.no_grad()
def rollout_test(model, batch):
    """Autoregressive rollout over T = batch.y.shape[-1] steps -> [N, 2, T]."""
    temp = adapt_batch_training(batch) if _is_batch(batch) else batch
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
