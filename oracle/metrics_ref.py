"""ORACLE (test infrastructure only): CPU restatement of the reference's rollout evaluation
metrics, the step after the rollout.  Pinned against tests/golden/
fx_metrics.npz, which oracle/gen_golden_metrics.py produced with the reference's own
functions.

  get_mean_error          training/loss.py:8-23
  mask_on_water           training/loss.py:25-35
  get_rollout_loss        utils/miscellaneous.py:177-199 (+ get_masked_diff :171-175)
  get_binary_rollouts     utils/miscellaneous.py:123-136
  get_rollout_confusion_matrix / get_CSI / get_F1   utils/miscellaneous.py:138-169
  get_mass_conservation_loss  utils/miscellaneous.py:116-121 -> conservation_loss
                              training/loss.py:120-169 -> get_inflow_volume dataset.py:577-591
"""
import torch


def get_mean_error(diff, type_loss, nodes_dim=0):
    """training/loss.py:8-23"""
    if type_loss == "RMSE":
        return torch.sqrt((diff ** 2).mean(nodes_dim))
    if type_loss == "MAE":
        return diff.abs().mean(nodes_dim)
    raise ValueError(type_loss)


def rollout_loss(pred, real, type_loss="RMSE", only_where_water=False):
    """utils/miscellaneous.py:177-199 for one simulation [N, 2, T] or a stack [S, N, 2, T]."""
    diff = pred - real
    nodes_dim, water_axis = (1, 2) if diff.dim() == 4 else (0, 1)
    if not only_where_water:
        return get_mean_error(diff, type_loss, nodes_dim=nodes_dim).mean(-1)
    where = (diff != 0).any(water_axis)  # training/loss.py:34

    def one(d, w):
        masked = torch.stack([d[:, v, :][w] for v in range(d.shape[1])])
        return get_mean_error(masked, type_loss, nodes_dim=-1)
    if diff.dim() == 4:
        return torch.stack([one(diff[i], where[i]) for i in range(diff.shape[0])])
    return one(diff, where)


def confusion(pred, real, thr):
    """utils/miscellaneous.py:123-151: flood = water depth (variable 0) > threshold."""
    p = (pred[:, :, 0, :] if pred.dim() == 4 else pred[:, 0, :]) > thr
    r = (real[:, :, 0, :] if real.dim() == 4 else real[:, 0, :]) > thr
    nd = 1 if pred.dim() == 4 else 0
    return (p & r).sum(nd), (~p & ~r).sum(nd), (p & ~r).sum(nd), (~p & r).sum(nd)


def csi(pred, real, thr):
    """utils/miscellaneous.py:153-160 (NaN where no flooded node in either map)"""
    TP, TN, FP, FN = confusion(pred, real, thr)
    return TP / (TP + FN + FP)


def f1(pred, real, thr):
    """utils/miscellaneous.py:162-169"""
    TP, TN, FP, FN = confusion(pred, real, thr)
    return TP / (TP + 0.5 * (FN + FP))


def inflow_volume(bc_t, edge_bc_length, temporal_res):
    """utils/dataset.py:577-591: sum(|q| * L_bc) * 60 s * temporal_res [m^3]"""
    return (bc_t * edge_bc_length).sum() * (60 * temporal_res)


def conservation_loss(pred_wd, input_wd, area, node_bc, bc_t, edge_bc_length, temporal_res):
    """training/loss.py:120-169 (single multi-scale graph; area already the finest rows)"""
    area = area if area.dim() == 2 else area.unsqueeze(1)
    delta = pred_wd - input_wd
    predicted = (area * delta).sum()
    inflow = inflow_volume(bc_t, edge_bc_length, temporal_res)
    correction = (area * delta)[node_bc].sum()
    return (predicted - inflow - correction) / 1e6


def mass_conservation_loss(rollout, area_all, node_ptr, BC, node_bc, edge_bc_length, temporal_res):
    """utils/miscellaneous.py:116-121: rollout = finest rows [n0, 2, T]; BC [n_BC, >= T+1]"""
    area = area_all[node_ptr[0]:node_ptr[1]]
    return torch.stack([conservation_loss(rollout[:, 0::2, t], rollout[:, 0::2, t - 1], area, node_bc,
                                          (BC[:, t] + BC[:, t + 1]) / 2, edge_bc_length, temporal_res)
                        for t in range(1, rollout.shape[-1])])
