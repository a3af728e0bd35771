"""On-device rollout evaluation through the C ABI ``msw_rollout_metrics``.

The reference evaluates a rollout on the host after it finished (test_model.py:93-104 ->
SpatialAnalysis, utils/miscellaneous.py:311-330 and :123-199): finest-scale rows only,
RMSE / MAE per water variable averaged over time, CSI and F1 per time step at water-depth
thresholds, and the mass-conservation error per step (miscellaneous.py:116-121 ->
training/loss.py:120-169, utils/dataset.py:577-591).  Here the kernel reduces the rollout where it lives (fp64 partial sums, exact
integer confusion counts) and only a few numbers per step come back.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L


def finest_ranges(graph):
    """Finest-scale row range of every simulation of a graph / batch (create_scale_mask == 0,
    utils/dataset.py:615-638): node_ptr[0:2] for one graph, node_ptr[g, 0:2] for a batch."""
    npt = graph.node_ptr
    if npt.dim() == 1:
        return [(int(npt[0]), int(npt[1]))]
    return [(int(npt[g, 0]), int(npt[g, 1])) for g in range(npt.shape[0])]


def rollout_metrics(pred, real, ranges, thresholds=(0.05, 0.3), mass=None, stream=None):
    """pred, real: [N, 2, T] on the GPU (graph numbering).  ranges: [(start, end)] finest
    rows per simulation.  Returns per simulation (leading dim S):
      rmse, mae             [S, 2]  get_rollout_loss(only_where_water=False)
      rmse_water, mae_water [S, 2]  get_rollout_loss(only_where_water=True)
      csi[thr], f1[thr]     [S, T]  get_CSI / get_F1 (NaN where the step has no flooded cell)
    mass (optional): dict(area=[N] cell areas by graph row, node_bc=[rows per simulation],
    bc=[per simulation [n_BC, >= T+1] boundary discharge], edge_bc_length=[per simulation
    [n_BC] or scalar], temporal_res=minutes per step (scalar or per simulation)) adds
      mass_loss             [S, T-1]  get_mass_conservation_loss (x 1e-6 m^3, as it returns)
    """
    if not (pred.is_cuda and real.is_cuda):
        raise RuntimeError("rollout_metrics runs on the GPU (HIP kernel); tensors are on the CPU")
    if pred.shape != real.shape or pred.dim() != 3 or pred.shape[1] != 2:
        raise ValueError("pred / real must both be [N, 2, T]")
    pred = pred.float().contiguous()
    real = real.float().contiguous()
    T = pred.shape[-1]
    S = len(ranges)
    thr = [float(t) for t in thresholds]
    sums = torch.zeros(S, T, 10, dtype=torch.float64, device=pred.device)
    area = None
    if mass is not None:
        area = torch.as_tensor(mass["area"]).to(pred.device, torch.float32).contiguous()
        if area.shape[0] != pred.shape[0]:
            raise ValueError("mass['area'] must hold one area per graph row")
    counts = torch.zeros(S, T, max(len(thr), 1), 4, dtype=torch.int64, device=pred.device)
    rng = (C.c_int64 * (2 * S))(*[v for r in ranges for v in r])
    th = (C.c_float * max(len(thr), 1))(*thr)
    st = C.c_void_p(stream if stream is not None else torch.cuda.current_stream(pred.device).cuda_stream)
    L.check(L.lib().msw_rollout_metrics(C.c_void_p(pred.data_ptr()), C.c_void_p(real.data_ptr()), T, rng, S,
                                        th, len(thr), C.c_void_p(area.data_ptr() if area is not None else 0),
                                        C.c_void_p(sums.data_ptr()),
                                        C.c_void_p(counts.data_ptr()), st))
    n0 = torch.tensor([e - s for s, e in ranges], dtype=torch.float64, device=pred.device)
    out = {}
    abs_t, sq_t = sums[..., 0:2], sums[..., 2:4]                      # [S, T, 2]
    out["mae"] = (abs_t / n0[:, None, None]).mean(1).float()           # loss.py:22, then .mean(-1)
    out["rmse"] = torch.sqrt(sq_t / n0[:, None, None]).mean(1).float()  # loss.py:20
    cnt = sums[..., 8].sum(1)[:, None]                                 # masked (n, t) pairs
    out["mae_water"] = (sums[..., 4:6].sum(1) / cnt).float()
    out["rmse_water"] = torch.sqrt(sums[..., 6:8].sum(1) / cnt).float()
    out["csi"], out["f1"] = {}, {}
    for k, t in enumerate(thr):
        tp, tn, fp, fn = (counts[:, :, k, i].double() for i in range(4))
        out["csi"][t] = (tp / (tp + fn + fp)).float()                  # miscellaneous.py:157
        out["f1"][t] = (tp / (tp + 0.5 * (fn + fp))).float()           # miscellaneous.py:166
    out["counts"] = counts
    if mass is not None:
        out["mass_loss"] = _mass_loss(pred, sums[..., 9], area, mass, S, T)
    return out


def _per_sim(v, S):
    return list(v) if isinstance(v, (list, tuple)) else [v] * S


def _mass_loss(pred, vol, area, mass, S, T):
    """(predicted volume change - inflow volume - change at the BC cells) / 1e6 per step
    t = 1..T-1 (conservation_loss, training/loss.py:120-169; inflow: get_inflow_volume,
    utils/dataset.py:577-591, with BC averaged over [t, t+1], miscellaneous.py:119-121)."""
    if T < 2:
        return torch.zeros(S, 0, device=pred.device)
    dv = vol[:, 1:] - vol[:, :-1]                                     # sum area * dh, finest rows
    res = torch.empty(S, T - 1, dtype=torch.float64, device=pred.device)
    tres = _per_sim(mass.get("temporal_res", 1), S)
    lens = _per_sim(mass["edge_bc_length"], S)
    for g in range(S):
        rows = torch.as_tensor(mass["node_bc"][g], dtype=torch.long, device=pred.device).reshape(-1)
        h = pred[rows, 0, :].double()                                  # [n_BC, T]
        corr = (area[rows].double()[:, None] * (h[:, 1:] - h[:, :-1])).sum(0)
        bc = torch.as_tensor(mass["bc"][g]).to(pred.device, torch.float64)
        if bc.dim() == 1:
            bc = bc[None]
        if bc.shape[-1] < T + 1:
            raise ValueError("mass['bc'] needs T + 1 time entries per BC cell")
        q = 0.5 * (bc[:, 1:T] + bc[:, 2:T + 1])                       # [n_BC, T-1]
        L_bc = torch.as_tensor(lens[g], dtype=torch.float64, device=pred.device).reshape(-1, 1)
        inflow = (q * L_bc).sum(0) * (60.0 * float(torch.as_tensor(tres[g])))
        res[g] = (dv[g] - inflow - corr) / 1e6
    return res.float()
