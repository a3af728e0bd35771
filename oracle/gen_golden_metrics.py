"""Golden vectors for the on-device rollout metrics, made by the REFERENCE's
own evaluation functions (test infrastructure only; runs where /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden_metrics.py

Inputs: two rollouts of the same synthetic multi-scale mesh from tests/golden
(fx_small_K4_F32_rollout48 = "real", fx_small_K2_F16_rollout48 = "predicted"), restricted
to the finest scale as SpatialAnalysis does (utils/miscellaneous.py:311-330,
create_scale_mask == 0), plus a 2-simulation stack.  Outputs: the reference's
get_rollout_loss (RMSE / MAE, all nodes and only_where_water), get_CSI and get_F1 at
0.05 and 0.3 m (utils/miscellaneous.py:123-199, training/loss.py:8-35), and
get_mass_conservation_loss (utils/miscellaneous.py:116-121 -> training/loss.py:120-169 ->
utils/dataset.py:577-591) on the mesh's raw cell areas, BC edge length and the hydrograph.
Writes tests/golden/fx_metrics.npz; no reference source is copied.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path[:0] = [os.path.join(ROOT, "oracle", "refstubs"), REF]
sys.dont_write_bytecode = True

from utils.miscellaneous import get_rollout_loss, get_CSI, get_F1, get_mass_conservation_loss  # noqa: E402
from torch_geometric.data import Data  # noqa: E402  (oracle/refstubs attribute bag)


def main():
    g = os.path.join(ROOT, "tests", "golden")
    real = torch.from_numpy(np.load(os.path.join(g, "fx_small_K4_F32_rollout48.npz"))["rollout"])
    pred = torch.from_numpy(np.load(os.path.join(g, "fx_small_K2_F16_rollout48.npz"))["rollout"])
    out = {}  # inputs: the two rollout fixtures named above
    # finest scale only (SpatialAnalysis: create_scale_mask == 0 -> rows [0, node_ptr[1]))
    sys.path.insert(0, os.path.join(ROOT, "mswe-gnn_amd"))
    from mswegnn.mesh import make_multiscale_mesh, mesh_config
    mesh = make_multiscale_mesh(**mesh_config("small"), T=48)
    n0 = int(mesh.node_ptr[1])
    out["n0"] = np.array(n0)
    rf, pf = real[:n0], pred[:n0]
    for tl in ("RMSE", "MAE"):
        out[f"loss_{tl}"] = get_rollout_loss(pf, rf, type_loss=tl).numpy()
        out[f"loss_{tl}_water"] = get_rollout_loss(pf, rf, type_loss=tl, only_where_water=True).numpy()
    for thr in (0.05, 0.3):
        out[f"csi_{thr}"] = get_CSI(pf, rf, water_threshold=thr).numpy()
        out[f"f1_{thr}"] = get_F1(pf, rf, water_threshold=thr).numpy()
    # two simulations stacked ([S, N, 2, T] branch of the same functions)
    p2, r2 = torch.stack([pf, rf.flip(-1)]), torch.stack([rf, pf])
    out["loss_RMSE_stack"] = get_rollout_loss(p2, r2, type_loss="RMSE").numpy()
    out["csi_0.05_stack"] = get_CSI(p2, r2, water_threshold=0.05).numpy()
    # mass conservation: rollout of the finest scale, raw BC = the newest column of the
    # sliding BC window ([n_BC, T+1]), the finest BC edge length, temporal_res minutes
    bc_raw = mesh.BC[:, -1, :].clone()
    data = Data(area=mesh.area.clone(), node_ptr=mesh.node_ptr.clone(), BC=bc_raw,
                node_BC=mesh.node_BC.long().clone(), edge_BC_length=mesh.edge_BC_length[:1].clone(),
                temporal_res=mesh.temporal_res.clone())
    out["mass_area"] = mesh.area.numpy()
    out["mass_bc"] = bc_raw.numpy()
    out["mass_edge_bc_length"] = mesh.edge_BC_length[:1].numpy()
    out["mass_temporal_res"] = mesh.temporal_res.numpy()
    out["mass_node_bc"] = mesh.node_BC.numpy()
    out["mass_loss_pred"] = get_mass_conservation_loss(pf.clone(), data.clone()).numpy()
    out["mass_loss_real"] = get_mass_conservation_loss(rf.clone(), data.clone()).numpy()
    np.savez_compressed(os.path.join(g, "fx_metrics.npz"), **out)
    print({k: np.asarray(v).shape for k, v in out.items()})


if __name__ == "__main__":
    main()
