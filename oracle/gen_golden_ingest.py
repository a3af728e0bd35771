"""Golden fixture of the reference's DATASET INGEST (test infrastructure only).

Runs only in the build container, where /root/reference exists:

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden_ingest.py

Raw simulations in the format of the reference's pickled datasets (what
database/graph_creation.py writes and utils/load.py:19-38 unpickles: a PyG ``Data`` per
simulation with WD / VX / VY [N, T_raw] maps, DEM, area, face_distance, edge_slope, slopes, a
hydrograph BC [n_BC, T_raw, 2], node_BC, type_BC, edge_BC_length, a ``MultiscaleMesh`` and
the node_ptr / edge_ptr / intra-edge arrays) are built from the synthetic mesh generator
(mswegnn.mesh) -- the real datasets are not in the container.  The REFERENCE's own pipeline
then prepares them exactly as main.py / test_model.py do with config.yaml's dataset section:
``get_scalers`` (utils/scaling.py:112-141, per-scale standard scalers of area and edge
length), ``create_data_attr`` (utils/dataset.py:232-289), ``to_temporal_dataset``
(utils/dataset.py:410-477, previous_t 3, rollout_steps -1 = the test horizon), and the
reference's ``rollout_test`` runs its MSGNN (K4_F32 checkpoint) on each ingested sample and
on a 2-graph PyG Batch of them.  The fixture (tests/golden/fx_ingest.npz) holds the ingested
model inputs and the reference's rollouts; the oracle restatement is checked against them
here (bit-identical) and by tests/test_oracle_golden.py, the HIP engine by
tests/test_gpu_parity.py::test_ingested_dataset_vs_reference.  No reference source is copied.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path[:0] = [os.path.join(ROOT, "oracle", "refstubs"), REF]
sys.dont_write_bytecode = True

from torch_geometric.data import Data, Batch  # noqa: E402  (stand-ins: PyG is absent)
from database.graph_creation import MultiscaleMesh  # noqa: E402
from utils.scaling import get_scalers  # noqa: E402  (the reference's modules from here on)
from utils.dataset import create_data_attr, to_temporal_dataset  # noqa: E402
from training.train import rollout_test  # noqa: E402
import models.gnn as _refgnn  # noqa: E402
assert _refgnn.__file__.startswith(REF), _refgnn.__file__
sys.path += [os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "oracle")]
from mswegnn.mesh import make_multiscale_mesh  # noqa: E402
import msgnn_torch as orc  # noqa: E402
from gen_golden import ref_msgnn, load_ckpt  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
T_RAW = 97            # 96 h of hourly maps
TEMPORAL_RES = 120    # config.yaml dataset_parameters.temporal_res -> 49 maps -> 48 steps
SCALERS = dict(DEM_scaler=None, slope_scaler=None, area_scaler="standard", edge_length_scaler="standard",
               edge_slope_scaler=None, WD_scaler=None, V_scaler=None)        # config.yaml scalers
NODE_FEATURES = dict(slopes=False, slope=False, area=True, DEM=True)          # config.yaml
EDGE_FEATURES = dict(edge_length=True, edge_relative_distance=False, edge_slope=False)
TEMPORAL = dict(previous_t=3, time_start=0, time_stop=-1, rollout_steps=-1)    # test split


def raw_simulation(n_coarse, seed, num_scales=4):
    """One simulation in the pickled-dataset layout: raw (unscaled) attributes."""
    g = make_multiscale_mesh(n_coarse=n_coarse, num_scales=num_scales, seed=seed, T=1)
    rng = np.random.default_rng(seed + 77)
    npt = g.node_ptr.numpy()
    N = int(npt[-1])
    ei = g.edge_index
    # raw face-centre distances per scale (the generator standardises them; undo per scale
    # with a synthetic length scale: scale s cells are 2^(S-1-s) times the finest)
    dist = g.edge_attr[:, 0].double().numpy().copy()
    ept = g.edge_ptr.numpy()
    for s in range(num_scales):
        dist[ept[s]:ept[s + 1]] = 20.0 * 2 ** s * (1.0 + 0.1 * dist[ept[s]:ept[s + 1]])
    dem = g.x[:, 1].double().numpy() + 3.0 + 0.5 * rng.random()
    # dry start, then a smooth inundation spreading from the BC cell over 96 hours
    t = np.arange(T_RAW) / (T_RAW - 1)
    wave = np.clip(1.5 * t[None, :] - 0.02 * (dem[:, None] - dem.min()) - 0.1, 0.0, None)
    wave[:, 0] = 0.0
    vx = 0.3 * wave * rng.uniform(0.5, 1.0, size=(N, 1))
    vy = 0.2 * wave * rng.uniform(0.5, 1.0, size=(N, 1))
    q = 60.0 * np.sin(np.pi * t) ** 2                          # hydrograph discharge [m^3/s]
    bc = np.stack([np.arange(T_RAW) * 3600.0, q], -1)[None]     # [n_BC, T_raw, (time, value)]
    mesh = MultiscaleMesh()
    mesh.num_meshes = num_scales
    f32 = lambda a: torch.tensor(a, dtype=torch.float32)  # noqa: E731  (FloatTensors, as pickled)
    return Data(edge_index=ei.clone(), face_distance=f32(dist),
                edge_slope=torch.zeros(ei.shape[1]), slopex=torch.zeros(N), slopey=torch.zeros(N),
                DEM=f32(dem), area=g.area.float().clone(),
                WD=f32(wave), VX=f32(vx), VY=f32(vy),
                BC=f32(bc), node_BC=g.node_BC.long().clone(), type_BC=torch.tensor(2),
                edge_BC_length=g.edge_BC_length[:1].float().clone(), mesh=mesh,
                node_ptr=g.node_ptr.clone(), edge_ptr=g.edge_ptr.clone(),
                intra_edge_ptr=g.intra_edge_ptr.clone(), intra_mesh_edge_index=g.intra_mesh_edge_index.clone())


def main():
    torch.set_num_threads(8)
    train = [raw_simulation(n, s) for n, s in ((2, 11), (3, 12), (2, 13))]
    test = [raw_simulation(n, s) for n, s in ((3, 21), (2, 22))]
    scalers = get_scalers(train, dict(SCALERS))
    ingested = create_data_attr(test, scalers=scalers, temporal_res=TEMPORAL_RES, device="cpu",
                                **NODE_FEATURES, **EDGE_FEATURES)
    samples = to_temporal_dataset(ingested, **TEMPORAL)
    assert len(samples) == len(test)
    sd = load_ckpt("K4_F32")
    cfg = dict(num_scales=4, hid_features=32, K_list=[4] * 4, mlp_layers=3)
    model = ref_msgnn(cfg, sd)
    P = {k: v.detach().clone() for k, v in model.state_dict().items()}
    ocfg = orc.msgnn_config(num_scales=4, hid_features=32, K=4)
    fx = {}
    keys = ("x", "edge_index", "edge_attr", "edge_ptr", "node_ptr", "intra_mesh_edge_index", "intra_edge_ptr",
            "BC", "node_BC", "y")
    with torch.no_grad():
        for i, smp in enumerate(samples):
            r = rollout_test(model, smp)
            assert r.shape == (smp.x.shape[0], 2, smp.y.shape[-1]), r.shape
            ro = orc.rollout(P, ocfg, smp, smp.y.shape[-1])
            assert torch.equal(ro, r), f"oracle != reference on ingested sample {i}"
            for k in keys:
                v = getattr(smp, k)
                fx[f"s{i}_{k}"] = v.numpy() if k != "y" else np.zeros(0)
            fx[f"s{i}_T"] = np.array(smp.y.shape[-1])
            fx[f"s{i}_type_BC"] = np.array(int(smp.type_BC))
            fx[f"s{i}_rollout"] = r.numpy()
        # the reference's batched path (PyG Batch -> adapt_batch_training) over both samples
        b = Batch.from_data_list(samples)
        rb = rollout_test(model, b)
        fx["batch_rollout"] = rb.numpy()
    fx["num_samples"] = np.array(len(samples))
    np.savez_compressed(os.path.join(OUT, "fx_ingest.npz"), **fx)
    mpath = os.path.join(OUT, "manifest.json")
    man = json.load(open(mpath))
    man["fx_ingest"] = {
        "generator": "oracle/gen_golden_ingest.py", "cpu": man.get("cpu"),
        "pipeline": "utils.scaling.get_scalers -> utils.dataset.create_data_attr -> to_temporal_dataset "
                    "(config.yaml dataset / scalers / features, rollout_steps -1) -> training.train.rollout_test",
        "checkpoint": "K4_F32", "raw_time_maps": T_RAW, "temporal_res": TEMPORAL_RES,
        "samples": [{"n_coarse": n, "seed": s} for n, s in ((3, 21), (2, 22))]}
    json.dump(man, open(mpath, "w"), indent=1)
    print("fx_ingest:", {k: v.shape for k, v in fx.items() if k.endswith(("_x", "_rollout"))})


if __name__ == "__main__":
    main()
