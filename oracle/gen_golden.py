"""Generate golden fixtures by running the REFERENCE itself (test infrastructure only).

Runs only in the build container, where /root/reference exists:

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden.py

It puts oracle/refstubs (sys.modules stand-ins for the absent torch_geometric /
lightning / wandb / database packages) and /root/reference on
sys.path, builds the reference's own MSGNN / GNN modules (models/gnn.py), loads the
shipped checkpoints with ``torch.load(weights_only=True)`` and runs the reference's own
``training.train.rollout_test`` on the synthetic meshes of mswegnn.mesh.  Outputs are
small .npz fixtures under tests/golden/ (inputs + expected outputs + exported weights);
no reference source is copied.  The oracle restatement (oracle/msgnn_torch.py) is checked
against the same outputs here as a first sanity gate; tests/test_oracle_golden.py repeats
that check without the reference.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
# Only the stand-ins and the reference on the path while the reference's modules import:
# its models/ has no __init__.py (a namespace package), so the drop-in's regular ``models``
# package would win from ANY position on sys.path.
sys.path[:0] = [os.path.join(ROOT, "oracle", "refstubs"), REF]
sys.dont_write_bytecode = True

from models.gnn import MSGNN, GNN  # noqa: E402  (the reference's modules)
from training.train import rollout_test  # noqa: E402
import models.gnn as _refgnn  # noqa: E402
assert _refgnn.__file__.startswith(REF), _refgnn.__file__
sys.path += [os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "oracle")]
from mswegnn.mesh import make_multiscale_mesh, make_single_scale_mesh, wet_state, mesh_config  # noqa: E402
import msgnn_torch as orc  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
os.makedirs(OUT, exist_ok=True)
torch.set_num_threads(8)
manifest = {}


def graph_digest(g):
    h = hashlib.sha256()
    for k in ("x", "edge_index", "edge_attr", "edge_ptr", "node_ptr", "intra_mesh_edge_index",
              "intra_edge_ptr", "BC", "node_BC"):
        if k in g.keys():
            h.update(np.ascontiguousarray(getattr(g, k).numpy()).tobytes())
    return h.hexdigest()


def load_ckpt(name):
    sd = torch.load(f"{REF}/results/Pareto_front/models/{name}.h5", map_location="cpu",
                    weights_only=True)["state_dict"]
    return {k[len("model."):]: v for k, v in sd.items() if k.startswith("model.")}


def ref_msgnn(cfg, sd=None):
    m = MSGNN(num_node_features=8, num_edge_features=1, num_scales=cfg["num_scales"],
              hid_features=cfg["hid_features"], K=cfg["K_list"][:cfg["num_scales"]],
              mlp_layers=cfg["mlp_layers"], seed=666, learned_residuals=True,
              mlp_activation="prelu", gnn_activation="tanh", edge_mlp=True, normalize=True,
              with_filter_matrix=True, with_gradient=True, with_WL=True, learned_pooling=False,
              skip_connections=True, previous_t=3)
    if sd is not None:
        m.load_state_dict(sd, strict=True)
    return m.eval()


def ref_gnn(cfg):
    m = GNN(num_node_features=8, num_edge_features=1, hid_features=cfg["hid_features"],
            K=cfg["K"], n_GNN_layers=cfg["n_GNN_layers"], mlp_layers=cfg["mlp_layers"],
            previous_t=3, learned_residuals=True, seed=42)
    return m.eval()


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: (v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v))
                                 for k, v in arrays.items()})
    manifest[name] = {k: list(np.asarray(v).shape) for k, v in arrays.items()}
    print(f"  wrote {name}.npz ({os.path.getsize(path) / 1e3:.0f} kB)")


def save_weights(name, model):
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    save("weights_" + name, **sd)
    return sd


def check_oracle(P, cfg, g, ref_out, steps=None, label=""):
    with torch.no_grad():
        o = orc.rollout(P, cfg, g, steps) if steps else orc.forward(P, cfg, g)
    d = (o - ref_out).abs().max().item()
    print(f"  oracle vs reference [{label}]: max|diff| = {d:.3e}")
    assert d == 0.0, "oracle restatement is not bit-identical to the reference"


def hooks(model, names):
    store = {}
    hs = []
    for n in names:
        mod = model.get_submodule(n)
        hs.append(mod.register_forward_hook(lambda m, i, o, n=n: store.__setitem__(n, o.detach().clone())))
    return store, hs


def main():
    t0 = time.time()
    # ------------------------------------------------------------ 4-scale checkpoints
    for ck in ("K4_F32", "K2_F16"):
        K = int(ck[1]); F = int(ck.split("_F")[1])
        cfg = orc.msgnn_config(num_scales=4, hid_features=F, K=K)
        model = ref_msgnn(cfg, load_ckpt(ck))
        P = save_weights(ck, model)
        manifest["weights_" + ck + "_cfg"] = cfg

        # single forward on a wet state + per-stage intermediates (tiny mesh)
        g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), T=48), seed=1)
        names = (["edge_encoder", "static_node_encoder", "dynamic_node_encoder"]
                 + [f"gnn_processor.{j}" for j in range(7)] + [f"intra_scale_gnn.{j}" for j in range(3)]
                 + ["node_decoder"])
        store, hs = hooks(model, names)
        with torch.no_grad():
            y = model(g)
        for h in hs:
            h.remove()
        check_oracle(P, cfg, g, y, label=f"{ck} tiny wet step")
        save(f"fx_tiny_{ck}_step", x=g.x, y=y, digest=np.frombuffer(bytes.fromhex(graph_digest(g)), np.uint8),
             **{"mid__" + k.replace(".", "_"): v for k, v in store.items()})

        # 48-step dry-start rollouts (small mesh)
        g = make_multiscale_mesh(**mesh_config("small"), T=48)
        with torch.no_grad():
            r = rollout_test(model, g)
        check_oracle(P, cfg, g, r, steps=48, label=f"{ck} small rollout48")
        save(f"fx_small_{ck}_rollout48", rollout=r, digest=np.frombuffer(bytes.fromhex(graph_digest(g)), np.uint8))
        print(f"  {ck}: max h over rollout {r[:, 0].max():.3f}, wet cells at T: {(r[:, 0, -1] > 0).sum().item()}")

    # ------------------------------------------------------------ config-2 size (K4_F32)
    cfg = orc.msgnn_config(num_scales=4, hid_features=32, K=4)
    model = ref_msgnn(cfg, load_ckpt("K4_F32"))
    g = make_multiscale_mesh(**mesh_config("zenodo4"), T=48)
    t = time.time()
    with torch.no_grad():
        r = rollout_test(model, g)
    print(f"  zenodo4 reference rollout48: {time.time() - t:.2f} s (8 threads)")
    sel = np.arange(48)  # every step (the bench times all of them)
    save("fx_zenodo4_K4_F32_rollout48", steps=sel, rollout_sel=r[..., sel].contiguous(),
         digest=np.frombuffer(bytes.fromhex(graph_digest(g)), np.uint8))
    manifest["zenodo4_ref_seconds_8thr"] = time.time() - t

    # ------------------------------------------------------------ config 4: dk15-like, 200 steps
    g = make_multiscale_mesh(**mesh_config("dk15"), T=200)
    t = time.time()
    with torch.no_grad():
        r = rollout_test(model, g)
    print(f"  dk15 reference rollout200: {time.time() - t:.2f} s (8 threads)")
    sel = np.array(sorted(set(range(0, 200, 20)) | set(range(19, 200, 20))))
    save("fx_dk15_K4_F32_rollout200", steps=sel, rollout_sel=r[..., sel].contiguous(),
         digest=np.frombuffer(bytes.fromhex(graph_digest(g)), np.uint8))
    manifest["dk15_ref_seconds_8thr"] = time.time() - t

    # ------------------------------------------------------------ 3-scale MSGNN, seeded init
    cfg = orc.msgnn_config(num_scales=3, hid_features=32, K=4)
    model = ref_msgnn(cfg)
    P = save_weights("msgnn3_F32_seed666", model)
    manifest["weights_msgnn3_F32_seed666_cfg"] = cfg
    g = wet_state(make_multiscale_mesh(**mesh_config("small3"), T=6), seed=3)
    with torch.no_grad():
        y = model(g)
        r = rollout_test(model, g)
    check_oracle(P, cfg, g, y, label="msgnn3 wet step")
    check_oracle(P, cfg, g, r, steps=6, label="msgnn3 wet rollout6")
    save("fx_small3_msgnn3_wet", x=g.x, y=y, rollout=r,
         digest=np.frombuffer(bytes.fromhex(graph_digest(g)), np.uint8))

    # ------------------------------------------------------------ 1-scale GNN (config 1)
    cfg = orc.gnn_config(hid_features=32, K=2, n_GNN_layers=2, mlp_layers=1)
    model = ref_gnn(cfg)
    P = save_weights("gnn_F32_seed42", model)
    manifest["weights_gnn_F32_seed42_cfg"] = cfg
    g = wet_state(make_single_scale_mesh(n_coarse=3, refinements=3, T=10), seed=2)
    with torch.no_grad():
        y = model(g)
        r = rollout_test(model, g)
    check_oracle(P, cfg, g, y, label="gnn wet step")
    check_oracle(P, cfg, g, r, steps=10, label="gnn rollout10")
    save("fx_gnn_small_rollout10", x=g.x, y=y, rollout=r,
         digest=np.frombuffer(bytes.fromhex(graph_digest(g)), np.uint8))

    gen_batches()
    gen_variants()

    manifest["cpu"] = cpu_model()
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, default=str)
    print(f"done in {time.time() - t0:.1f} s")


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# Batched rollouts: heterogeneous meshes collated as a PyG Batch
# (oracle/refstubs/torch_geometric/data: PyG's collation restated) and run through the
# reference's own rollout_test -> adapt_batch_training -> update_batch_multiscale
# (training/train.py:14-95).  Each member is described by the arguments that regenerate it.
BATCHES = {
    # 4-scale, shipped K4_F32 checkpoint: three meshes of two sizes, one wet start
    "fx_batch_K4_F32": dict(kind="msgnn", S=4, F=32, K=4, ckpt="K4_F32", T=12, members=[
        dict(n_coarse=2, seed=11, wet=None), dict(n_coarse=3, seed=12, wet=5),
        dict(n_coarse=2, seed=13, wet=None)]),
    # 3-scale, seeded init (msgnn3 weights): two sizes, wet starts
    "fx_batch_msgnn3": dict(kind="msgnn", S=3, F=32, K=4, ckpt=None, T=6, members=[
        dict(n_coarse=5, seed=21, wet=6), dict(n_coarse=6, seed=22, wet=7)]),
    # 1-scale GNN (config 1 model): the single-scale branch of adapt_batch_training
    "fx_batch_gnn": dict(kind="gnn", T=5, members=[
        dict(n_coarse=2, seed=31, wet=8), dict(n_coarse=3, seed=32, wet=9)]),
}


def gen_variants():
    """Reference outputs for options no shipped config sets: upwind_mode=True on every
    processor (gnn.py:365,431-432) of the seeded 3-scale MSGNN, wet start."""
    cfg = orc.msgnn_config(num_scales=3, hid_features=32, K=2, upwind_mode=True)
    model = ref_msgnn(dict(cfg, K_list=[2, 2, 2, 2, 2]))
    for p in model.gnn_processor:
        p.upwind_mode = True
    P = {k: v.detach().clone() for k, v in model.state_dict().items()}
    g = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=3, T=4), seed=11)
    with torch.no_grad():
        r = rollout_test(model, g)
    check_oracle(P, cfg, g, r, steps=4, label="msgnn3 K2 upwind rollout4")
    # weights: the seeded init (seed 666), which the drop-in reproduces bit for bit
    save("fx_upwind_msgnn3_K2", rollout=r, digest=np.frombuffer(bytes.fromhex(graph_digest(g)), np.uint8))
    manifest["fx_upwind_msgnn3_K2_cfg"] = cfg


def batch_member(spec, m):
    """The synthetic graph of one batch member (also used by tests/)."""
    if spec["kind"] == "gnn":
        g = make_single_scale_mesh(n_coarse=m["n_coarse"], refinements=3, seed=m["seed"], T=spec["T"])
    else:
        g = make_multiscale_mesh(n_coarse=m["n_coarse"], num_scales=spec["S"], seed=m["seed"], T=spec["T"])
    return wet_state(g, seed=m["wet"]) if m["wet"] is not None else g


def gen_batches():
    from torch_geometric.data import Data, Batch
    from training.train import adapt_batch_training
    for name, spec in BATCHES.items():
        if spec["kind"] == "gnn":
            cfg = orc.gnn_config(hid_features=32, K=2, n_GNN_layers=2, mlp_layers=1)
            model = ref_gnn(cfg)
        else:
            cfg = orc.msgnn_config(num_scales=spec["S"], hid_features=spec["F"], K=spec["K"])
            model = ref_msgnn(cfg, load_ckpt(spec["ckpt"]) if spec["ckpt"] else None)
        P = {k: v.detach().clone() for k, v in model.state_dict().items()}
        gs = [batch_member(spec, m) for m in spec["members"]]
        batch = Batch.from_data_list([Data(**g.__dict__) for g in gs])
        with torch.no_grad():
            r = rollout_test(model, batch)
        temp = adapt_batch_training(batch)
        # the members one by one through the oracle (batching must not change a member)
        ptr = batch.ptr
        for i, g in enumerate(gs):
            with torch.no_grad():
                o = orc.rollout(P, cfg, g, spec["T"])
            d = (r[ptr[i]:ptr[i + 1]] - o).abs().max().item()
            print(f"  {name} member {i}: reference batch vs oracle single max|diff| = {d:.3e}")
        arrays = dict(rollout=r, ptr=ptr, node_BC=temp.node_BC, node_BC_ptr=temp.node_BC_ptr,
                      edge_index=temp.edge_index)
        if spec["kind"] != "gnn":
            arrays.update(node_ptr=temp.node_ptr, edge_ptr=temp.edge_ptr, intra_edge_ptr=temp.intra_edge_ptr,
                          intra_mesh_edge_index=temp.intra_mesh_edge_index, edge_attr=temp.edge_attr)
        arrays["digests"] = np.stack([np.frombuffer(bytes.fromhex(graph_digest(g)), np.uint8) for g in gs])
        save(name, **arrays)
        manifest[name + "_spec"] = spec


if __name__ == "__main__":
    if "--batches-only" in sys.argv or "--variants-only" in sys.argv:  # add to an existing manifest
        with open(os.path.join(OUT, "manifest.json")) as f:
            manifest.update(json.load(f))
        if "--batches-only" in sys.argv:
            gen_batches()
        if "--variants-only" in sys.argv:
            gen_variants()
        with open(os.path.join(OUT, "manifest.json"), "w") as f:
            json.dump(manifest, f, indent=1, default=str)
    else:
        main()
