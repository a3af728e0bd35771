"""sha256 of a rollout's output bytes under the library this process loads.

Run once per library (MSW_LIB_VARIANT=<name> selects lib/libmswegnn_<name>.so) to compare a
build variant with the default bit for bit:
    python tools/rollout_digest.py --mesh dk15 --T 3 [--eh-loop]
Prints one JSON line {"mesh", "T", "variant", "sha256", "max_abs", "kernels_per_step"}.
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mesh", default="dk15")
    ap.add_argument("--T", type=int, default=3)
    ap.add_argument("--eh-loop", action="store_true", help="force the grid-stride edge hops (MSW_EH_LOOP=1)")
    ap.add_argument("--hid", type=int, default=32, help="hidden width F (32: K4_F32 weights; else seeded init)")
    a = ap.parse_args()
    if a.eh_loop:
        os.environ["MSW_EH_LOOP"] = "1"
    import torch
    from conftest import build_msgnn, weights
    from mswegnn.engine import EnginePlan
    from mswegnn.mesh import make_multiscale_mesh, mesh_config, wet_state
    dev = torch.device("cuda:0")
    g = wet_state(make_multiscale_mesh(**mesh_config(a.mesh), T=a.T), seed=4).to(dev)
    S = mesh_config(a.mesh)["num_scales"]
    if a.hid == 32:
        m = build_msgnn(S, 32, 4, state=weights("K4_F32" if S == 4 else "msgnn3_F32_seed666")).to(dev)
    else:
        m = build_msgnn(S, a.hid, 4).to(dev)
    plan = EnginePlan(m, g, dev)
    out = plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, a.T)
    torch.cuda.synchronize()
    y = out.detach().cpu().contiguous()
    st = plan.stats() if hasattr(plan, "stats") else {}
    plan.close()
    print(json.dumps({"mesh": a.mesh, "T": a.T, "hid": a.hid, "variant": os.environ.get("MSW_LIB_VARIANT", ""),
                      "eh_loop": a.eh_loop, "sha256": hashlib.sha256(y.numpy().tobytes()).hexdigest(),
                      "max_abs": float(y.abs().max()), "kernels_per_step": st.get("kernels_per_step")}))


if __name__ == "__main__":
    main()
