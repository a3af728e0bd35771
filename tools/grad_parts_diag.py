"""Which HIP training layer kind carries a gradient difference?  The reference fixture's
training_step (tests/golden/fx_grad_train_K4_F32.npz) on the GPU with the HIP training
kernels switched on one layer kind at a time (as tools/train_bench.py --parts does); per
tensor the error against the reference's float64 gradients (max-abs relative), for the
tensors named on the command line (default: every tensor whose error exceeds 1e-4 with all
kinds on).  One JSON line per (set, R, parts).

    python tools/grad_parts_diag.py [--sets b1] [--R 1 4] [tensor names ...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", nargs="+", default=["b1"])
    ap.add_argument("--R", nargs="+", type=int, default=[1, 4])
    ap.add_argument("--all-tensors", action="store_true", help="report every parameter tensor")
    ap.add_argument("--subsets", default="", help="comma list of subsets (default: all of them)")
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    import torch
    import grad_cases as gc
    from conftest import rel_err
    from mswegnn import autograd as ag
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    fx = gc.golden("fx_grad_train_K4_F32")
    orig = (ag.supported, ag.mlp_supported, ag.pool_supported)
    off = lambda *args: False  # noqa: E731
    subsets = {"all": (1, 1, 1), "swegnn": (1, 0, 0), "mlp": (0, 1, 0), "pool": (0, 0, 1), "none": (0, 0, 0),
               "swegnn+mlp": (1, 1, 0), "swegnn+pool": (1, 0, 1), "mlp+pool": (0, 1, 1)}
    if a.subsets:
        subsets = {k: v for k, v in subsets.items() if k in a.subsets.split(",")}
    for sname in a.sets:
        for R in a.R:
            p64 = f"{sname}_R{R}_fp64__"
            names = list(a.names)
            for label, (s, m, p) in subsets.items():
                ag.supported, ag.mlp_supported, ag.pool_supported = (orig[0] if s else off, orig[1] if m else off,
                                                                     orig[2] if p else off)
                ours, _ = gc.training_step_case(dev, sname, R)
                if not names and label == "all":
                    names = [k[len("g__"):] for k in ours if k.startswith("g__") and
                             (a.all_tensors or rel_err(ours[k], torch.from_numpy(fx[p64 + k])) > 1e-4)]
                errs = {n: rel_err(ours["g__" + n], torch.from_numpy(fx[p64 + "g__" + n])) for n in names}
                ref = {n: rel_err(torch.from_numpy(fx[f"{sname}_R{R}__g__{n}"]), torch.from_numpy(fx[p64 + "g__" + n]))
                       for n in names}
                print(json.dumps({"set": sname, "R": R, "hip_parts": label, "loss": float(ours["loss"]),
                                  "loss_ref": float(fx[f"{sname}_R{R}__loss"]), "global_vs_fp64": gc.global_rel(ours, fx, p64),
                                  "tensor_vs_fp64": errs, "reference_fp32_vs_fp64": ref}), flush=True)
    ag.supported, ag.mlp_supported, ag.pool_supported = orig


if __name__ == "__main__":
    main()
