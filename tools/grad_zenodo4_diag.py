"""Training gradients at BASELINE config 2's size against the reference's own (diagnostic).

The reference's training_step on the zenodo4 mesh (tests/golden/fx_grad_train_zenodo4.npz,
oracle/gen_golden_grad.py: K4_F32, one-graph batch, R = 1..4 rollout steps, fp32 and fp64)
recomputed on this GPU by the HIP training kernels ('auto') and by the drop-in's torch path
('torch'): per R the loss, the global relative L2 error of every parameter gradient against the
reference's fp32 and fp64 results, the worst tensor, and the cells where _mask_small_WD decides
differently from the fp64 run (grad_cases.mask_forks).  One JSON line per (engine, R).

    python tools/grad_zenodo4_diag.py [--engines auto,torch] [--R 1,2,3,4]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import grad_cases as gc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engines", default="auto,torch")
    ap.add_argument("--R", default="1,2,3,4")
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args()
    dev = torch.device(a.device)
    fx = gc.golden("fx_grad_train_zenodo4")
    for engine in a.engines.split(","):
        for R in (int(r) for r in a.R.split(",")):
            pre = []
            ours, _ = gc.zenodo4_training_step_case(dev, R, engine=engine, premask=pre)
            p, p64 = f"R{R}__", f"R{R}_fp64__"
            errs = gc.compare(ours, fx, p)
            errs64 = gc.compare(ours, fx, p64)
            ref32 = {k[len(p):]: torch.from_numpy(v) for k, v in fx.items() if k.startswith(p + "g__")}
            worst = max(errs, key=errs.get)
            worst64 = max(errs64, key=errs64.get)
            rec = {"engine": engine, "R": R, "loss": float(ours["loss"]), "loss_ref": float(fx[p + "loss"]),
                   "global_vs_ref_fp32": gc.global_rel(ours, fx, p),
                   "global_vs_ref_fp64": gc.global_rel(ours, fx, p64),
                   "ref_fp32_vs_fp64": gc.global_rel(ref32, fx, p64),
                   "worst_vs_fp32": [worst, errs[worst]], "worst_vs_fp64": [worst64, errs64[worst64]],
                   "ref_fp32_worst_vs_fp64": max(gc.compare(ref32, fx, p64, keys=list(ref32)).values())}
            if R == 4:
                rec["mask_forks_vs_fp64"] = gc.mask_forks(pre, fx)[:20]
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
