"""Which HIP layer call moves the zenodo4 training gradient away from the reference's?  (diagnostic)

The reference's training_step on the zenodo4 fixture (tests/golden/fx_grad_train_zenodo4) with
the drop-in's torch path everywhere EXCEPT the listed SWEGNN calls (by order of call in one
rollout step; --mlp / --pool: the make_mlp stacks / mean pooling too), which run on the HIP
training kernels.  One JSON line per selection: loss, global relative L2 error of every
parameter gradient against the reference's fp32 and fp64 results, the worst tensors.

    python tools/grad_ablate_diag.py [--R 1] [--each] [--mlp] [--pool]
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
    ap.add_argument("--R", type=int, default=1)
    ap.add_argument("--calls", type=int, default=10, help="SWEGNN calls per forward (4 scales: 10)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from models.gnn import SWEGNN, MSGNN
    fx = gc.golden("fx_grad_train_zenodo4")
    orig = SWEGNN.forward
    sel = {"swegnn": set(), "model": "torch"}
    count = [0]

    def fwd(self, x_s, x_d, edge_index, edge_attr=None):
        k = count[0] % a.calls
        count[0] += 1
        old = self.train_engine
        self.train_engine = "auto" if k in sel["swegnn"] else "torch"
        try:
            return orig(self, x_s, x_d, edge_index, edge_attr)
        finally:
            self.train_engine = old
    SWEGNN.forward = fwd
    orig_te = MSGNN.train_engine
    runs = [("none", set(), "torch"), ("all_swegnn", set(range(a.calls)), "torch"),
            ("mlp_pool_only", set(), "auto"), ("all", set(range(a.calls)), "auto")]
    runs += [(f"swegnn_{k}", {k}, "torch") for k in range(a.calls)]
    try:
        for label, calls, model_te in runs:
            sel["swegnn"] = calls
            MSGNN.train_engine = model_te
            count[0] = 0
            ours, _ = gc.zenodo4_training_step_case(dev, a.R)
            p, p64 = f"R{a.R}__", f"R{a.R}_fp64__"
            errs = gc.compare(ours, fx, p)
            top = sorted(errs.items(), key=lambda kv: -kv[1])[:4]
            print(json.dumps({"hip": label, "R": a.R, "loss": float(ours["loss"]),
                              "global_vs_fp32": gc.global_rel(ours, fx, p),
                              "global_vs_fp64": gc.global_rel(ours, fx, p64), "worst_vs_fp32": top}), flush=True)
    finally:
        SWEGNN.forward = orig
        MSGNN.train_engine = orig_te


if __name__ == "__main__":
    main()
