"""Which layer call carries a training-gradient error at zenodo4 size?  (diagnostic)

Runs the reference's training_step on the zenodo4 fixture (tests/golden/fx_grad_train_zenodo4,
grad_cases.zenodo4_training_step_case) with the HIP training kernels, recording every SWEGNN
layer call's inputs and the gradient arriving at its output.  Each call is then replayed alone
with that same output gradient three ways -- HIP fp32, the drop-in's torch path in fp32, and
the torch path in float64 (exact-arithmetic yardstick) -- and per parameter / input the
max-abs relative error of HIP and of torch fp32 against float64 is printed (one JSON line per
call).  Also the make_mlp calls (encoders, decoder) the same way.

    python tools/grad_layer_diag.py [--R 1]
"""
import argparse
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import grad_cases as gc  # noqa: E402
from conftest import rel_err  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=1)
    ap.add_argument("--all", action="store_true", help="every tensor (default: those where HIP > 1e-5)")
    ap.add_argument("--hip-calls", default="all",
                    help="SWEGNN calls (by order in the forward) on the HIP kernels in the recorded run, "
                         "the others and every make_mlp / pooling on the torch path; 'all' = the HIP path")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from models.gnn import SWEGNN
    import models.gnn as mg
    calls = []
    orig_fwd = SWEGNN.forward

    hip_calls = None if a.hip_calls == "all" else {int(c) for c in a.hip_calls.split(",") if c}

    def recording(self, x_s, x_d, edge_index, edge_attr=None):
        old = self.train_engine
        if hip_calls is not None:
            self.train_engine = "auto" if len(calls) in hip_calls else "torch"
        try:
            y = orig_fwd(self, x_s, x_d, edge_index, edge_attr)
        finally:
            self.train_engine = old
        rec = {"layer": self, "args": [t.detach().clone() if t is not None else None
                                       for t in (x_s, x_d, edge_index, edge_attr)]}
        calls.append(rec)
        if y.requires_grad:
            y.register_hook(lambda g, rec=rec: rec.__setitem__("dout", g.detach().clone()))
        return y
    SWEGNN.forward = recording
    mlp_calls = []
    orig_mlp = mg._mlp_call

    def mlp_recording(owner, seq, x):
        y = orig_mlp(owner, seq, x)
        rec = {"layer": seq, "args": [x.detach().clone()]}
        mlp_calls.append(rec)
        if y.requires_grad:
            y.register_hook(lambda g, rec=rec: rec.__setitem__("dout", g.detach().clone()))
        return y
    mg._mlp_call = mlp_recording
    from models.gnn import MSGNN
    orig_te = MSGNN.train_engine
    if hip_calls is not None:
        MSGNN.train_engine = "torch"
    try:
        gc.zenodo4_training_step_case(dev, a.R)
    finally:
        SWEGNN.forward = orig_fwd
        mg._mlp_call = orig_mlp
        MSGNN.train_engine = orig_te

    def run(layer, args, dout, engine, dtype, mlp=False):
        lay = copy.deepcopy(layer).to(dtype)
        lay.zero_grad(set_to_none=True)
        ins = [t.to(dtype).requires_grad_(True) if t is not None and t.is_floating_point() else t for t in args]
        if mlp:
            y = mg._mlp_call(_Owner(engine), lay, ins[0])
        else:
            lay.train_engine = engine
            y = lay(*ins)
        y.backward(dout.to(dtype))
        out = {"out": y.detach()}
        for i, t in enumerate(ins):
            if t is not None and t.is_floating_point():
                out[f"d_in{i}"] = t.grad
        out.update({"g__" + n: p.grad for n, p in lay.named_parameters() if p.grad is not None})
        return out

    class _Owner:
        def __init__(self, engine):
            self.train_engine = engine

    for kind, lst in (("swegnn", calls), ("mlp", mlp_calls)):
        for i, rec in enumerate(lst):
            if "dout" not in rec:
                continue
            mlp = kind == "mlp"
            hip = run(rec["layer"], rec["args"], rec["dout"], "auto", torch.float32, mlp)
            t32 = run(rec["layer"], rec["args"], rec["dout"], "torch", torch.float32, mlp)
            t64 = run(rec["layer"], rec["args"], rec["dout"], "torch", torch.float64, mlp)
            res = {}
            for k in t64:
                if t64[k] is None or hip.get(k) is None or t32.get(k) is None:
                    continue
                eh, et = rel_err(hip[k], t64[k]), rel_err(t32[k], t64[k])
                if a.all or eh > 1e-5:
                    res[k] = [eh, et]
            print(json.dumps({"kind": kind, "call": i, "rows": int(rec["args"][1 if not mlp else 0].shape[0]),
                              "edges": int(rec["args"][2].shape[1]) if not mlp else None,
                              "dout_nonzero_rows": int((rec["dout"].abs().sum(1) > 0).sum()),
                              "hip_vs_fp64__torch32_vs_fp64": res}), flush=True)


if __name__ == "__main__":
    main()
