"""One SWEGNN call of the zenodo4 training step, HIP against the torch path on identical inputs
(diagnostic): forward output and every gradient, exact-zero patterns, worst rows.

Records call --call's inputs and output gradient from the training step of
tests/golden/fx_grad_train_zenodo4 run on the torch path (--record torch) or the HIP path
(--record hip), then runs that call alone through the HIP kernels and through the torch path
(fp32 and fp64) with the same inputs and output gradient.

    python tools/grad_call_diag.py [--call 4] [--record torch] [--R 1]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--call", type=int, default=4)
    ap.add_argument("--record", default="torch", choices=["torch", "hip"])
    ap.add_argument("--R", type=int, default=1)
    ap.add_argument("--save", default="", help="also save the call's inputs, output gradient and the HIP / torch "
                                              "results here (torch.save) for offline analysis")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from models.gnn import SWEGNN, MSGNN
    calls = []
    orig = SWEGNN.forward

    def rec_fwd(self, x_s, x_d, edge_index, edge_attr=None):
        k = len(calls)
        y = orig(self, x_s, x_d, edge_index, edge_attr)
        r = {"layer": self, "args": [t.detach().clone() if t is not None else None for t in (x_s, x_d, edge_index, edge_attr)]}
        calls.append(r)
        if k == a.call and y.requires_grad:
            y.register_hook(lambda g: r.__setitem__("dout", g.detach().clone()))
        return y
    SWEGNN.forward = rec_fwd
    te = MSGNN.train_engine
    try:
        gc.zenodo4_training_step_case(dev, a.R, engine="torch" if a.record == "torch" else "auto")
    finally:
        SWEGNN.forward = orig
        MSGNN.train_engine = te
    r = calls[a.call]

    def run(engine, dtype):
        lay = copy.deepcopy(r["layer"]).to(dtype)
        lay.train_engine = engine
        lay.zero_grad(set_to_none=True)
        ins = [t.detach().clone().to(dtype).requires_grad_(True) if t is not None and t.is_floating_point() else t
               for t in r["args"]]
        keep = [t.detach().clone() if t is not None else None for t in ins]
        dout = r["dout"].detach().clone().to(dtype)
        dkeep = dout.clone()
        y = lay(*ins)
        y.backward(dout)
        for i, (t, k0) in enumerate(zip(ins, keep)):  # no kernel may write its inputs
            if t is not None and not torch.equal(t.detach(), k0):
                print(json.dumps({"engine": engine, "input_modified": i,
                                  "rows": int((t.detach() != k0).any(-1).sum()) if t.dim() == 2 else -1}), flush=True)
        if not torch.equal(dout, dkeep):
            print(json.dumps({"engine": engine, "dout_modified": int((dout != dkeep).any(-1).sum())}), flush=True)
        out = {"out": y.detach().double()}
        for name, t in (("d_x_s", ins[0]), ("d_x_d", ins[1])):
            out[name] = t.grad.double() if t.grad is not None else torch.zeros_like(t, dtype=torch.float64)
        if ins[3] is not None and ins[3].grad is not None:
            out["d_edge_attr"] = ins[3].grad.double()
        out.update({"g__" + n: p.grad.double() for n, p in lay.named_parameters() if p.grad is not None})
        return out
    hip, t32, t64 = run("auto", torch.float32), run("torch", torch.float32), run("torch", torch.float64)
    res = {}
    for k in t64:
        h, t, e = hip[k], t32[k], t64[k]
        den = e.abs().max().item() or 1.0
        d_h = (h - e).abs()
        rec = {"hip_vs_fp64": d_h.max().item() / den, "t32_vs_fp64": (t - e).abs().max().item() / den,
               "hip_vs_t32": (h - t).abs().max().item() / den}
        if h.dim() == 2:
            zh, zt = (h == 0).all(1), (t == 0).all(1)
            rec["zero_rows_hip"], rec["zero_rows_t32"] = int(zh.sum()), int(zt.sum())
            rec["zero_row_mismatch"] = int((zh != zt).sum())
            i = int(d_h.amax(1).argmax())
            rec["worst_row"] = [i, h[i].abs().max().item(), e[i].abs().max().item()]
        res[k] = rec
    if a.save:
        torch.save({"args": [t.cpu() if t is not None else None for t in r["args"]], "dout": r["dout"].cpu(),
                    "state": {k: v.cpu() for k, v in r["layer"].state_dict().items()},
                    "hip": {k: v.cpu() for k, v in hip.items()}, "t32": {k: v.cpu() for k, v in t32.items()}}, a.save)
    print(json.dumps({"call": a.call, "record": a.record, "rows": int(r["args"][1].shape[0]),
                      "edges": int(r["args"][2].shape[1]), "x_d_zero_rows": int((r["args"][1] == 0).all(1).sum()),
                      "dout_zero_rows": int((r["dout"] == 0).all(1).sum()), "tensors": res}), flush=True)


if __name__ == "__main__":
    main()
