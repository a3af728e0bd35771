"""Training-step throughput of MSGNN on MI355X: the reference's training_step
(training/train.py:125-145: curriculum rollout of R steps, BC write, forward, use_prediction,
per-step RMSE loss, mean) + backward + gradient clipping (main.py: gradient_clip_val=1) +
AdamW step, with every SWEGNN layer on the HIP training kernels (mswegnn/autograd.py) against
the all-torch autograd path of the same drop-in model on the same GPU.  Also reports the loss
and gradient agreement of the two paths at the first step.

    python tools/train_bench.py [--workload zenodo4] [--rollout-steps 4] [--steps 5] [--amp] [--fp64-ref]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mswe-gnn_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def rmse_loss(pred, real, n0, velocity_scaler=1.0):
    """loss_function(type_loss='RMSE', only_where_water=False, conservation=0) on the finest
    scale (training/loss.py:76-118, get_multiscale_loss single graph)."""
    diff = pred[:n0] - real[:n0]
    per_var = torch.sqrt(torch.mean(diff ** 2, 0))
    sc = torch.tensor([1.0, velocity_scaler], device=pred.device, dtype=pred.dtype)
    return torch.dot(per_var, sc) / sc.sum()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="zenodo4")
    ap.add_argument("--rollout-steps", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--only", choices=["hip", "torch"], default=None)
    ap.add_argument("--fp64-ref", action="store_true",
                    help="also the first-step gradients of the torch path in float64 (the yardstick)")
    ap.add_argument("--amp", action="store_true",
                    help="also both paths under main.py's precision='16-mixed' (autocast fp16 + GradScaler)")
    ap.add_argument("--parts", default="swegnn,mlp,pool",
                    help="diagnostics: which layer kinds run on the HIP training kernels")
    a = ap.parse_args()
    from mswegnn import autograd as ag
    parts = set(a.parts.split(","))
    if "mlp" not in parts:
        ag.mlp_supported = lambda *args: False
    if "pool" not in parts:
        ag.pool_supported = lambda *args: False
    if "swegnn" not in parts:
        ag.supported = lambda *args: False
    from mswegnn.rollout import apply_boundary_condition, use_prediction
    dev = torch.device("cuda", 0)
    R = a.rollout_steps
    g, m0, w, desc = bench.build_workload(a.workload, seed=0, T=R + 1)
    g = g.to(dev)
    n0 = desc["fine_nodes"]
    # target: the model's own rollout from a perturbed state (any smooth field will do)
    m0 = m0.to(dev)
    with torch.no_grad():  # a target the model does not already reproduce (well-conditioned RMSE)
        y = (m0.rollout(g, R) * 1.1 + 0.01).detach()
    state0 = {k: v.detach().clone() for k, v in m0.state_dict().items()}

    def run(engine, amp=False):
        """Training steps of one path; amp: main.py's precision='16-mixed' (autocast fp16 around
        the forward + loss, GradScaler, unscale before clipping -- Lightning's order)."""
        from models.gnn import MSGNN  # noqa: F401
        m = m0
        m.load_state_dict(state0)
        m.train()
        m.engine = engine
        opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=0.0)
        scaler = torch.amp.GradScaler("cuda", enabled=amp)
        dyn = m.previous_t * m.NUM_WATER_VARS

        def step():
            opt.zero_grad(set_to_none=True)
            temp = g.clone()
            losses = []
            with torch.autocast("cuda", dtype=torch.float16, enabled=amp):
                for i in range(R):
                    temp.x[:, -dyn:] = apply_boundary_condition(temp.x[:, -dyn:], temp.BC[:, :, i], temp.node_BC,
                                                                type_BC=temp.type_BC)
                    preds = m(temp)
                    temp.x = use_prediction(temp.x, preds, m.previous_t)
                    losses.append(rmse_loss(preds, y[:, :, i], n0))
                loss = torch.stack(losses).mean()
            scaler.scale(loss).backward()
            scaler.unscale_(opt)
            torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
            return loss

        def opt_step():
            scaler.step(opt)
            scaler.update()
        first = step()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
        opt_step()
        for _ in range(a.warmup):
            step()
            opt_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
            opt_step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / max(a.steps, 1), float(first.detach()), grads
    if a.only:
        t, l, _ = run("auto" if a.only == "hip" else "torch")
        print(json.dumps({"only": a.only, "ms_per_training_step": t * 1e3, "first_loss": l}), flush=True)
        return
    t_hip, l_hip, g_hip = run("auto")
    t_torch, l_torch, g_torch = run("torch")
    _, _, g_hip2 = run("auto")      # run-to-run: the HIP path is deterministic (no atomics)
    _, _, g_torch2 = run("torch")   # torch's index_add / scatter use atomics on the GPU

    def per_tensor(a, b):
        return {k: ((a[k] - b[k]).abs().max() / b[k].abs().max().clamp(min=1e-30)).item() for k in b}

    def global_rel(a, b):
        num = sum(((a[k] - b[k]) ** 2).sum() for k in b).sqrt()
        den = sum((b[k] ** 2).sum() for k in b).sqrt()
        return (num / den).item()
    fp64 = None
    if a.fp64_ref:  # exact-arithmetic yardstick: the same first step, torch path, float64
        import copy
        m64 = copy.deepcopy(m0).double()
        m64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in state0.items()})
        m64.train()
        m64.engine = "torch"
        g64 = g.clone()
        for k in ("x", "edge_attr", "BC"):
            setattr(g64, k, getattr(g, k).double())
        y64 = y.double()
        dyn = m64.previous_t * m64.NUM_WATER_VARS
        temp = g64.clone()
        losses = []
        for i in range(R):
            temp.x[:, -dyn:] = apply_boundary_condition(temp.x[:, -dyn:], temp.BC[:, :, i], temp.node_BC,
                                                        type_BC=temp.type_BC)
            preds = m64(temp)
            temp.x = use_prediction(temp.x, preds, m64.previous_t)
            losses.append(rmse_loss(preds, y64[:, :, i], n0))
        torch.stack(losses).mean().backward()
        torch.nn.utils.clip_grad_norm_(m64.parameters(), 1.0)
        g64s = {n: p.grad.detach().float() for n, p in m64.named_parameters() if p.grad is not None}
        fp64 = {"hip_vs_fp64_global_rel": global_rel(g_hip, g64s), "torch_vs_fp64_global_rel": global_rel(g_torch, g64s),
                "hip_vs_fp64_worst_tensor_rel": max(per_tensor(g_hip, g64s).values()),
                "torch_vs_fp64_worst_tensor_rel": max(per_tensor(g_torch, g64s).values())}
    # main.py's training configuration: precision='16-mixed' (autocast fp16 + GradScaler).  The
    # HIP training kernels run under autocast in fp32; torch's own AMP path is the reference's
    amp = None
    if a.amp:
        t_hip_amp, _, g_hip_amp = run("auto", amp=True)
        t_torch_amp, _, g_torch_amp = run("torch", amp=True)
        amp = {"hip_ms_per_training_step": t_hip_amp * 1e3, "torch_amp_ms_per_training_step": t_torch_amp * 1e3,
               "speedup_vs_torch_amp": t_torch_amp / t_hip_amp,
               "hip_amp_vs_hip_fp32_global_rel": global_rel(g_hip_amp, g_hip),
               "torch_amp_vs_torch_fp32_global_rel": global_rel(g_torch_amp, g_torch)}
        if fp64 is not None:
            amp["hip_amp_vs_fp64_global_rel"] = global_rel(g_hip_amp, g64s)
            amp["torch_amp_vs_fp64_global_rel"] = global_rel(g_torch_amp, g64s)
    pt = per_tensor(g_hip, g_torch)
    worst_k = max(pt, key=pt.get)
    print(json.dumps({"workload": a.workload, "fine_nodes": n0, "all_nodes": desc["all_nodes"],
                      "rollout_steps_per_training_step": R, "hip_parts": sorted(parts),
                      "hip_ms_per_training_step": t_hip * 1e3, "torch_ms_per_training_step": t_torch * 1e3,
                      "speedup": t_torch / t_hip,
                      "fine_node_steps_per_s_hip": n0 * R / t_hip,
                      "fine_node_steps_per_s_torch": n0 * R / t_torch,
                      "first_loss_hip": l_hip, "first_loss_torch": l_torch,
                      "first_step_grad": {
                          "hip_vs_torch_global_rel": global_rel(g_hip, g_torch),
                          "hip_vs_torch_worst_tensor": [worst_k, pt[worst_k]],
                          "torch_vs_torch_global_rel": global_rel(g_torch2, g_torch),
                          "torch_vs_torch_worst_tensor_rel": max(per_tensor(g_torch2, g_torch).values()),
                          "hip_vs_hip_max_abs": max((g_hip2[k] - g_hip[k]).abs().max().item() for k in g_hip),
                          "fp64": fp64},
                      "amp_16_mixed": amp,
                      "note": "SWEGNN layers (7 processors + 3 unpooling), encoders, decoder and mean pooling on "
                              "HIP training kernels; scale selections, loss, clipping, AdamW: torch on the same "
                              "GPU. Gradients after clip_grad_norm_(1.0) of the first training step."}),
          flush=True)


if __name__ == "__main__":
    main()
