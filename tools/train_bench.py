"""Training-step throughput of MSGNN on MI355X: the reference's training_step
(training/train.py:125-145: curriculum rollout of R steps, BC write, forward, use_prediction,
per-step RMSE loss, mean) + backward + gradient clipping (main.py: gradient_clip_val=1) +
AdamW step, with every SWEGNN layer on the HIP training kernels (mswegnn/autograd.py) against
the all-torch autograd path of the same drop-in model on the same GPU.  Also reports the loss
and gradient agreement of the two paths at the first step.

    python tools/train_bench.py [--workload zenodo4] [--rollout-steps 4] [--steps 5]
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
    sc = torch.tensor([1.0, velocity_scaler], device=pred.device)
    return torch.dot(per_var, sc) / sc.sum()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="zenodo4")
    ap.add_argument("--rollout-steps", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--only", choices=["hip", "torch"], default=None)
    a = ap.parse_args()
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

    def run(engine):
        from models.gnn import MSGNN  # noqa: F401
        m = m0
        m.load_state_dict(state0)
        m.train()
        m.engine = engine
        opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=0.0)
        dyn = m.previous_t * m.NUM_WATER_VARS

        def step():
            opt.zero_grad(set_to_none=True)
            temp = g.clone()
            losses = []
            for i in range(R):
                temp.x[:, -dyn:] = apply_boundary_condition(temp.x[:, -dyn:], temp.BC[:, :, i], temp.node_BC,
                                                            type_BC=temp.type_BC)
                preds = m(temp)
                temp.x = use_prediction(temp.x, preds, m.previous_t)
                losses.append(rmse_loss(preds, y[:, :, i], n0))
            loss = torch.stack(losses).mean()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
            return loss
        first = step()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
        opt.step()
        for _ in range(a.warmup):
            step()
            opt.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
            opt.step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps, float(first), grads
    if a.only:
        t, l, _ = run("auto" if a.only == "hip" else "torch")
        print(json.dumps({"only": a.only, "ms_per_training_step": t * 1e3, "first_loss": l}), flush=True)
        return
    t_hip, l_hip, g_hip = run("auto")
    t_torch, l_torch, g_torch = run("torch")
    worst = max(((g_hip[k] - g_torch[k]).abs().max() / g_torch[k].abs().max().clamp(min=1e-30)).item()
                for k in g_torch)
    print(json.dumps({"workload": a.workload, "fine_nodes": n0, "all_nodes": desc["all_nodes"],
                      "rollout_steps_per_training_step": R,
                      "hip_ms_per_training_step": t_hip * 1e3, "torch_ms_per_training_step": t_torch * 1e3,
                      "speedup": t_torch / t_hip,
                      "fine_node_steps_per_s_hip": n0 * R / t_hip,
                      "fine_node_steps_per_s_torch": n0 * R / t_torch,
                      "first_loss_hip": l_hip, "first_loss_torch": l_torch,
                      "first_step_grad_max_rel_diff": worst,
                      "note": "SWEGNN layers (7 processors + 3 unpooling) on HIP training kernels; "
                              "encoders, pooling, decoder, loss, optimizer: torch on the same GPU"}),
          flush=True)


if __name__ == "__main__":
    main()
