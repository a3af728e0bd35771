"""Thread sweep of the CPU baseline (bench.py cpu_baseline): the oracle's rollout of one
zenodo4 simulation (the reference's algorithm, same ATen CPU ops) at 1 / 8 / 16 / 32 / 64
host threads (and all of them on hosts of at most 64 cores), fine-node-steps/s each.  Why bench.py caps the baseline at 16 threads: the
GPU box gives one GPU a 16-thread CPU share, and the rate does not grow past it.

    python tools/cpu_threads.py [--steps 3] > profiles/r06/cpu_threads.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mswe-gnn_amd"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import bench  # noqa: E402
import msgnn_torch as orc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--workload", default="zenodo4")
    args = ap.parse_args()
    g, m, w, desc = bench.build_workload(args.workload, 0, 48)
    P = {k: v.detach() for k, v in m.state_dict().items()}
    cfg = orc.msgnn_config(num_scales=w["S"], hid_features=w["F"], K=w["K"])
    host = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    rows = []
    # the host's full core count only where it is small: on the GPU box the process has a 16-CPU
    # share of a 256-core machine, and 256 threads there took > 3 minutes for one step (the
    # round-6 run was killed there; 64 threads already run 5x slower than 16)
    counts = {1, 8, 16, 32, 64} | ({host} if host <= 64 else set())
    for n in sorted(c for c in counts if c <= host):
        torch.set_num_threads(n)
        orc.rollout(P, cfg, g, 1)  # warm
        t0 = time.perf_counter()
        orc.rollout(P, cfg, g, args.steps)
        dt = time.perf_counter() - t0
        rows.append({"threads": n, "seconds": dt, "value": desc["fine_nodes"] * args.steps / dt})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"workload": args.workload, "fine_nodes": desc["fine_nodes"], "steps": args.steps,
                      "unit": "fine-node-steps/s", "host_cores": host, "affinity_cores": aff,
                      "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "torch": torch.__version__,
                      "sweep": rows}))


if __name__ == "__main__":
    main()
