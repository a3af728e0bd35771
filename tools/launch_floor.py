"""Floor of a chain of dependent launches on this GPU, for comparison with the rollout step.

Captures N dependent kernels in one graph (as msw_rollout does), replays it, and reports
the time per launch for
  (a) a trivial kernel (in-place scale of 1 K floats: boundary + launch only),
  (b) a gather of every row of the previous launch's output (index_select of R rows of F
      floats through a fixed random permutation: boundary + one dependent gather of data
      the previous launch wrote -- what every hop of the rollout does at least once).
usage: python tools/launch_floor.py [--n 35] [--rows 10369] [--feat 32]
"""
import argparse
import json
import time

import torch


def per_launch_us(fn, n, reps=200):
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(3):
            fn()  # warm
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(n):
                fn()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            g.replay()
        e1.record(st)
        e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=35)
    ap.add_argument("--rows", type=int, default=10369)
    ap.add_argument("--feat", type=int, default=32)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    small = torch.ones(1024, device=dev)
    t_triv = per_launch_us(lambda: small.mul_(1.0), a.n)
    perm = torch.randperm(a.rows, device=dev)
    bufs = [torch.randn(a.rows, a.feat, device=dev), torch.empty(a.rows, a.feat, device=dev)]
    state = {"i": 0}

    def gather():
        i = state["i"]
        torch.index_select(bufs[i], 0, perm, out=bufs[1 - i])
        state["i"] = 1 - i
    t_gather = per_launch_us(gather, a.n)
    print(json.dumps({"launches_per_graph": a.n, "trivial_us_per_launch": t_triv,
                      "row_gather_us_per_launch": t_gather, "rows": a.rows, "feat": a.feat,
                      "gather_bytes": 2 * a.rows * a.feat * 4 + a.rows * 8,
                      "device": torch.cuda.get_device_name(0), "time": time.time()}))


if __name__ == "__main__":
    main()
