"""Practical HBM store / copy bandwidth on one MI355X (torch fill_ / copy_, HIP events): the
ceiling a store-bound launch such as config 5's encoder (1.26 GB of stores per launch) is
compared with.  Prints one JSON line.

    python tools/hbm_write_bw.py [--gb 1.26] [--iters 20]
"""
import argparse
import json

import torch


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=1.26)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n = int(a.gb * 1e9 / 4)
    x = torch.empty(n, device="cuda")
    y = torch.empty(n, device="cuda")
    t_fill = timed(lambda: x.fill_(1.0), a.iters)
    t_copy = timed(lambda: y.copy_(x), a.iters)
    print(json.dumps({"bytes": 4 * n, "fill_s": t_fill, "fill_TBps": 4 * n / t_fill / 1e12,
                      "copy_s": t_copy, "copy_TBps_read_plus_write": 8 * n / t_copy / 1e12,
                      "device": torch.cuda.get_device_name(0)}), flush=True)


if __name__ == "__main__":
    main()
