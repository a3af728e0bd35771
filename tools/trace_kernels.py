"""Phase-by-phase latency chain of single launches (diagnostic build, GPU box).

    python mswe-gnn_amd/build_engine.py --trace      # here (cross-compiles)
    MSW_LIB_VARIANT=trace python tools/trace_kernels.py [workload]   # on the GPU box

Wave 0 of workgroup 0 drains its memory counters at each phase mark and records
{shader clock, 100 MHz clock} (kernels_impl.h MSW_MARK), so each line below is the time
from the kernel's first instruction to that mark along ONE wave's dependency chain
(the drains remove overlap: a lower bound on what a phase costs in the real kernel is the
difference between consecutive marks).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mswe-gnn_amd")]
os.environ.setdefault("MSW_LIB_VARIANT", "trace")

import ctypes as C  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mswegnn import _lib as L  # noqa: E402
from mswegnn.engine import plan_for  # noqa: E402

PHASES = {0: "entry", 1: "tile/args", 2: "weights staged", 3: "indices", 4: "gathers",
          5: "edge MLP", 6: "message", 7: "segmented sum", 8: "filter", 9: "end (epilogue)"}


def wg_report(t):
    """Span of the launch over all workgroups (first start -> last wave's end) and where the
    late workgroups are: start / end percentiles, in us from the first start."""
    st = t[32::2]
    en = t[33::2]
    wgs = [(b, st[b], en[b]) for b in range(len(st)) if st[b] and en[b]]
    if not wgs:
        return
    s0 = min(w[1] for w in wgs)
    ends = sorted((w[2] - s0) / 100.0 for w in wgs)
    starts = sorted((w[1] - s0) / 100.0 for w in wgs)
    durs = sorted((w[2] - w[1]) / 100.0 for w in wgs)
    pct = lambda v, q: v[min(len(v) - 1, int(q * len(v)))]
    late = max(wgs, key=lambda w: w[2])
    print(f"    {len(wgs)} workgroups: span {ends[-1]:6.2f} us; start p50/p90/max {pct(starts, .5):.2f}/"
          f"{pct(starts, .9):.2f}/{starts[-1]:.2f}; end p10/p50/p90 {pct(ends, .1):.2f}/{pct(ends, .5):.2f}/"
          f"{pct(ends, .9):.2f}; own duration p50/max {pct(durs, .5):.2f}/{durs[-1]:.2f}; last = wg {late[0]}")
    nb = 8
    n = len(st)
    hi = max(w[0] for w in wgs) + 1
    row = []
    for i in range(nb):
        grp = [w for w in wgs if i * hi // nb <= w[0] < (i + 1) * hi // nb]
        if grp:
            row.append(f"{i * hi // nb}-: {max((w[2] - s0) / 100.0 for w in grp):.1f}")
    print("    latest end by workgroup range (us): " + ", ".join(row))
    if len(wgs) >= 64:  # by XCD (workgroup i -> XCD i % 8): median start, latest end
        per = []
        for x in range(8):
            grp = [w for w in wgs if w[0] % 8 == x]
            if grp:
                ss = sorted((w[1] - s0) / 100.0 for w in grp)
                per.append(f"{x}: {ss[len(ss) // 2]:.2f}/{max((w[2] - s0) / 100.0 for w in grp):.2f}")
        print("    by XCD (median start / latest end, us): " + ", ".join(per))


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "zenodo4"
    dev = torch.device("cuda:0")
    g, m, w, desc = bench.build_workload(wl, seed=0, T=8)
    g = g.to(dev)
    m = m.to(dev)
    m.engine = "hip"
    plan = plan_for(m, g)
    plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, 8)
    NWG = 8192  # kernels_impl.h kTraceWG: per-workgroup start / end at [32 + 2 b], [33 + 2 b]
    buf = torch.zeros(32 + 2 * NWG, dtype=torch.int64, device=dev)
    L.check(L.lib().msw_set_trace(plan._h, C.c_void_p(buf.data_ptr())))
    S = desc["num_scales"]
    cases = [("encode", 0)] + [(k, s) for s in range(S) for k in ("edge_hop", "hop")] + \
        [("pool", s) for s in range(1, S)] + [("unpool", s) for s in range(S - 1)] + \
        [("hop", s) for s in range(S)]
    for kern, scale in cases:
        try:
            for rep in range(3):  # the last repetition is reported (warm caches)
                buf.zero_()
                plan.bench_kernel(kern, scale, 1)
                torch.cuda.synchronize()
        except RuntimeError as e:  # e.g. pooling fused into the coarse scale's first launch
            print(f"{kern:9s} scale {scale}: n/a ({e})")
            continue
        t = buf.cpu().tolist()
        clk0, rt0 = t[0], t[1]
        marks = [(k, t[2 * k] - clk0, (t[2 * k + 1] - rt0) * 10.0) for k in range(10) if t[2 * k] != 0]
        if len(marks) < 2:
            print(f"{kern:9s} scale {scale}: no phase marks in this kernel")
            continue
        last = marks[-1]
        mhz = last[1] / (last[2] / 1e3) if last[2] > 0 else float("nan")
        print(f"{kern:9s} scale {scale}: {last[2] / 1e3:6.2f} us on wave 0 (~{mhz:.0f} MHz)")
        wg_report(t)
        prev = 0.0
        for k, cyc, ns in marks[1:]:
            print(f"    {PHASES[k]:16s} +{(ns - prev) / 1e3:6.2f} us  (at {ns / 1e3:6.2f} us, {cyc} clk)")
            prev = ns
    if os.environ.get("MSW_TRACE_ENCODE"):  # rollout-mode encoder (deferred decoder first)
        L.check(L.lib().msw_set_trace(plan._h, C.c_void_p(buf.data_ptr())))
        buf.zero_()
        plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, 3)
        torch.cuda.synchronize()
        t = buf.cpu().tolist()
        clk0, rt0 = t[0], t[1]
        marks = [(k, t[2 * k] - clk0, (t[2 * k + 1] - rt0) * 10.0) for k in range(10) if t[2 * k] != 0]
        print(f"encode (rollout step 2, decoder of step 1 first): {marks[-1][2] / 1e3:6.2f} us on wave 0")
        wg_report(t)
        prev = 0.0
        names = {**PHASES, 2: "weights + decoder", 5: "static encoder", 6: "dynamic encoder",
                 8: "projection 0", 9: "unpool V (end)"}
        for k, cyc, ns in marks[1:]:
            print(f"    {names[k]:18s} +{(ns - prev) / 1e3:6.2f} us  (at {ns / 1e3:6.2f} us, {cyc} clk)")
            prev = ns
    # the finest scale's last hop + decoder epilogue: the last launch of a rollout step, so a
    # one-step rollout leaves its marks in the buffer (marks it does not set are skipped)
    buf.zero_()
    plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, 1)
    torch.cuda.synchronize()
    t = buf.cpu().tolist()
    clk0, rt0 = t[0], t[1]
    marks = sorted([(k, t[2 * k] - clk0, (t[2 * k + 1] - rt0) * 10.0) for k in (0, 1, 2, 4, 6, 7, 8, 9)
                    if t[2 * k] != 0], key=lambda mk: mk[2])  # time order (the staging wait is late)
    if len(marks) >= 2:
        print(f"last hop + decoder, scale 0 (last launch of a rollout step): {marks[-1][2] / 1e3:6.2f} us on wave 0")
        prev = 0.0
        for k, cyc, ns in marks[1:]:
            print(f"    {PHASES[k]:16s} +{(ns - prev) / 1e3:6.2f} us  (at {ns / 1e3:6.2f} us, {cyc} clk)")
            prev = ns
    L.check(L.lib().msw_set_trace(plan._h, None))


if __name__ == "__main__":
    main()
