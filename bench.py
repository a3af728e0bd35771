#!/usr/bin/env python
"""Benchmark: multi-scale SWE-GNN rollout throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload zenodo4]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one full T=48 autoregressive rollout (rollout_test semantics) of one simulation
per rank, with inputs resident in HBM, through the HIP engine (fused msw_rollout: the T
steps replay a captured hipGraph).  Ranks run independent simulations (weak scaling, one
sim per GPU, seed = rank); at N>1 each step ends with ONE RCCL all-gather of the fine-scale
rollouts (the north star's end-of-rollout collective).  Throughput = all ranks' fine-scale
nodes x rollout steps / max-over-ranks wall time.

Rank 0 also reports:
  roofline      -- the aggregation (hop) kernel at the finest scale, timed live with HIP
                   events on the stream it is launched on, algorithmic bytes per launch
                   E*(4F+4) + N*(12F+4), peak 8 TB/s;
  cpu_baseline  -- (N=1 only) the reference algorithm on the host cores (oracle, same ATen
                   CPU ops as the reference, bit-identical to it), bounded sample;
  parity        -- max |GPU - CPU reference| over the rollout (the metric's error term).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "mswe-gnn_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFS = 157.3  # dense fp32 matrix peak (spec)


def load_weights(name):
    z = np.load(os.path.join(ROOT, "tests", "golden", f"weights_{name}.npz"))
    return {k: torch.from_numpy(z[k]) for k in z.files}


WORKLOADS = {
    # config 2: Zenodo-like mesh, 4 scales, shipped K4_F32 checkpoint
    "zenodo4": dict(mesh="zenodo4", S=4, F=32, K=4, weights="K4_F32"),
    # config 2, "3-scale" wording: same N0, 3 scales, seeded init (no 3-scale checkpoint)
    "zenodo3": dict(mesh="zenodo3", S=3, F=32, K=4, weights=None),
    # config 2 with the other shipped 4-scale checkpoint (hid_features 16, K 2)
    "zenodo4_k2f16": dict(mesh="zenodo4", S=4, F=16, K=2, weights="K2_F16"),
    # config 2 at the reference's default config.yaml width (hid_features 64, K 4; no
    # F = 64 checkpoint is shipped -> seeded init)
    "zenodo4_f64": dict(mesh="zenodo4", S=4, F=64, K=4, weights=None),
    # config 3: Zenodo-like test meshes of 8,193-12,801 fine nodes (member i: size cycled,
    # seed i; mswegnn.mesh.config3_members), 3 scales seeded init / 4 scales K4_F32
    "config3": dict(mesh="config3", S=3, F=32, K=4, weights=None),
    "config3_k4": dict(mesh="config3", S=4, F=32, K=4, weights="K4_F32"),
    # config 4: dk15-like mesh (fine-tune checkpoint not shipped -> K4_F32 weights)
    "dk15": dict(mesh="dk15", S=4, F=32, K=4, weights="K4_F32"),
    # config 5: ~1M fine nodes, 3 scales, fully wet (every edge active)
    "hbm1m": dict(mesh="hbm1m", S=3, F=32, K=4, weights=None),
    # plumbing size for the CPU (gloo) tests of the multi-rank path
    "tiny": dict(mesh="tiny", S=4, F=32, K=4, weights="K4_F32"),
    # two sizes alternating by seed (CPU gloo test of the all-gather's padding path)
    "tiny_mixed": dict(mesh="tiny_mixed", S=4, F=32, K=4, weights="K4_F32"),
}


def sim_mesh_kwargs(name, seed):
    """make_multiscale_mesh keywords of simulation `seed` of a workload."""
    from mswegnn.mesh import mesh_config, config3_members
    w = WORKLOADS[name]
    if w["mesh"] == "config3":
        return config3_members(w["S"], count=seed + 1)[seed]
    if w["mesh"] == "tiny_mixed":
        return dict(n_coarse=2 + seed % 2, num_scales=4, seed=seed)
    return dict(mesh_config(w["mesh"]), seed=seed)


def sim_fine_nodes(name, seed):
    """Fine-scale nodes of simulation `seed` without building it: the generator's coarse
    n x n x 2 triangles refined 1 -> 4 (S - 1) times, plus the ghost cell (mswegnn/mesh.py)."""
    kw = sim_mesh_kwargs(name, seed)
    return 2 * kw["n_coarse"] ** 2 * 4 ** (kw["num_scales"] - 1) + 1


def build_workload(name, seed, T):
    """Simulation `seed` of a workload -> (graph, model, workload row, description)."""
    from models.gnn import MSGNN
    from mswegnn.mesh import make_multiscale_mesh
    w = WORKLOADS[name]
    g = make_multiscale_mesh(**sim_mesh_kwargs(name, seed), T=T)
    if name == "hbm1m":
        from mswegnn.mesh import wet_state
        g = wet_state(g, seed=seed, all_wet=True)
    m = MSGNN(num_node_features=8, num_edge_features=1, num_scales=w["S"], hid_features=w["F"],
              K=w["K"], mlp_layers=3, seed=666, learned_residuals=True, mlp_activation="prelu",
              gnn_activation="tanh", edge_mlp=True, normalize=True, with_filter_matrix=True,
              with_gradient=True, with_WL=True, learned_pooling=False, skip_connections=True,
              previous_t=3)
    if w["weights"]:
        m.load_state_dict(load_weights(w["weights"]), strict=True)
    m.eval()
    n0 = int(g.node_ptr[1])
    desc = dict(workload=name, mesh=w["mesh"], num_scales=w["S"], hid_features=w["F"], K=w["K"],
                mlp_layers=3, weights=w["weights"] or "seeded-init(seed=666)",
                fine_nodes=n0, all_nodes=int(g.x.shape[0]), edges=int(g.edge_index.shape[1]),
                rollout_steps=T)
    return g, m, w, desc


CPU_SHARE_NOTE = ("threads = the CPU share of one GPU on the GPU box, 16 (gpurun sets OMP_NUM_THREADS=16; "
                  "os.cpu_count() there reports the whole machine, host_cores); more threads run slower: "
                  "one zenodo4 simulation at 1 / 8 / 16 / 32 / 64 threads 0.065 / 0.113 / 0.131 / 0.062 / "
                  "0.028 M fine-node-steps/s (profiles/r06/cpu_threads.json)")


def cpu_share():
    """(host cores, threads the CPU baseline uses): OMP_NUM_THREADS (the GPU box's per-GPU share)
    else the host's cores, at most 16."""
    host = os.cpu_count() or 1
    return host, min(int(os.environ.get("OMP_NUM_THREADS", "0")) or host, 16)


def _cpu_sim_worker(job):
    """One simulation of a workload through the oracle on the host (a spawned process of
    cpu_batch_baseline): built, then every worker starts its timed rollout together."""
    name, seed, T, Tc, threads, seconds, barrier = job
    torch.set_num_threads(threads)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import msgnn_torch as orc  # test/baseline infrastructure only
    g, m, w, desc = build_workload(name, seed, T)
    P = {k: v.detach() for k, v in m.state_dict().items()}
    cfg = orc.msgnn_config(num_scales=w["S"], hid_features=w["F"], K=w["K"])
    barrier.wait(timeout=300)
    c0 = time.time()
    steps = 0
    while steps == 0 or time.time() - c0 < seconds:  # whole Tc-step rollouts for ~`seconds`
        orc.rollout(P, cfg, g, Tc)
        steps += Tc
    return desc["fine_nodes"], steps, c0, time.time()


def cpu_batch_baseline(name, ids, T, share, seconds, t1, t1_threads):
    """The CPU analogue of the reference's batched evaluation: the simulations `ids` one per
    process, all at once, over the `share` host threads (threads split evenly), each a
    Tc-step rollout sized from the single-simulation step time t1 (measured on t1_threads),
    repeated for ~`seconds`.  -> {value, unit, processes, threads_per_process, sample}."""
    import multiprocessing as mp
    ids = list(ids)[:share]
    procs = len(ids)
    tpp = max(1, share // procs)
    Tc = int(min(T, max(1, seconds / max(t1 * t1_threads / tpp, 1e-6))))
    ctx = mp.get_context("spawn")  # fresh interpreters: no GPU state, no fork of this process
    with ctx.Manager() as man:
        bar = man.Barrier(procs)
        with ctx.Pool(procs) as pool:
            res = pool.map(_cpu_sim_worker, [(name, i, T, Tc, tpp, seconds, bar) for i in ids], chunksize=1)
    wall = max(r[3] for r in res) - min(r[2] for r in res)
    work = sum(r[0] * r[1] for r in res)
    return {"value": work / wall, "unit": "fine-node-steps/s", "processes": procs, "threads_per_process": tpp,
            "cores": procs * tpp, "kind": "port",
            "sample": f"{procs} simulations of the workload (ids {ids[0]}..{ids[-1]}), {Tc}-step rollouts repeated "
                      f"for ~{seconds:.0f} s in one process each, started together; "
                      f"{sum(r[1] for r in res)} simulation-steps in all, wall {wall:.1f} s"}


def make_gatherer(dist, world, n0, T, device):
    """The end-of-rollout collective: ONE all-gather of every rank's fine-scale rollout
    [n0_r, 2, T].  Sizes are exchanged once here (meshes may differ per rank); payloads are
    padded to the largest n0.  Returns gather(out_fine) -> list of [n0_r, 2, T] per rank.
    dist None (a single rank without a process group): no collective."""
    if dist is None:
        return lambda out_fine: [out_fine]
    sz = torch.tensor([n0], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(sz) for _ in range(world)]
    dist.all_gather(sizes, sz)
    sizes = [int(x.item()) for x in sizes]
    nmax = max(sizes)
    slots = [torch.empty(nmax, 2, T, device=device) for _ in range(world)]
    pad = torch.zeros(nmax, 2, T, device=device)

    def gather(out_fine):
        src = out_fine.to(device)
        if n0 != nmax:
            pad[:n0].copy_(out_fine)
            src = pad
        dist.all_gather(slots, src.contiguous())
        return [slots[r][:sizes[r]] for r in range(world)]
    return gather


def time_kernel(plan, kernel, scale, iters=200):
    """Average duration (s) of one launch, HIP events on the launching stream."""
    st = torch.cuda.current_stream()
    plan.bench_kernel(kernel, scale, 5)  # warm
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    units = plan.bench_kernel(kernel, scale, iters)
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / 1e3 / iters, units


def summary_provenance(d, lib_sha):
    """Which library a committed profile summary was measured on, against the one loaded now."""
    src = d.get("library_sha256")
    return {"source_library_sha256": src, "stale": (src != lib_sha) if src else True,
            "source": d.get("source")}


def read_traffic(path, kernel_prefix, lib_sha=None):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (profiles/), or None.
    With lib_sha: {"bytes_per_launch", "source_library_sha256", "stale"} instead."""
    try:
        with open(path) as f:
            d = json.load(f)
    except OSError:
        return None
    v = d.get(kernel_prefix, {}).get("hbm_bytes_per_launch")
    if lib_sha is None or v is None:
        return v
    return dict(summary_provenance(d, lib_sha), bytes_per_launch=v, kernel=d.get(kernel_prefix, {}).get("kernel"))


def lpt_split(sizes, world):
    """Longest-processing-time assignment of simulations (work ~ fine nodes) to `world`
    ranks: largest first, each to the least-loaded rank (lowest rank on ties).  Returns the
    ascending simulation ids of every rank."""
    load = [0] * world
    own = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda i: (-sizes[i], i)):
        r = min(range(world), key=lambda q: (load[q], q))
        load[r] += sizes[i]
        own[r].append(i)
    return [sorted(o) for o in own]


def simulations_of_rank(args, rank, world, workload=None):
    """Simulation ids this rank runs.  --global-batch G: a FIXED set of G simulations split
    over the ranks by size (lpt_split on fine nodes; SURVEY §8(e), strong scaling).
    Otherwise --batch B per rank, ids r*B .. r*B+B-1 (weak scaling)."""
    if args.global_batch:
        if args.global_batch < world:
            raise SystemExit(f"--global-batch {args.global_batch} < {world} ranks")
        wl = workload or getattr(args, "workload", "zenodo4")
        sizes = [sim_fine_nodes(wl, i) for i in range(args.global_batch)]
        return lpt_split(sizes, world)[rank], "strong"
    B = max(1, args.batch)
    return [rank * B + i for i in range(B)], "weak"


def rank_batch(workload, ids, T, cache=None):
    """This rank's simulations as ONE graph: the single simulation, or a disjoint-union batch
    in the reference's layout (PyG collation + adapt_batch_training / update_batch_multiscale,
    train.py:14-65).  -> (sims, graph, fine_rows or None, fine nodes per rollout).
    cache: optional dict id -> build_workload result, reused across calls."""
    if cache is None:
        cache = {}
    for i in ids:
        if i not in cache:
            cache[i] = build_workload(workload, seed=i, T=T)
    sims = [cache[i] for i in ids]
    fine = sum(s[3]["fine_nodes"] for s in sims)
    if len(sims) == 1:
        return sims, sims[0][0], None, fine
    from mswegnn.batch import collate
    from mswegnn.rollout import adapt_batch_training
    gb = adapt_batch_training(collate([s[0] for s in sims]))
    npt = gb.node_ptr
    rows = torch.cat([torch.arange(int(npt[i, 0]), int(npt[i, 1])) for i in range(len(sims))])
    return sims, gb, rows, fine


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def make_runner(workload, ids, T, dev, engine, cache):
    """One rank's share as ONE batch on `dev` -> (run() -> [N, 2, T], fine_of(out) -> this
    share's fine-scale rows [sum n0, 2, T] in id order, fine nodes, close()).
    engine 'hip': a dedicated EnginePlan (msw_rollout); 'torch': the drop-in's torch path
    (CPU tests of the multi-rank logic)."""
    sims, gb, rows, fine = rank_batch(workload, ids, T, cache)
    g = gb.to(dev)
    m = sims[0][1].to(dev)
    m.engine = engine
    if engine == "hip":
        from mswegnn.engine import EnginePlan
        plan = EnginePlan(m, g, dev)
        out = torch.empty(g.num_nodes, 2, T, device=dev)

        def run():
            return plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, T, out=out)

        close = plan.close
    else:
        def run():
            return m.rollout(g, T)

        def close():
            pass
    fr = rows.to(dev) if rows is not None else None

    def fine_of(r):
        return r[:fine] if fr is None else r.index_select(0, fr)
    return run, fine_of, fine, close


def strong_scaling_section(dist, rank, world, dev, engine, sets, T, steps, warmup, barrier,
                           workload="config3"):
    """The north star's strong scaling, measured in-run (BASELINE config 3):
    for each fixed set of G simulations, rank 0 first runs the WHOLE set alone as one batch
    (t1) while the other ranks wait; then every rank runs its share (lpt_split by fine nodes,
    one batch per rank) and each rollout ends with the real all-gather of the fine-scale
    rollouts over the default process group (RCCL on nccl) -- tW = max over ranks.  Rank 0
    also checks that the gathered rollouts equal its single-GPU ones.  Returns the record
    (complete on rank 0)."""
    red_dev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    cache = {}
    rec = {"workload": workload, "rollout_steps": T, "timed_rollouts": steps, "warmup": warmup,
           "rccl_world": dist.get_world_size(), "backend": dist.get_backend(),
           "split": "longest-processing-time by fine nodes (bench.lpt_split)", "sets": []}
    for G in sets:
        if G < world:
            rec["sets"].append({"G": G, "skipped": f"fewer simulations than the {world} ranks"})
            continue
        sizes = [sim_fine_nodes(workload, i) for i in range(G)]
        split = lpt_split(sizes, world)
        ent = {"G": G, "sims_per_rank": [len(s) for s in split],
               "fine_nodes_per_rank": [sum(sizes[i] for i in s) for s in split],
               "fine_nodes_total": sum(sizes)}
        # ---- phase A: the whole set on rank 0 alone
        ref = None
        if rank == 0:
            run, fine_of, _, close = make_runner(workload, list(range(G)), T, dev, engine, cache)
            for _ in range(warmup):
                run()
            _sync(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                r = run()
            _sync(dev)
            t1 = (time.perf_counter() - t0) / steps
            ref = fine_of(r).cpu()
            close()
            ent["t1_ms"] = t1 * 1e3
        barrier()
        # ---- phase B: every rank its share + the end-of-rollout all-gather
        run, fine_of, fine, close = make_runner(workload, split[rank], T, dev, engine, cache)
        gather = make_gatherer(dist, world, fine, T, red_dev)

        def step():
            return gather(fine_of(run()).contiguous())
        parts = None
        for _ in range(warmup):
            parts = step()
        _sync(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            parts = step()
        _sync(dev)
        dist.barrier()
        tw_local = (time.perf_counter() - t0) / steps
        tt = torch.tensor([tw_local], device=red_dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        tw = float(tt.item())
        tl = [torch.zeros(1, device=red_dev, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(tl, torch.tensor([tw_local], device=red_dev, dtype=torch.float64))
        close()
        if rank == 0:
            start = [0]
            for n in sizes:
                start.append(start[-1] + n)
            worst = 0.0
            den = max(float(ref.abs().max()), 1e-30)
            for q in range(world):
                slot, o = parts[q].cpu(), 0
                for i in split[q]:
                    n = sizes[i]
                    worst = max(worst, float((slot[o:o + n] - ref[start[i]:start[i] + n]).abs().max()) / den)
                    o += n
            t1 = ent["t1_ms"] / 1e3
            ent.update({"tW_ms": tw * 1e3, "rank_ms": [float(x.item()) * 1e3 for x in tl],
                        "speedup": t1 / tw,
                        "fine_node_steps_per_s_1gpu": sum(sizes) * T / t1,
                        "fine_node_steps_per_s_Wgpu": sum(sizes) * T / tw,
                        "gathered_vs_single_gpu_max_rel": worst})
        rec["sets"].append(ent)
    return rec


def child_json_record(cmd, timeout):
    """Run a checker as a child in its own session with a time limit and return the JSON line
    it prints (on a time-out the child AND its rank processes are killed) -- recorded, never
    fatal, and a hang cannot stall the bench."""
    import signal
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    try:
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                             start_new_session=True)
        try:
            so, se = p.communicate(timeout=timeout)
            lines = [ln for ln in so.splitlines() if ln.startswith("{")]
            res = json.loads(lines[-1]) if lines else {"error": "no result line", "stderr_tail": se[-800:]}
            res["exit_code"] = p.returncode
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            res = {"error": f"timed out after {timeout} s"}
    except Exception as e:  # noqa: BLE001
        res = {"error": repr(e)}
    return res


def partitioned_rollout_check(rank, world, barrier, timeout=300, parts=2, mesh="zenodo4", steps=5):
    """Single-mesh domain decomposition over RCCL: rank 0 runs
    tools/rccl_partition_check.py (`parts` fresh processes on GPUs 0..parts-1,
    DistributedRollout with the RCCL halo exchange, gather_owned over RCCL, compared with the
    undivided plan) as a child (child_json_record)."""
    res = None
    if rank == 0:
        cmd = [sys.executable, os.path.join(ROOT, "tools", "rccl_partition_check.py"), str(parts), "--mesh", mesh,
               "--steps", str(steps), "--wait", str(max(30, timeout - 30))]
        res = child_json_record(cmd, timeout)
    barrier()
    return res


def ddp_training_check(rank, world, barrier, timeout=150):
    """Training on several GPUs over RCCL: rank 0 runs tools/ddp_train_check.py
    (DistributedDataParallel over the HIP training kernels, one GPU per rank, nccl; gradients
    against one process's mean of the ranks' gradients) as a child (child_json_record)."""
    res = None
    if rank == 0:
        W = min(world, torch.cuda.device_count())
        cmd = [sys.executable, os.path.join(ROOT, "tools", "ddp_train_check.py"), str(W), "--backend", "nccl",
               "--wait", str(max(30, timeout - 30))]
        res = child_json_record(cmd, timeout)
    barrier()
    return res


# N > 1 records after the weak line's timed region, run in this order inside ONE wall-clock
# budget (--extras-budget): a section starts only when its estimated cost fits what is left,
# so the line is printed before a driver time limit whatever the node does.  Estimates (s):
# a strong-scaling set of G config-3 simulations ~ 10 + 0.4 G (mesh generation on rank 0
# dominates: ~26 s for G = 128); the RCCL children get min(their limit, what is left) and
# start only with at least `start_s` left.
CHILD_SECTIONS = {  # name -> (limit s, minimum left to start s)
    "zenodo4_2_parts": (180, 60), "ddp": (150, 60), "hbm1m_parts": (240, 120)}


def strong_set_cost(G):
    return 10.0 + 0.4 * G


def run_extras(dist, rank, world, dev, args, cpu_barrier, backend, group=None, engine="hip",
               workload="config3", gpus=None):
    """The N > 1 records (strong scaling, RCCL single-mesh decomposition, DDP training) under
    one budget.  Every rank calls this; rank 0 decides whether a section starts and broadcasts
    the decision (host group), so all ranks take the same branches.  Returns the records
    (complete on rank 0): skipped sections are {"skipped": ...}, every section has wall_s."""
    t0 = time.perf_counter()
    budget = float(args.extras_budget)
    gpus = torch.cuda.device_count() if gpus is None else gpus

    def left():
        return budget - (time.perf_counter() - t0)

    def agree(ok):
        obj = [bool(ok)]
        dist.broadcast_object_list(obj, src=0, group=group)
        return obj[0]
    sets = [int(x) for x in str(args.strong_sets).split(",") if x.strip()]
    small = [G for G in sets if G <= 16]
    large = [G for G in sets if G > 16]
    rccl_ok = backend == "nccl" and gpus >= 2 and not args.no_partition_check
    W = min(world, gpus)
    order = ([("strong", G) for G in small] + [("child", "zenodo4_2_parts"), ("child", "ddp")]
             + [("strong", G) for G in large] + [("child", "hbm1m_parts")])
    strong = None
    part, ddp = {}, None
    log = []
    for kind, what in order:
        s0 = time.perf_counter()
        if kind == "strong":
            need = strong_set_cost(what)
            go = agree(left() >= need)
            if go:
                try:
                    rec = strong_scaling_section(dist, rank, world, dev, engine, [what], args.T, args.strong_steps,
                                                 1, cpu_barrier, workload=workload)
                except Exception as e:  # noqa: BLE001
                    rec = {"sets": [{"G": what, "error": repr(e)}]}
                ent = rec["sets"][0] if rec.get("sets") else {"G": what}
                if strong is None:
                    strong = {k: v for k, v in rec.items() if k != "sets"}
                    strong["sets"] = []
            else:
                ent = {"G": what, "skipped": "budget", "left_s": round(left(), 1), "needs_s": need}
                if strong is None:
                    strong = {"workload": workload, "sets": []}
            ent["wall_s"] = round(time.perf_counter() - s0, 2)
            strong["sets"].append(ent)
            log.append((f"strong_G{what}", ent["wall_s"], "skipped" in ent))
            continue
        limit, start = CHILD_SECTIONS[what]
        if what == "hbm1m_parts" and (args.no_partition_large or W < 4):
            res = {"skipped": "single-mesh decomposition of the ~1.3M-node mesh runs at N >= 4"
                              + (" (--no-partition-large)" if args.no_partition_large else "")}
        elif not rccl_ok:
            res = {"skipped": "needs the nccl (RCCL) backend and >= 2 GPUs"
                              + (" (--no-partition-check)" if args.no_partition_check else "")}
        elif not agree(left() >= start):
            res = {"skipped": "budget", "left_s": round(left(), 1), "needs_s": start}
        else:
            tl = int(max(30, min(limit, left())))
            if what == "ddp":
                res = ddp_training_check(rank, world, cpu_barrier, timeout=tl)
            elif what == "zenodo4_2_parts":
                res = partitioned_rollout_check(rank, world, cpu_barrier, timeout=tl)
            else:
                res = partitioned_rollout_check(rank, world, cpu_barrier, timeout=tl, parts=W, mesh="hbm1m", steps=2)
            res = dict(res or {}, time_limit_s=tl)
        res["wall_s"] = round(time.perf_counter() - s0, 2)
        log.append((what, res["wall_s"], "skipped" in res))
        if what == "ddp":
            ddp = res
        else:
            part[f"hbm1m_{W}_parts" if what == "hbm1m_parts" else what] = res
    return {"strong_scaling": strong, "partitioned_rollout_rccl": part, "ddp_training_rccl": ddp,
            "extras": {"budget_s": budget, "wall_s": round(time.perf_counter() - t0, 2),
                       "order": [{"section": n, "wall_s": w, "skipped": sk} for n, w, sk in log]}}


def msw_env():
    """The engine switches set in this process (DESIGN §4 'Switches'): empty on a default run."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("MSW_")}


def _built_from_sources():
    try:
        import build_engine
        return build_engine.library_matches_sources()
    except Exception:  # noqa: BLE001
        return None


def self_launch(n, backend):
    """`bench.py --gpus N` run without a launcher: N ranks under torch.distributed.run on this
    node (127.0.0.1, a free port), the same arguments; rank 0 prints the line.  With RCCL the
    node must have N GPUs (counted without initialising one); gloo rehearsals may share them."""
    import socket
    import subprocess
    ngpu = torch.cuda.device_count()
    if backend == "nccl" and ngpu < n:
        print(f"bench.py: --gpus {n} needs {n} GPUs for one RCCL rank each; this node has {ngpu}",
              file=sys.stderr, flush=True)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench.py: launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    # stdout carries the ONE result line: the ranks' other output (the gloo library prints
    # connection notes to stdout) goes to stderr
    with subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1) as p:
        for line in p.stdout:
            out = sys.stdout if line.startswith("{") else sys.stderr
            out.write(line)
            out.flush()
    return p.returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each); default: the launcher's WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="zenodo4", choices=sorted(WORKLOADS))
    ap.add_argument("--T", type=int, default=48)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-roofline-large", action="store_true",
                    help="skip the hop-kernel roofline on the ~1M-node mesh (config 5)")
    ap.add_argument("--batch", type=int, default=1,
                    help="simulations per GPU, run as one disjoint-union batch (SURVEY §8 f1)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="a fixed set of G simulations split round-robin over the ranks "
                         "(strong scaling; each rank runs its share as one batch)")
    ap.add_argument("--caller", default="fused", choices=["fused", "reference-loop"],
                    help="fused: rollout_test as ONE msw_rollout; reference-loop: the reference's "
                         "own rollout_test loop (train.py:87-95), one HIP msw_forward per step")
    ap.add_argument("--strong-sets", default="8,128",
                    help="N > 1: fixed config-3 sets (G simulations each) of the strong_scaling "
                         "record; '' = none")
    ap.add_argument("--strong-steps", type=int, default=3)
    ap.add_argument("--no-partition-large", action="store_true",
                    help="N > 1: skip the ~1.3M-node mesh in the RCCL single-mesh decomposition record")
    ap.add_argument("--no-partition-check", action="store_true",
                    help="N > 1: skip the RCCL single-mesh decomposition check")
    ap.add_argument("--extras-budget", type=float, default=180.0,
                    help="N > 1: wall-clock budget (s) of the records after the timed region, run in "
                         "the order strong G<=16, zenodo4 2 parts, DDP, strong G>16, hbm1m parts; "
                         "a section that does not fit is recorded as skipped")
    args = ap.parse_args()

    # one rank per GPU; MSW_DIST_BACKEND=gloo + more ranks than GPUs rehearses the N > 1 path
    # on a one-GPU box (ranks share the device; RCCL refuses two ranks on one device)
    backend = os.environ.get("MSW_DIST_BACKEND", "nccl")
    gpus_given = args.gpus is not None
    if not gpus_given:
        args.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` without a launcher: start the N ranks ourselves, before anything
        # here touches a GPU (no exec: the ranks are children, their exit code is ours)
        sys.exit(self_launch(args.gpus, backend))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if gpus_given and world != args.gpus:  # an explicit --gpus that contradicts the launcher
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks",
              file=sys.stderr, flush=True)
        sys.exit(2)
    if not torch.cuda.is_available():
        print(f"bench.py rank {rank}/{world}: no GPU visible (the HIP engine needs an MI355X)",
              file=sys.stderr, flush=True)
        sys.exit(3)
    dist = None
    gpu = local % max(1, torch.cuda.device_count()) if backend != "nccl" else local
    cpu_group = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
        # host-side barrier for long waits (rank 0 alone on the GPU): no spinning collective
        cpu_group = dist.new_group(backend="gloo")
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    T = args.T
    ids, scaling = simulations_of_rank(args, rank, world, args.workload)
    B = len(ids)
    sims, gb, fine_rows, fine_rank = rank_batch(args.workload, ids, T)
    g_cpu, model_cpu, w, desc = sims[0]
    n0_list = [s[3]["fine_nodes"] for s in sims]
    n0 = n0_list[0]
    if B > 1:
        desc = dict(desc, batch=B, batch_nodes=int(gb.x.shape[0]), batch_fine_nodes=fine_rank,
                    member_fine_nodes=n0_list)
        fine_rows = fine_rows.to(dev)
    g = gb.to(dev)
    model = model_cpu.to(dev)
    model.engine = "hip"

    from mswegnn.engine import plan_for
    from mswegnn import _lib
    t_plan = time.perf_counter()
    plan = plan_for(model, g)
    torch.cuda.synchronize()
    t_plan = time.perf_counter() - t_plan
    out = torch.empty(g.num_nodes, 2, T, device=dev)
    # the all-gather runs on the GPU over RCCL; gloo (rehearsal) gathers host copies
    gather = make_gatherer(dist, world, fine_rank, T, dev if backend == "nccl" else torch.device("cpu"))

    if args.caller == "fused":
        def rollout():
            plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, T, out=out)
            return out
    else:
        from mswegnn.rollout import apply_boundary_condition, use_prediction
        dyn = model.previous_t * model.NUM_WATER_VARS

        def rollout(fwd=model):  # training/train.py:87-95 verbatim semantics, model(temp) -> msw_forward
            temp = g.clone()
            preds = []
            with torch.no_grad():
                for t in range(T):
                    temp.x[:, -dyn:] = apply_boundary_condition(temp.x[:, -dyn:], temp.BC[:, :, t],
                                                                temp.node_BC, type_BC=temp.type_BC)
                    pred = fwd(temp)
                    temp.x = use_prediction(temp.x, pred, model.previous_t)
                    preds.append(pred)
            return torch.stack(preds, -1)

    def one_step():
        r = rollout()
        if world > 1:
            gather(r[:n0] if fine_rows is None else r.index_select(0, fine_rows))

    t_first = None
    for i in range(args.warmup):
        t0 = time.perf_counter()
        one_step()
        if i == 0:
            torch.cuda.synchronize()
            t_first = time.perf_counter() - t0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        red_dev = dev if backend == "nccl" else torch.device("cpu")
        tt = torch.tensor([dt], device=red_dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_per_step = dt / max(args.steps, 1) * 1e3
    nodes_all = fine_rank  # fine nodes simulated per step, summed over ranks (meshes may differ)
    if world > 1:
        tn = torch.tensor([fine_rank], device=red_dev, dtype=torch.float64)
        dist.all_reduce(tn, op=dist.ReduceOp.SUM)
        nodes_all = float(tn.item())
    value = nodes_all * T * args.steps / dt

    caller_overhead = None
    if args.caller == "reference-loop" and world == 1:
        # the caller's own cost: the same loop with the model replaced by a stub that returns a
        # fresh [N, 2] tensor (no GPU work): its index_put / slice copy / cat kernels and its
        # per-step host synchronisation (check_type_BC reads the GPU tensor type_BC)
        def stub(temp):
            return torch.zeros(temp.x.shape[0], 2, device=temp.x.device)
        rollout(stub)
        torch.cuda.synchronize()
        c0 = time.perf_counter()
        for _ in range(3):
            rollout(stub)
        torch.cuda.synchronize()
        tc = (time.perf_counter() - c0) / 3
        caller_overhead = {"ms_per_rollout": tc * 1e3, "us_per_step": tc / T * 1e6,
                           "note": "the reference loop with a no-op model (stub returning zeros): "
                                   "what the caller itself costs per step"}

    result = None
    if rank == 0:
        st = plan.stats()
        # ---------------- roofline: aggregation (hop) kernel at the finest scale
        F = desc["hid_features"]
        t_hop, (rows, edges) = time_kernel(plan, "hop", 0)
        hop_bytes = edges * (4 * F + 4) + rows * (12 * F + 4)
        t_eh, (_, e_eh) = time_kernel(plan, "edge_hop", 0)
        mlp_flops = e_eh * 2 * (2 * F * 2 * F + 2 * F * F)  # edge-MLP layers 2-3 on MFMA
        try:  # small coarse scales pool inside their first edge hop (no pooling launch)
            t_pool, (r_pool, _) = time_kernel(plan, "pool", 1) if desc["num_scales"] > 1 else (0.0, (0, 0))
            pool_rec = {"avg_launch_us": t_pool * 1e6, "rows": r_pool}
        except _lib.EngineError:
            pool_rec = {"fused": "mean pooling into scale 1 runs inside scale 1's first edge-MLP + hop launch"}
        # the PMC summary holds the default workload's finest hop ("k_hop") and the config-5
        # mesh's ("k_hop_large"); other workloads have no committed counter pass
        pmc_key = {"zenodo4": "k_hop", "hbm1m": "k_hop_large"}.get(args.workload) if B == 1 else None
        lib_sha = _lib.lib_info()["sha256"]
        pmc_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
        traffic_rec = read_traffic(pmc_path, pmc_key, lib_sha) if pmc_key else None
        traffic = traffic_rec["bytes_per_launch"] if traffic_rec else None
        roof = {"kernel": "k_hop<32> (SWEGNN hop: CSR pull + filter), finest scale",
                "bound": "hbm", "achieved": hop_bytes / t_hop / 1e9, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": hop_bytes / t_hop / 1e9 / HBM_PEAK_GBS,
                "traffic": traffic, "traffic_source": traffic_rec, "algorithmic_bytes_per_launch": hop_bytes,
                "avg_launch_us": t_hop * 1e6, "rows": rows, "edges": edges,
                "timer": "HIP events on the launching stream around 200 back-to-back launches: "
                         "launch-to-launch period (kernel + boundary); rocprof = rocprofv3 kernel "
                         "durations from the committed trace summary of this command "
                         "(tools/roofline_check.py), on the library named by its source_library_sha256 "
                         "(stale = measured on another build than the one loaded now)",
                "other_kernels": {
                    "k_edge_hop<32> (edge MLP + hop 1)": {
                        "avg_launch_us": t_eh * 1e6, "edges": e_eh,
                        "achieved_tflops": mlp_flops / t_eh / 1e12,
                        "peak_tflops": FP32_MFMA_PEAK_TFS},
                    "k_pool<32> (mean pool + projection), scale 1": pool_rec}}
        # ---------------- the launch floor the zenodo-size hop is bound by: one dependent
        # gather of the previous launch's rows (torch.index_select, same rows x F) per launch
        # of a captured 35-launch graph (tools/launch_floor.py)
        try:  # optional: a failure here is recorded, never drops the result line
            if world == 1:
                sys.path.insert(0, os.path.join(ROOT, "tools"))
                import launch_floor as lf
                small = torch.ones(1024, device=dev)
                perm = torch.randperm(rows, device=dev)
                bufs = [torch.randn(rows, F, device=dev), torch.empty(rows, F, device=dev)]
                flip = {"i": 0}

                def _gather():
                    i = flip["i"]
                    torch.index_select(bufs[i], 0, perm, out=bufs[1 - i])
                    flip["i"] = 1 - i
                roof["launch_floor"] = {
                    "trivial_us": lf.per_launch_us(lambda: small.mul_(1.0), 35),
                    "dependent_row_gather_us": lf.per_launch_us(_gather, 35),
                    "note": "per launch, 35 dependent launches in one graph; the gather reads the "
                            "previous launch's rows (same rows x F as the roofline hop)"}
                del small, perm, bufs
        except Exception as e:  # noqa: BLE001
            roof["launch_floor"] = {"error": repr(e)}
        # ---------------- the same hop kernel where HBM, not latency, bounds it: the ~1M-node
        # mesh of config 5 (fully wet; one rollout step to populate the buffers)
        try:  # optional: a failure here is recorded, never drops the result line
            if world == 1 and not args.no_roofline_large and args.workload != "hbm1m":
                gl, ml, _, dl = build_workload("hbm1m", seed=0, T=1)
                gl = gl.to(dev)
                ml = ml.to(dev)
                ml.engine = "hip"
                pl = plan_for(ml, gl)
                pl.rollout(gl.x, gl.BC, gl.node_BC, gl.type_BC, 1)
                tl, (rl, el) = time_kernel(pl, "hop", 0, iters=50)
                bl = el * (4 * F + 4) + rl * (12 * F + 4)
                # the edge-MLP kernel on the same mesh: fused edge MLP + hop 1, finest scale.
                # Two ceilings: MFMA (edge-MLP layers 2-3, fp32) and HBM -- per edge U[src] (2F),
                # the edge term Pe (2F), out[src] (F) read, s (F) stored, the 16-B lane record;
                # per node V (2F), the hop input (F) read, the result (F) stored.  The bound
                # reported is the ceiling it sits closer to.
                tle, (rle, ele) = time_kernel(pl, "edge_hop", 0, iters=20)
                fle = ele * 2 * (2 * F * 2 * F + 2 * F * F)
                ble = ele * (24 * F + 16) + rle * 16 * F
                mf = {"flops_per_launch": fle, "achieved": fle / tle / 1e12, "peak": FP32_MFMA_PEAK_TFS,
                      "unit": "TFLOP/s", "frac": fle / tle / 1e12 / FP32_MFMA_PEAK_TFS}
                hb = {"algorithmic_bytes_per_launch": ble, "achieved": ble / tle / 1e9, "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": ble / tle / 1e9 / HBM_PEAK_GBS,
                      "traffic": read_traffic(pmc_path, "k_edge_hop_large"),
                      "traffic_source": read_traffic(pmc_path, "k_edge_hop_large", lib_sha)}
                roof["large_mesh"] = {
                    "workload": "hbm1m", "fine_nodes": dl["fine_nodes"], "rows": rl, "edges": el,
                    "algorithmic_bytes_per_launch": bl, "avg_launch_us": tl * 1e6,
                    "achieved": bl / tl / 1e9, "frac": bl / tl / 1e9 / HBM_PEAK_GBS,
                    "traffic": read_traffic(pmc_path, "k_hop_large"),
                    "traffic_source": read_traffic(pmc_path, "k_hop_large", lib_sha),
                    "edge_mlp": {"kernel": "k_edge_hop<32> (edge MLP + hop 1), finest scale",
                                 "bound": "hbm" if hb["frac"] >= mf["frac"] else "mfma",
                                 "edges": ele, "rows": rle, "avg_launch_us": tle * 1e6, "mfma": mf, "hbm": hb}}
                del pl, ml, gl
                torch.cuda.empty_cache()
        except Exception as e:  # noqa: BLE001
            roof["large_mesh"] = {"error": repr(e)}
        # the same kernels' durations from the committed rocprofv3 trace of this command
        # (kernel time without the launch boundary the HIP-event period includes)
        try:
            if args.workload == "zenodo4" and B == 1:
                with open(os.path.join(ROOT, "profiles", "roofline_rocprof.json")) as f:
                    rpd = json.load(f)
                rp = rpd["by_role"]
                rr = summary_provenance(rpd, lib_sha)
                if "hop" in rp:
                    d = rp["hop"]["avg_duration_us"] * 1e-6
                    rr["hop"] = {"kernel": rp["hop"]["kernel"], "avg_duration_us": d * 1e6,
                                 "achieved": hop_bytes / d / 1e9, "frac": hop_bytes / d / 1e9 / HBM_PEAK_GBS}
                lm = roof.get("large_mesh", {})
                if "hop_large" in rp and "algorithmic_bytes_per_launch" in lm:
                    d = rp["hop_large"]["avg_duration_us"] * 1e-6
                    bl = lm["algorithmic_bytes_per_launch"]
                    rr["hop_large"] = {"kernel": rp["hop_large"]["kernel"], "avg_duration_us": d * 1e6,
                                       "achieved": bl / d / 1e9, "frac": bl / d / 1e9 / HBM_PEAK_GBS}
                roof["rocprof"] = rr
        except (OSError, KeyError, ValueError) as e:
            roof["rocprof"] = {"error": repr(e)}
        # ---------------- parity vs the reference fixture (zenodo4 only; CPU reference run)
        parity = {}
        r_gpu = plan.rollout(g.x, g.BC, g.node_BC, g.type_BC, T).cpu()
        try:  # optional: a failure here is recorded, never drops the result line
            if args.workload == "zenodo4" and rank == 0 and T == 48 and B == 1:
                fx = np.load(os.path.join(ROOT, "tests", "golden", "fx_zenodo4_K4_F32_rollout48.npz"))
                ref = torch.from_numpy(fx["rollout_sel"])
                sel = r_gpu[..., fx["steps"]]
                parity["vs_reference_fixture"] = {
                    "steps": fx["steps"].tolist(), "max_abs_err": float((sel - ref).abs().max()),
                    "max_rel_err": float(max((sel[..., i] - ref[..., i]).abs().max() / ref[..., i].abs().max()
                                             for i in range(ref.shape[-1])))}
            # ---------------- CPU baseline (reference algorithm on the host cores)
        except Exception as e:  # noqa: BLE001
            parity["vs_reference_fixture"] = {"error": repr(e)}
        cpu = None
        try:  # optional: a failure here is recorded, never drops the result line
            if world == 1 and not args.no_cpu_baseline:
                sys.path.insert(0, os.path.join(ROOT, "oracle"))
                import msgnn_torch as orc  # test/baseline infrastructure only
                host_cores, share = cpu_share()
                threads = share
                torch.set_num_threads(threads)
                P = {k: v.detach().cpu() for k, v in model_cpu.state_dict().items()}
                cfg = orc.msgnn_config(num_scales=desc["num_scales"], hid_features=F, K=desc["K"])
                # bounded sample: one step first, then as many rollout steps of simulation 0 as
                # fit ~cpu_seconds (whole rollouts repeated for small meshes, up to 4)
                c0 = time.perf_counter()
                orc.rollout(P, cfg, g_cpu, 1)
                t1 = time.perf_counter() - c0
                Tc = int(min(T, max(1, args.cpu_seconds / max(t1, 1e-6))))
                reps, t_cpu, r_cpu = 0, 0.0, None
                while reps < 4 and (reps == 0 or t_cpu < args.cpu_seconds):
                    c0 = time.perf_counter()
                    r = orc.rollout(P, cfg, g_cpu, Tc)
                    t_cpu += time.perf_counter() - c0
                    reps += 1
                    r_cpu = r if r_cpu is None else r_cpu
                    if Tc < T:
                        break
                cpu = {"value": n0 * Tc * reps / t_cpu, "unit": "fine-node-steps/s", "cores": threads,
                       "kind": "port",
                       "sample": f"{reps} x {Tc}-step rollout of one simulation of the workload "
                                 f"(N0={n0}), reference algorithm in oracle/msgnn_torch.py (same ATen "
                                 f"CPU ops, bit-identical to the reference), torch {torch.__version__}, "
                                 f"{threads} threads, {t_cpu:.1f} s",
                       "host_cores": host_cores,
                       "threads_note": CPU_SHARE_NOTE}
                if B > 1:
                    # the reference evaluates batches of simulations (test_model.py:37): on the host
                    # that is one simulation per process over the CPU share
                    try:
                        cpu["batch"] = cpu_batch_baseline(args.workload, ids, T, share, args.cpu_seconds, t1, threads)
                    except Exception as e:  # noqa: BLE001
                        cpu["batch"] = {"error": repr(e)}
                r0 = r_gpu[:g_cpu.num_nodes, :, :Tc]  # simulation 0 = the batch's first graph
                d = (r0 - r_cpu).abs()
                parity["vs_cpu_reference"] = {
                    "steps": Tc, "max_abs_err": float(d.max()),
                    "max_rel_err": float(max(d[..., t].max() / max(r_cpu[..., t].abs().max(), 1e-30)
                                             for t in range(Tc)))}
        except Exception as e:  # noqa: BLE001
            cpu = {"error": repr(e)}
        result = {
            "metric": "mesh-nodes x rollout-steps / sec (fine-scale nodes); fp32 max-abs err vs CPU ref",
            "value": value, "unit": "fine-node-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step,
            "ms_per_rollout": ms_per_step / B, "us_per_timestep": ms_per_step * 1e3 / T,
            "step_note": "one bench step = one T-step rollout of this rank's simulation(s): ms_per_step = "
                         "ms per rollout call (ms_per_rollout: per simulation of the batch), "
                         "us_per_timestep = one autoregressive time step of the whole batch",
            "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (own multi-scale triangular mesh generator; dry start + hydrograph BC)",
            "config": dict(desc, caller=args.caller, global_batch=args.global_batch or None,
                           parallelism=f"sim-sharded x{world} ({B} sim on rank 0, "
                           f"{'RCCL' if backend == 'nccl' else backend} all-gather at end)"
                           if world > 1 else ("single GPU" if B == 1 else f"single GPU, batch of {B} sims")),
            "timed_region": "whole rollouts (T steps each) incl. the per-rollout edge encoder + edge "
                            "terms of every processor (msw_rollout prologue); inputs resident in HBM",
            "library": dict(_lib.lib_info(), built_from_current_sources=_built_from_sources()),
            "msw_env": msw_env(),
            "all_node_steps_per_s": value * desc.get("batch_nodes", desc["all_nodes"]) / fine_rank,
            "roofline": roof, "cpu_baseline": cpu, "parity": parity,
            "engine": {"kernels_per_step": st["kernels_per_step"], "graph_captured": st["graph_captured"],
                       "device_bytes": st["device_bytes"],
                       "device_bytes_note": "plan-owned: graph tables, weights, per-node buffers and the "
                                            "edge-encoder inputs / outputs kept for the per-rollout "
                                            "recompute of the edge terms",
                       "plan_build_s": t_plan, "first_rollout_s": t_first,
                       "setup_note": "once per mesh, outside the timed region: plan_build_s = host graph "
                                     "tables (CSR, tiles, exchange lists) + uploads + first-use kernel "
                                     "setup; first_rollout_s = the first warmup rollout incl. its "
                                     "hipGraph capture"},
        }
        if caller_overhead is not None:
            result["caller_overhead"] = caller_overhead
    if world > 1:
        # the north star's strong scaling (fixed config-3 sets, rank 0 alone vs all ranks with
        # the RCCL all-gather), the RCCL single-mesh decomposition and DDP training: after the
        # weak line's timed region and its rank-0 records, inside --extras-budget, never fatal
        def cpu_barrier():
            dist.barrier(group=cpu_group)
        extras = run_extras(dist, rank, world, dev, args, cpu_barrier, backend, group=cpu_group)
        if rank == 0:
            result.update(extras)
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
