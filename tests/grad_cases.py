"""Gradient cases of the reference-made fixtures (oracle/gen_golden_grad.py), runnable on any
device and engine: the CPU tests run the drop-in's torch path, the GPU tests the HIP training
kernels (mswegnn/autograd.py).  Each returns {name: tensor} in the fixture's key names.

Reference: SWEGNN.forward models/gnn.py:387-445, MSGNN.forward :267-350,
LightningTrainer.training_step training/train.py:125-145, loss_function training/loss.py:76-118.
"""
import numpy as np
import torch

from conftest import build_gnn, build_msgnn, golden, graph_digest, manifest, rel_err, weights

import loss_ref  # oracle/: the reference's loss and training step, restated


def grad_graph(name, T):
    """A fixture graph regenerated from its mesh arguments (manifest 'grad_graphs')."""
    from mswegnn.mesh import make_multiscale_mesh, make_single_scale_mesh, wet_state
    kind, kw, wet = manifest()["grad_graphs"][name]
    g = make_multiscale_mesh(**kw, T=T) if kind == "msgnn" else make_single_scale_mesh(**kw, T=T)
    return wet_state(g, seed=wet)


def processor_case(dev, train_engine="auto"):
    """gnn_processor[0], [2] and intra_scale_gnn[2] of K4_F32: out, input and parameter
    gradients of sum(out * wout)."""
    fx = golden("fx_grad_processor_K4_F32")
    g = grad_graph("tiny4", 4)
    assert np.array_equal(graph_digest(g), fx["digest"])
    m = build_msgnn(4, 32, 4, state=weights("K4_F32")).to(dev)
    x_s, x_d, ea, wout = (torch.from_numpy(fx[k]).to(dev) for k in ("x_s", "x_d", "edge_attr", "wout"))
    ep, iep = g.edge_ptr, g.intra_edge_ptr
    ei, iei = g.edge_index.to(dev), g.intra_mesh_edge_index.to(dev)
    cases = {"proc0": (m.gnn_processor[0], ei[:, ep[0]:ep[1]], ea[ep[0]:ep[1]]),
             "proc2": (m.gnn_processor[2], ei[:, ep[2]:ep[3]], ea[ep[2]:ep[3]]),
             "intra2": (m.intra_scale_gnn[2], iei[:, iep[0]:iep[1]], None)}
    out = {}
    for name, (layer, e_idx, e) in cases.items():
        layer.train_engine = train_engine
        layer.zero_grad(set_to_none=True)
        xs = x_s.clone().requires_grad_(True)
        xd = x_d.clone().requires_grad_(True)
        ee = e.clone().requires_grad_(True) if e is not None else None
        y = layer(xs, xd, e_idx, ee)
        (y * wout).sum().backward()
        out[f"{name}__out"] = y.detach()
        out[f"{name}__d_x_s"] = xs.grad
        out[f"{name}__d_x_d"] = xd.grad
        if ee is not None:
            out[f"{name}__d_edge_attr"] = ee.grad
        for n, p in layer.named_parameters():
            out[f"{name}__g__{n}"] = p.grad
        layer.train_engine = "auto"
    return out, fx


def msgnn_mse_case(dev, engine="auto"):
    """MSGNN (K4_F32) with an MSE loss against the fixture's target: every parameter gradient."""
    fx = golden("fx_grad_msgnn_K4_F32")
    g = grad_graph("tiny4", 4)
    assert np.array_equal(graph_digest(g), fx["digest"])
    m = build_msgnn(4, 32, 4, state=weights("K4_F32")).to(dev).train()
    m.engine = engine
    tgt = torch.from_numpy(fx["tgt"]).to(dev)
    y = m(g.to(dev))
    loss = ((y - tgt) ** 2).mean()
    loss.backward()
    out = {"y": y.detach(), "loss": loss.detach()}
    out.update({"g__" + n: p.grad for n, p in m.named_parameters() if p.grad is not None})
    return out, fx


def training_batch(prefix_y, names, T, fx, dev, dtype=torch.float32):
    """The fixture's PyG-style batch: members regenerated, targets y from the fixture, collated
    (mswegnn.batch, PyG semantics) and adapted as training_step does (train.py:130)."""
    from mswegnn.batch import collate
    from mswegnn.rollout import adapt_batch_training
    gs = []
    for n in names:
        g = grad_graph(n, T)
        g.y = torch.from_numpy(fx[f"{prefix_y}y_{n}"])
        gs.append(g)
    b = collate(gs)
    for k in ("x", "edge_attr", "BC", "y"):
        setattr(b, k, getattr(b, k).to(dtype))
    return adapt_batch_training(b.to(dev))


def training_step_case(dev, sname, R, engine="auto", dtype=torch.float32, model=None):
    """The reference's training_step (config.yaml trainer_options) on the fixture's batch
    `sname` ('b1': one graph, 'b2': two) with R rollout steps -> (loss, gradients)."""
    fx = golden("fx_grad_train_K4_F32")
    names = manifest()["fx_grad_train_K4_F32_sets"][sname]
    m = model if model is not None else build_msgnn(4, 32, 4, state=weights("K4_F32"))
    m = m.to(dev).to(dtype).train()
    m.engine = engine
    m.zero_grad(set_to_none=True)
    temp = training_batch(f"{sname}__", names, 5, fx, dev, dtype)
    loss = loss_ref.training_step(m, temp, R)
    loss.backward()
    out = {"loss": loss.detach()}
    out.update({"g__" + n: p.grad for n, p in m.named_parameters() if p.grad is not None})
    return out, fx


def f64_training_step_case(dev, R=4, engine="auto"):
    """config.yaml's default width F = 64 (mlp_layers 3, K 4): the reference's training_step
    on the two-graph batch from the seeded initialisation (seed 666), whose state dict must
    match the reference's bit for bit (fixture digest) -> (loss, gradients)."""
    import hashlib
    fx = golden("fx_grad_train_F64")
    names = manifest()["fx_grad_train_F64_sets"]["b2"]
    m = build_msgnn(4, 64, 4)
    h = hashlib.sha256()
    for v in m.state_dict().values():
        h.update(v.detach().float().contiguous().numpy().tobytes())
    assert np.frombuffer(h.digest(), dtype=np.uint8).tolist() == fx["sd_digest"].tolist(), \
        "seeded F = 64 init differs from the reference's"
    m = m.to(dev).train()
    m.engine = engine
    m.zero_grad(set_to_none=True)
    temp = training_batch("b2__", names, 5, fx, dev)
    loss = loss_ref.training_step(m, temp, R)
    loss.backward()
    out = {"loss": loss.detach()}
    out.update({"g__" + n: p.grad for n, p in m.named_parameters() if p.grad is not None})
    return out, fx


def zenodo4_graph(T=5):
    """The zenodo4 mesh of fx_grad_train_zenodo4 (bench.py's config-2 workload, dry start)."""
    from mswegnn.mesh import make_multiscale_mesh
    kind, kw, wet = manifest()["fx_grad_train_zenodo4_graph"]
    assert kind == "msgnn" and wet is None
    return make_multiscale_mesh(**kw, T=T)


def zenodo4_batch(dev, dtype=torch.float32):
    """The fixture's one-graph batch, adapted as training_step does (train.py:127)."""
    from mswegnn.batch import collate
    from mswegnn.rollout import adapt_batch_training
    fx = golden("fx_grad_train_zenodo4")
    g = zenodo4_graph()
    assert np.array_equal(graph_digest(g), fx["digest"])
    g.y = torch.from_numpy(fx["y"])
    b = collate([g])
    for k in ("x", "edge_attr", "BC", "y"):
        setattr(b, k, getattr(b, k).to(dtype))
    return adapt_batch_training(b.to(dev)), int(g.node_ptr[1]), fx


def zenodo4_training_step_case(dev, R, engine="auto", dtype=torch.float32, premask=None, record=None):
    """BASELINE config 2 at the bench's size: the reference's training_step on the zenodo4 mesh
    (K4_F32, one-graph batch, R rollout steps) -> (loss, gradients).  `premask`, a list, receives
    the fine-scale decoder output entering _mask_small_WD at every rollout step (the quantity
    whose side of the 1e-4 threshold decides a fork).  `record`, a list, receives the tape of
    every discrete decision the run took, in call order (mswegnn.autograd.RECORD for the HIP
    training kernels, plus the relu'd output of each forward): what msgnn_torch.following
    replays in float64 (oracle_zenodo4_step(tape=...))."""
    from mswegnn import autograd as ag
    temp, n0, fx = zenodo4_batch(dev, dtype)
    m = build_msgnn(4, 32, 4, state=weights("K4_F32")).to(dev).to(dtype).train()
    m.engine = engine
    if premask is not None or record is not None:
        orig = type(m)._mask_small_WD

        def recording(self, x, epsilon=0.001):
            if premask is not None:
                premask.append(x.detach()[:n0].clone())
            if record is not None:
                record.append({"kind": "out", "x": x.detach().clone()})
            return orig(self, x, epsilon)
        m._mask_small_WD = recording.__get__(m)
    m.zero_grad(set_to_none=True)
    ag.RECORD = record
    try:
        loss = loss_ref.training_step(m, temp, R)
    finally:
        ag.RECORD = None
    loss.backward()
    out = {"loss": loss.detach()}
    out.update({"g__" + n: p.grad for n, p in m.named_parameters() if p.grad is not None})
    return out, fx


def mask_forks(premask, fx, eps=1e-4):
    """Cells where _mask_small_WD (models/models.py:79-91) decides differently than in the
    reference's float64 run, per rollout step of the R = 4 training rollout.  Its two
    discontinuities: the depth mask h * (|h| > eps) and the velocity mask v * (h != 0), h being
    the depth after the ReLU (gnn.py:345) -- so a pre-ReLU depth on the other side of 0 switches
    the cell's whole velocity on or off.  -> [(step, fine row, kind, ours h, fp64 h)]."""
    ref = np.asarray(fx["R4_fp64__premask_wd_f64"])
    forks = []
    for t, x in enumerate(premask):
        h = x[:, 0].detach().double().cpu().numpy()
        r = ref[:, t]
        for kind, a, b in (("depth", np.abs(h) > eps, np.abs(r) > eps), ("velocity", h != 0, r != 0)):
            for i in np.nonzero(a != b)[0]:
                forks.append((t, int(i), kind, float(h[i]), float(r[i])))
    return forks


def gnn_training_step_case(dev, R, engine="auto"):
    """training_step of the 1-scale GNN (config 1 model) on a batch of two graphs."""
    fx = golden("fx_grad_train_gnn")
    m = build_gnn(state=weights("gnn_F32_seed42")).to(dev).train()
    m.engine = engine
    m.zero_grad(set_to_none=True)
    temp = training_batch("", ["g1_0", "g1_1"], 3, fx, dev)
    loss = loss_ref.training_step(m, temp, R)
    loss.backward()
    out = {"loss": loss.detach()}
    out.update({"g__" + n: p.grad for n, p in m.named_parameters() if p.grad is not None})
    return out, fx


def compare(ours, fx, prefix, keys=None):
    """{key: rel err} of ours[key] against fx[prefix + key] (every gradient the fixture holds
    under `prefix`, which must all be present in ours)."""
    want = [k[len(prefix):] for k in fx if k.startswith(prefix)] if keys is None else keys
    errs = {}
    for k in want:
        if not (k in ("out", "y", "loss") or k.startswith(("g__", "d_"))):
            continue  # inputs, targets, digests
        mine = ours.get(k, ours.get(prefix + k))
        assert mine is not None, f"missing {prefix}{k}"
        errs[k] = rel_err(mine, torch.from_numpy(np.asarray(fx[prefix + k])))
    return errs


def global_rel(ours, fx, prefix):
    """Global relative L2 difference over every parameter gradient ('g__*')."""
    num = den = 0.0
    for k in fx:
        if k.startswith(prefix + "g__"):
            ref = torch.from_numpy(fx[k]).double()
            a = ours[k[len(prefix):]].detach().double().cpu()
            num += float(((a - ref) ** 2).sum())
            den += float((ref ** 2).sum())
    return (num / den) ** 0.5


def check(ours, fx, prefix, tol, fp64_prefix=None, slack=3.0, floor=1e-2, floor_rel=1e-2, noise=None):
    """The gradient bar, per parameter tensor (max-abs relative: max|ours - ref| / max|ref|):
    1. within `tol` of the reference's fp32 result; or
    2. (`floor`) an absolute error within tol x floor x the largest gradient entry of the
       model -- i.e. atol = 1e-6 x max|g| at the defaults, ten times tighter than
       torch.testing's float32 atol: tensors whose gradient is ~1e-4 of the model's (a PReLU
       slope or a bias summed over every edge with cancellation) are resolved only to ~1e-4
       relative by ANY fp32 summation order (the reference's own fp32 run: up to 1.8e-4) --
       and still within `floor_rel` relative, with the sign of the reference's largest entry:
       a small tensor that is zero, or of the wrong sign, does not pass here; or
    3. (the fp64 rule) no further from the reference's float64 result than `slack` x the
       reference's OWN fp32 run is (a rollout the fp32 reference cannot resolve: a mask flip of
       _mask_small_WD forks it) -- or (`noise`, reference_fp32_noise) than `slack` x the
       farthest of an ensemble of the reference's arithmetic in fp32 on one-ulp-perturbed
       inputs.  Nothing of ours is a yardstick.
    Returns (worst error vs fp32, {tensor: how it passed past rule 1}); asserts.  The tensors
    passed by rule 2 or 3 are printed."""
    errs = compare(ours, fx, prefix)
    worst = max(errs.values())
    big = max((float(np.abs(fx[prefix + k]).max()) for k in errs if k.startswith("g__")), default=0.0)
    rule64, bad = {}, {}
    for k, e in errs.items():
        if e <= tol:
            continue
        ref = np.asarray(fx[prefix + k])
        e_abs = e * float(np.abs(ref).max())
        if floor and k.startswith("g__") and e_abs <= tol * floor * big and e <= floor_rel:
            mine = ours.get(k, ours.get(prefix + k)).detach().double().cpu().numpy().reshape(-1)
            i = int(np.abs(ref).reshape(-1).argmax())
            if np.sign(mine[i]) == np.sign(ref.reshape(-1)[i]):
                rule64[k] = ("floor", e, e_abs / big)
                continue
        if fp64_prefix is None or (fp64_prefix + k) not in fx:
            bad[k] = e
            continue
        ref64 = torch.from_numpy(fx[fp64_prefix + k])
        e_o = rel_err(ours.get(k, ours.get(prefix + k)), ref64)
        e_r = rel_err(torch.from_numpy(ref), ref64)
        if noise is not None and k in noise:
            e_r = max(e_r, noise[k])
        rule64[k] = ("fp64", e_o, e_r)
        if not e_o <= max(tol, slack * e_r):
            bad[k] = (e, e_o, e_r)
    if rule64:
        print(f"{prefix}: past rule 1 -> {rule64}")
    assert not bad, (prefix, bad)
    return worst, rule64


def oracle_training_step(temp, P, cfg, R, tape=None, record=False):
    """The reference's training_step through the oracle restatement (oracle/msgnn_torch.py,
    loss_ref.py) on an adapted batch `temp`, weights P {state-dict name: tensor} in the dtype of
    the run -- following `tape` or recording its own decisions (record=True; see
    msgnn_torch.following) -> (loss, gradients, the following context)."""
    import msgnn_torch as orc
    P = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}

    class Model:  # loss_ref.training_step's view of a model
        previous_t = 3
        NUM_WATER_VARS = 2

        def __call__(self, graph):
            return orc.msgnn_forward(P, cfg, graph)
    with orc.following(None if record else tape) as fl:
        loss = loss_ref.training_step(Model(), temp, R)
    loss.backward()
    return loss.detach(), {"g__" + k: p.grad.float() for k, p in P.items() if p.grad is not None}, fl


def oracle_zenodo4_step(R, dtype, tape=None, record=False):
    """oracle_training_step on the zenodo4 fixture's batch (CPU, `dtype`)."""
    import msgnn_torch as orc
    temp, _, _ = zenodo4_batch(torch.device("cpu"), dtype)
    P = {k: v.to(dtype) for k, v in weights("K4_F32").items()}
    return oracle_training_step(temp, P, orc.msgnn_config(num_scales=4, hid_features=32, K=4), R, tape, record)


# the ensemble may widen a tensor's bar to at most this multiple of the fixture's own fp32 run's
# distance from float64 (the noise must not loosen the bar by orders of magnitude)
NOISE_CAP = 4.0


def reference_fp32_noise(make_batch, P, cfg, R, fx, p64, n=6, seed=0, p32=None, cap=NOISE_CAP):
    """How far the REFERENCE's arithmetic in fp32 lands from its float64 result per gradient
    tensor, over an ensemble: the oracle restatement (bit-identical to the reference on CPU) run
    n times in fp32 on the batch's float inputs perturbed by one ulp at random (x, edge_attr,
    BC) -- each run another equally valid fp32 rounding of the same problem.  Exact zeros stay
    zero: a dry start's zeros decide the hop predicate and the loss's water mask, so moving them
    to a subnormal would pose a different problem, not round the same one.  One run (the
    fixture's) is one sample of that noise; a tensor whose sum cancels heavily (a PReLU slope
    sums every element of its layer) spreads over a range no fp32 implementation can be held
    below.  With `p32` (the fixture's fp32 prefix) each tensor's spread is capped at `cap` x
    the fixture's own fp32 distance from fp64.
    -> {tensor: max over the ensemble of max|run - fp64| / max|fp64|}."""
    gen = torch.Generator().manual_seed(seed)
    worst = {}
    for _ in range(n):
        temp = make_batch()
        for k in ("x", "edge_attr", "BC"):
            v = getattr(temp, k)
            bump = torch.randint(0, 3, v.shape, generator=gen).to(v.device) - 1  # -1 / 0 / +1 ulp
            bump = torch.where(v == 0, torch.zeros_like(bump), bump)
            setattr(temp, k, torch.where(bump > 0, torch.nextafter(v, v.new_tensor(float("inf"))),
                                         torch.where(bump < 0, torch.nextafter(v, v.new_tensor(float("-inf"))), v)))
        _, g, _ = oracle_training_step(temp, {k: v.float() for k, v in P.items()}, cfg, R)
        for k, v in g.items():
            if p64 + k in fx:
                worst[k] = max(worst.get(k, 0.0), rel_err(v, torch.from_numpy(fx[p64 + k])))
    if p32 is not None:
        for k in list(worst):
            if p32 + k in fx:
                own = rel_err(torch.from_numpy(np.asarray(fx[p32 + k])), torch.from_numpy(fx[p64 + k]))
                worst[k] = min(worst[k], cap * own)
    return worst


def as_fixture(grads, prefix="X__"):
    """{g__name: tensor} -> {prefix + g__name: ndarray} (compare / global_rel against it)."""
    return {prefix + k: v.detach().cpu().numpy() for k, v in grads.items()}


# a decision whose float64 value lies this close to its threshold is "within rounding" of it:
# the values are O(1) (pre-activations, depths), fp32 dot products of 64 terms round at ~1e-6
FLIP_DIST = 1e-5
