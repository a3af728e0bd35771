"""The drop-in against the reference's own callers (build container only).

Runs in a subprocess the way a user would switch a reference checkout over: the working
directory and the script's sys.path entry are the reference checkout, and ``mswe-gnn_amd/``
is merely on the path (PYTHONPATH).  Import-only stand-ins for the third-party packages
absent from this image (torch_geometric, lightning, wandb, networkx, the mesh library behind
``database``) come from oracle/refstubs.  Checks:

* the import lines of test_model.py:1-13 and main.py:1-16, read from the files themselves,
  all execute; ``models`` resolves to the drop-in, ``training`` / ``utils`` to the reference;
* ``get_model('MSGNN')(**config.yaml models:)`` builds the drop-in MSGNN (hid_features 64);
* the reference's own ``rollout_test`` (single graph and a 2-graph PyG Batch through its
  ``adapt_batch_training`` / ``update_batch_multiscale``) on the drop-in model matches the
  oracle;
* ``MSWEGNN_FUSED_ROLLOUT=1`` swaps ``training.train.rollout_test`` for the fused one in both
  import orders, and ``LightningTrainer.predict_step`` (train.py:182-185) returns the same
  per-graph pieces as the reference's loop.

Skipped when /root/reference is absent (the GPU box).
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, PKG

REF = "/root/reference"
STUBS = os.path.join(ROOT, "oracle", "refstubs")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "models")),
                                reason="reference checkout not present (GPU box)")

DRIVER = r'''
import json, os, sys
REF, STUBS, ROOT, PKG, ORDER = sys.argv[1:6]
# python script.py in the reference checkout: the script directory leads sys.path; the
# stand-ins for absent third-party packages go in front of it, the drop-in stays behind
sys.path[:0] = [STUBS, REF]
sys.path.append(PKG)
sys.path.append(os.path.join(ROOT, "oracle"))
import torch
res = {}

def import_lines(path, last):
    src = open(os.path.join(REF, path)).read().splitlines()[:last]
    return [l for l in src if l.startswith(("import ", "from "))]

if ORDER == "train_first":
    import training.train  # imports models while training.train is half-initialised
for path, last in (("test_model.py", 13), ("main.py", 16)):
    for line in import_lines(path, last):
        exec(line)
    res[path] = "ok"

import models.gnn, training.train, utils.dataset, utils.miscellaneous, utils.load
res["models"] = models.gnn.__file__
res["training"] = training.train.__file__
res["utils"] = utils.dataset.__file__
res["caller_symbols"] = all(hasattr(training.train, n) for n in
                            ("LightningTrainer", "DataModule", "CurriculumLearning", "rollout_test"))

cfg = read_config(os.path.join(REF, "config.yaml"))
mp = dict(cfg["models"])
model_type = mp.pop("model_type")
model = get_model(model_type)(num_node_features=8, num_edge_features=1, previous_t=3, device="cpu",
                              num_scales=4, **mp).eval()
res["model_class"] = type(model).__module__ + "." + type(model).__name__
res["hid_features"] = model.hid_features
if os.environ.get("MSWEGNN_FUSED_ROLLOUT") == "1":
    # building the model applies a patch deferred by a half-initialised training.train, so
    # the FIRST rollout_test call below is already the fused one
    from mswegnn.rollout import rollout_test as fused_fn
    res["patched_at_build"] = training.train.rollout_test is fused_fn

from torch_geometric.data import Data, Batch
from mswegnn.mesh import make_multiscale_mesh, wet_state
import msgnn_torch as orc
P = {k: v.detach().clone() for k, v in model.state_dict().items()}
ocfg = orc.msgnn_config(num_scales=4, hid_features=64, K=4)
g1 = wet_state(make_multiscale_mesh(n_coarse=2, num_scales=4, seed=3, T=3), seed=4)
g2 = make_multiscale_mesh(n_coarse=3, num_scales=4, seed=5, T=3)
d1, d2 = Data(**g1.__dict__), Data(**g2.__dict__)
o1, o2 = orc.rollout(P, ocfg, g1, 3), orc.rollout(P, ocfg, g2, 3)

def rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))

r = training.train.rollout_test(model, d1)
res["single_rel"] = rel(r, o1)
batch = Batch.from_data_list([d1, d2])
r = training.train.rollout_test(model, batch)
n1 = g1.x.shape[0]
res["batch_rel"] = max(rel(r[:n1], o1), rel(r[n1:], o2))

if os.environ.get("MSWEGNN_FUSED_ROLLOUT") == "1":
    from mswegnn.rollout import rollout_test as fused
    model(d1)  # the forward-time fallback of the deferred patch is harmless once applied
    res["patched"] = training.train.rollout_test is fused
    res["kept_reference"] = callable(getattr(training.train, "_reference_rollout_test", None))
    tr = cfg["trainer_options"]
    plm = training.train.LightningTrainer(model, cfg["lr_info"], tr, {})
    parts = plm.predict_step(batch, 0)
    res["predict_step_rel"] = max(rel(parts[0], o1), rel(parts[1], o2))
    res["predict_step_shapes"] = [list(p.shape) for p in parts]
print("RESULT " + json.dumps(res))
'''


def _run(order, fused):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MSWEGNN_FUSED_ROLLOUT="1" if fused else "0",
               OMP_NUM_THREADS="4")
    env.pop("PYTHONPATH", None)
    p = subprocess.run([sys.executable, "-c", DRIVER, REF, STUBS, ROOT, PKG, order], cwd=REF, env=env,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


@pytest.mark.parametrize("order,fused", [("callers", False), ("callers", True), ("train_first", True)])
def test_reference_callers_run_with_dropin(order, fused):
    r = _run(order, fused)
    assert r["test_model.py"] == "ok" and r["main.py"] == "ok"
    assert r["models"].startswith(PKG), r["models"]
    assert r["training"].startswith(REF) and r["utils"].startswith(REF)
    assert r["caller_symbols"]
    assert r["model_class"] == "models.gnn.MSGNN" and r["hid_features"] == 64
    assert r["single_rel"] <= 1e-5 and r["batch_rel"] <= 1e-5, r
    if fused:
        assert r["patched"] and r["kept_reference"] and r["patched_at_build"], r
        assert r["predict_step_rel"] <= 1e-5, r
