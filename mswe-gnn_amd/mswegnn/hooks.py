"""Opt-in: route the reference's own ``training.train.rollout_test`` to the fused engine.

The drop-in replaces only the reference's ``models`` package.  With it,
the reference's ``rollout_test`` (training/train.py:67-95) steps the model in Python and
every step is one HIP ``msw_forward``.  ``install_fused_rollout()`` swaps that function for
:func:`mswegnn.rollout.rollout_test` (same semantics, the whole T-step loop as ONE
``msw_rollout``) inside the reference's module, so ``LightningTrainer.validation_step`` /
``predict_step`` (train.py:157-185), which look the name up in their module's globals at
call time, reach the fused path with no change to the callers.  ``models/__init__.py``
calls it when ``MSWEGNN_FUSED_ROLLOUT=1``.  The reference's function stays available as
``training.train._reference_rollout_test``.
"""
import importlib.abc
import sys

TARGET = "training.train"


def _patch(mod):
    from .rollout import rollout_test
    if getattr(mod, "rollout_test", None) is rollout_test:
        return
    mod._reference_rollout_test = getattr(mod, "rollout_test", None)
    mod.rollout_test = rollout_test


class _PatchingLoader(importlib.abc.Loader):
    def __init__(self, loader):
        self.loader = loader

    def create_module(self, spec):
        return self.loader.create_module(spec)

    def exec_module(self, module):
        self.loader.exec_module(module)
        _patch(module)


class _Finder(importlib.abc.MetaPathFinder):
    def find_spec(self, name, path, target=None):
        if name != TARGET:
            return None
        for f in sys.meta_path:
            if f is self or not hasattr(f, "find_spec"):
                continue
            spec = f.find_spec(name, path, target)
            if spec is not None:
                if spec.loader is not None:
                    spec.loader = _PatchingLoader(spec.loader)
                return spec
        return None


PENDING = False  # training.train was mid-import when the hook was installed


def _initializing(mod):
    return bool(getattr(getattr(mod, "__spec__", None), "_initializing", False))


def install_fused_rollout():
    """Patch ``training.train.rollout_test`` now if it is imported, else when it is.

    If ``training.train`` is itself being imported (it imports ``models`` through
    utils.miscellaneous before defining ``rollout_test``), the patch is applied by
    :func:`maybe_patch` at the first model call instead."""
    global PENDING
    mod = sys.modules.get(TARGET)
    if mod is not None:
        if _initializing(mod):
            PENDING = True
        else:
            _patch(mod)
    if not any(isinstance(f, _Finder) for f in sys.meta_path):
        sys.meta_path.insert(0, _Finder())


def maybe_patch():
    global PENDING
    mod = sys.modules.get(TARGET)
    if mod is not None and not _initializing(mod):
        _patch(mod)
        PENDING = False
