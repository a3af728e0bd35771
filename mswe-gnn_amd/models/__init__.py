"""Drop-in ``models`` package (reference: models/gnn.py, models/models.py).

The reference's ``models/`` directory has no ``__init__.py`` (a namespace package); this is
a regular package, so with ``mswe-gnn_amd/`` anywhere on ``sys.path`` (e.g. PYTHONPATH)
Python resolves ``models`` here even though the running script's own directory comes first
on the path.  The reference's ``training`` and ``utils`` are not shadowed.
"""
import os

if os.environ.get("MSWEGNN_FUSED_ROLLOUT", "") not in ("", "0"):
    from mswegnn.hooks import install_fused_rollout
    install_fused_rollout()
