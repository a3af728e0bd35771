"""MI355X-native engine of the mSWE-GNN multi-scale rollout (host side).

The drop-in surface is the sibling package ``models`` (models.gnn, models.models), which
replaces the reference's ``models`` namespace package; the reference's own ``training`` and
``utils`` stay in charge of everything else.  This package holds the C-ABI
binding (``_lib``), plans (``engine``), the rollout-path operators and the fused
``rollout_test`` (``rollout``), batching (``batch``), partitioning (``partition``),
on-device metrics (``metrics``) and the synthetic meshes (``mesh``).
"""
import os
import sys

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG_ROOT not in sys.path:
    sys.path.insert(0, _PKG_ROOT)

__version__ = "0.2.0"
