"""MI355X-native engine of the mSWE-GNN multi-scale rollout (host side).

The drop-in surface lives in the sibling packages ``models`` (models.gnn, models.models),
``training`` (training.train.rollout_test) and ``utils`` (utils.dataset step operators,
utils.miscellaneous.get_model), mirroring the reference's module names.
"""
import os
import sys

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG_ROOT not in sys.path:
    sys.path.insert(0, _PKG_ROOT)

__version__ = "0.1.0"
