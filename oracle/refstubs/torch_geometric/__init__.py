"""Stub of torch_geometric for running the read-only reference on CPU (test infrastructure only).

Only `torch_geometric.utils.scatter` computes anything; it restates PyG 2.4.0's
published semantics (requirements.txt:25 of the reference pins torch_geometric==2.4.0;
the package is absent from this image, so this restatement is "parity unpinned" at
this boundary -- see DESIGN.md).
"""
from . import utils, nn, data, loader  # noqa: F401
