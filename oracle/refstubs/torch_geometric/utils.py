"""Restatement of torch_geometric.utils.scatter (PyG 2.4.0, CPU path without torch_scatter).

sum/add : zeros(dim_size, ...).scatter_add_(dim, index, src)
mean    : the same sum divided by count.clamp(min=1), count = scatter_add_ of ones.
Call sites in the reference: models/gnn.py:254,256,437.
"""
import torch


def _broadcast(index, src, dim):
    if dim < 0:
        dim = src.dim() + dim
    if index.dim() == 1:
        for _ in range(0, dim):
            index = index.unsqueeze(0)
    for _ in range(index.dim(), src.dim()):
        index = index.unsqueeze(-1)
    return index.expand_as(src)


def scatter(src, index, dim=0, dim_size=None, reduce='sum'):
    if dim < 0:
        dim = src.dim() + dim
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() > 0 else 0
    size = list(src.size())
    size[dim] = dim_size
    if reduce in ('sum', 'add'):
        idx = _broadcast(index, src, dim)
        return src.new_zeros(size).scatter_add_(dim, idx, src)
    if reduce == 'mean':
        count = src.new_zeros(dim_size)
        count.scatter_add_(0, index, src.new_ones(src.size(dim)))
        count = count.clamp(min=1)
        idx = _broadcast(index, src, dim)
        out = src.new_zeros(size).scatter_add_(dim, idx, src)
        return out / _broadcast(count, out, dim)
    raise NotImplementedError(reduce)


def to_undirected(*args, **kwargs):
    raise NotImplementedError("stub")
