"""Disjoint-union batching of simulations with PyG ``Batch`` collation semantics.

The reference batches simulations with torch_geometric's DataLoader (test_model.py:37,
batch_size=20): attributes whose name contains ``index`` are offset by the number of nodes
of the preceding graphs and concatenated along the last dim, everything else is
concatenated along dim 0 (0-d tensors are stacked), ``ptr`` holds node offsets.
``training.train.adapt_batch_training`` / ``update_batch_multiscale`` (train.py:14-65) then
regroup the edges scale-major.  This module reproduces that collation without PyG.
"""
import torch

from .mesh import Graph

__all__ = ["Batch", "collate"]


class Batch(Graph):
    """A collated batch; ``batch[i]`` returns the i-th graph's un-offset attributes."""

    def __getitem__(self, i):
        return self._graphs[i]

    def clone(self):
        out = Batch()
        for k, v in self.__dict__.items():
            out.__dict__[k] = v.clone() if isinstance(v, torch.Tensor) else v
        return out

    def to(self, device):
        out = Batch()
        for k, v in self.__dict__.items():
            if k == "_graphs":
                out.__dict__[k] = [g.to(device) for g in v]
            else:
                out.__dict__[k] = v.to(device) if isinstance(v, torch.Tensor) else v
        return out

    def keys(self):
        return [k for k in self.__dict__ if k != "_graphs"]


def collate(graphs):
    b = Batch()
    counts = [int(g.x.shape[0]) for g in graphs]
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    for k in graphs[0].keys():
        vals = [getattr(g, k) for g in graphs]
        if not isinstance(vals[0], torch.Tensor):
            setattr(b, k, vals)
        elif "index" in k:
            setattr(b, k, torch.cat([v + o for v, o in zip(vals, offs)], -1))
        elif vals[0].dim() == 0:
            setattr(b, k, torch.stack(vals))
        else:
            setattr(b, k, torch.cat(vals, 0))
    b.ptr = torch.tensor(offs, dtype=torch.long)
    b.num_graphs = len(graphs)
    b._graphs = list(graphs)
    return b
