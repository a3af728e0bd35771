"""Stand-ins for torch_geometric.data (test infrastructure only; torch_geometric 2.4.0 is
absent from the image).  ``Batch.from_data_list`` restates PyG's published collation
(``Data.__inc__`` / ``__cat_dim__``): attributes whose name contains ``index`` are offset by
the node count of the preceding graphs and concatenated on the last dim, 0-d tensors are
stacked, other tensors concatenated on dim 0, non-tensors collected in lists; ``ptr`` holds
the node offsets and ``batch[i]`` returns the i-th graph un-offset."""
import copy

import torch


class Data:
    """Attribute bag standing in for torch_geometric.data.Data.  As in PyG, the standard
    attributes (x, edge_index, edge_attr, y, pos, ...) read as None when absent, and
    ``data['key']`` is attribute access."""

    _PYG_ATTRS = ("x", "edge_index", "edge_attr", "edge_weight", "y", "pos", "batch", "face", "normal")

    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    def __getattr__(self, key):  # only called for missing attributes
        if key in Data._PYG_ATTRS:
            return None
        raise AttributeError(f"'{type(self).__name__}' object has no attribute '{key}'")

    def __getitem__(self, key):
        return getattr(self, key)

    def keys(self):
        return [k for k in self.__dict__.keys() if not k.startswith('_')]

    def __contains__(self, key):
        return key in self.keys()

    @property
    def num_nodes(self):
        return int(self.x.shape[0])

    def clone(self):
        out = self.__class__.__new__(self.__class__)
        for k, v in self.__dict__.items():
            out.__dict__[k] = v.clone() if hasattr(v, 'clone') else copy.copy(v)
        return out

    def to(self, device):
        out = self.__class__.__new__(self.__class__)
        for k, v in self.__dict__.items():
            out.__dict__[k] = v.to(device) if isinstance(v, torch.Tensor) else v
        return out


class Batch(Data):
    @classmethod
    def from_data_list(cls, data_list):
        b = cls()
        offs = [0]
        for d in data_list:
            offs.append(offs[-1] + d.num_nodes)
        for k in data_list[0].keys():
            vals = [getattr(d, k) for d in data_list]
            if not isinstance(vals[0], torch.Tensor):
                setattr(b, k, list(vals))
            elif 'index' in k or k == 'face':
                setattr(b, k, torch.cat([v + o for v, o in zip(vals, offs)], -1))
            elif vals[0].dim() == 0:
                setattr(b, k, torch.stack(vals))
            else:
                setattr(b, k, torch.cat(vals, 0))
        b.ptr = torch.tensor(offs, dtype=torch.long)
        b.batch = torch.cat([torch.full((d.num_nodes,), i, dtype=torch.long)
                             for i, d in enumerate(data_list)])
        b._data_list = list(data_list)
        return b

    @property
    def num_graphs(self):
        return len(self._data_list)

    def __getitem__(self, i):
        if isinstance(i, str):
            return getattr(self, i)
        return self._data_list[i]

    def clone(self):
        out = super().clone()
        out._data_list = list(self._data_list)
        return out

    def to(self, device):
        out = super().to(device)
        out._data_list = [d.to(device) for d in self._data_list]
        return out


class DataLoader:  # torch_geometric.data.DataLoader (deprecated alias), import-only
    def __init__(self, *a, **k):
        raise NotImplementedError("stub")
