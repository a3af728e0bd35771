import copy


class Data:
    """Attribute bag standing in for torch_geometric.data.Data."""

    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    def keys(self):
        return list(self.__dict__.keys())

    def clone(self):
        out = self.__class__.__new__(self.__class__)
        for k, v in self.__dict__.items():
            out.__dict__[k] = v.clone() if hasattr(v, 'clone') else copy.copy(v)
        return out


class Batch(Data):
    pass
