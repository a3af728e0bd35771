import torch
from . import pytorch  # noqa: F401


class LightningModule(torch.nn.Module):
    def log(self, *a, **k):
        pass


class LightningDataModule:
    pass


def seed_everything(seed):
    torch.manual_seed(seed)
