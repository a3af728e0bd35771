"""Drop-in for the reference's ``models.models`` (sdat2/mSWE-GNN models/models.py).

Same public names, constructor signatures, Sequential layouts and parameter names, so the
reference's Lightning checkpoints (``state_dict`` keys ``model.*``) load unchanged and a
seeded construction draws the same random numbers in the same order.

  BaseFloodModel              models/models.py:7-91
  init_true_residuals_weights models/models.py:93-100
  add_norm_dropout_activation models/models.py:102-112
  make_mlp                    models/models.py:121-146
  activation_functions        models/models.py:149-169
"""
import torch
import torch.nn as nn

NUM_WATER_VARS = 2  # water depth h and unit discharge |q|

_ACTIVATIONS = {
    "relu": lambda device: nn.ReLU(),
    "prelu": lambda device: nn.PReLU(device=device),
    "leakyrelu": lambda device: nn.LeakyReLU(0.1),
    "elu": lambda device: nn.ELU(),
    "swish": lambda device: nn.SiLU(),
    "sigmoid": lambda device: nn.Sigmoid(),
    "tanh": lambda device: nn.Tanh(),
}


def activation_functions(activation_name, device="cpu"):
    """Activation module by name (None -> None); models/models.py:149-169."""
    if activation_name is None:
        return None
    try:
        return _ACTIVATIONS[activation_name](device)
    except KeyError:
        raise AttributeError('Please choose one of the following options:\n'
                             '"relu", "prelu", "leakyrelu", "elu", "gelu", "sigmoid", "tanh"')


def add_norm_dropout_activation(hidden_size, layer_norm=False, dropout=0, activation="relu",
                                device="cpu"):
    """[LayerNorm] -> [Dropout] -> [activation] block appended after every Linear."""
    layers = []
    if layer_norm:
        layers.append(nn.LayerNorm(hidden_size, eps=1e-5, device=device))
    if dropout:
        layers.append(nn.Dropout(dropout))
    if activation is not None:
        layers.append(activation_functions(activation, device=device))
    return layers


def init_weights(layer):
    if isinstance(layer, nn.Linear):
        nn.init.xavier_normal_(layer.weight)
        if layer.bias is not None:
            nn.init.normal_(layer.bias)


def make_mlp(input_size, output_size, hidden_size=32, n_layers=2, bias=False,
             activation="relu", dropout=0, layer_norm=False, device="cpu"):
    """Linear stack with the activation block after EVERY layer (also the last)."""
    dims = [input_size] + [hidden_size] * (n_layers - 1) + [output_size]
    layers = []
    for i in range(n_layers):
        layers.append(nn.Linear(dims[i], dims[i + 1], bias=bias, device=device))
        layers += add_norm_dropout_activation(dims[i + 1], layer_norm=layer_norm, dropout=dropout,
                                              activation=activation, device=device)
    return nn.Sequential(*layers)


def init_true_residuals_weights(previous_t: int, base=2, repeat=1, device="cpu"):
    """Exponentially growing, normalised weights: later steps weigh more."""
    w = torch.tensor([float(base ** e) for e in range(previous_t)], device=device)
    w = w / w.sum()
    return nn.Parameter(w.repeat(repeat).reshape(repeat, -1).T.contiguous())


class BaseFloodModel(nn.Module):
    """Residual connection from the input water variables and small-depth masking."""

    def __init__(self, previous_t=1, learned_residuals=None, seed=42, residuals_base=2,
                 residual_init="exp", with_WL=False, device="cpu"):
        super().__init__()
        torch.manual_seed(seed)
        self.previous_t = previous_t
        self.with_WL = with_WL
        self.learned_residuals = learned_residuals
        self.device = device
        self.residuals_base = residuals_base
        self.residual_init = residual_init
        assert residual_init in ("exp", "random"), \
            "Argument 'residual_init' can only be either 'exp' or 'random'"
        self.NUM_WATER_VARS = NUM_WATER_VARS
        self.out_dim = self.NUM_WATER_VARS
        if learned_residuals is True or learned_residuals == "all":
            repeat = 1 if learned_residuals is True else self.out_dim
            if residual_init == "exp":
                self.residual_weights = init_true_residuals_weights(previous_t, residuals_base,
                                                                    repeat=repeat, device=device)
            else:
                self.residual_weights = nn.Parameter(torch.Tensor(previous_t, repeat).to(device))
                nn.init.xavier_normal_(self.residual_weights)

    # ---------------------------------------------------------------- residual / mask
    def _residual_matrix(self):
        """[p, 2] matrix M with residual_var = sum_tau M[tau, var] * x[:, dyn(tau, var)],
        or None when there is no residual connection."""
        p, nv = self.previous_t, self.NUM_WATER_VARS
        lr = self.learned_residuals
        if lr is True:
            return self.residual_weights[:, :1].expand(p, nv)
        if lr == "all":
            return self.residual_weights
        if lr is False:
            M = torch.zeros(p, nv, device=self.residual_device())
            M[-1] = 1.0
            return M
        return None

    def residual_device(self):
        for prm in self.parameters():
            return prm.device
        return torch.device("cpu")

    def _add_residual_connection(self, x):
        """models/models.py:50-77."""
        nv, p = self.NUM_WATER_VARS, self.previous_t
        lr = self.learned_residuals
        if lr is True or lr == "all":
            x0 = x[:, -p * nv:].reshape(-1, p, nv)
            cols = [0] * nv if lr is True else list(range(nv))
            return torch.stack([x0[:, :, i] @ self.residual_weights[:, c] for i, c in enumerate(cols)], -1)
        if lr is False:
            return x[:, -self.out_dim:]
        return torch.zeros(x.shape[0], self.out_dim, device=x.device)

    def _mask_small_WD(self, x, epsilon=0.001):
        """Zero depths with |h| <= epsilon, and velocities where h == 0."""
        h = x[:, 0::self.NUM_WATER_VARS]
        v = x[:, 1::self.NUM_WATER_VARS]
        return torch.cat((h * (h.abs() > epsilon), v * (h != 0)), dim=-1)
