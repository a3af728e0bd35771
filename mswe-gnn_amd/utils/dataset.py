"""Drop-in subset of the reference's ``utils.dataset`` used on the rollout path.

  apply_boundary_condition  utils/dataset.py:486-497
  check_type_BC             utils/dataset.py:499-506
  use_prediction            utils/dataset.py:508-529
  create_scale_mask         utils/dataset.py:615-638

Dataset construction (create_model_dataset, to_temporal_dataset, scalers) is offline
preprocessing outside the MI355X hot path.
"""
import torch

NUM_WATER_VARS = 2


def _is_batch(data):
    return hasattr(data, "num_graphs") and hasattr(data, "ptr")


def check_type_BC(type_BC, num_water_vars):
    if type_BC == 1 or type_BC == 2:
        assert type_BC <= num_water_vars, \
            "The boundary conditions are not compatible with the data format you are using."
    elif type_BC == 3:
        raise ValueError("Vector boundary conditions are not implemented.")
    else:
        raise ValueError(f"BC_type={type_BC} is not a valid input. Please select either:\n"
                         "1: Inflow water depth\n2: Inflow discharge")


def apply_boundary_condition(x_d, BC, node_BC, type_BC=2):
    """Write the inflow BC into the dynamic columns of the BC nodes:
    x_d[node_BC, (type_BC-1)::2] = BC (type 1: depth h, type 2: discharge |q|)."""
    type_BC = int(type_BC)
    check_type_BC(type_BC, NUM_WATER_VARS)
    x_d[node_BC.long(), (type_BC - 1)::NUM_WATER_VARS] = BC
    return x_d


def use_prediction(x, pred, previous_t):
    """Slide the dynamic window by one step and append the prediction."""
    assert pred.shape[-1] == NUM_WATER_VARS, \
        "The number of predictions is not consistent with the number of future time steps"
    dyn = previous_t * NUM_WATER_VARS
    n_static = x.shape[1] - dyn
    keep = x[:, n_static + NUM_WATER_VARS:] if previous_t > 1 else x[:, :0]
    out = torch.cat((x[:, :n_static], keep, pred), 1)
    assert out.shape == x.shape, f'The shape of the input has changed from {x.shape} to {out.shape}'
    return out


def create_scale_mask(num_nodes, num_scales, node_ptr, data_type=None, device='cpu'):
    """Scale id per node from node_ptr ([S+1], or [G, S+1] for a batch)."""
    mask = torch.zeros(num_nodes, dtype=torch.int, device=device)
    ptr = node_ptr.reshape(-1, node_ptr.shape[-1]) if node_ptr.dim() == 2 else node_ptr.reshape(1, -1)
    for i in range(num_scales):
        for j in ptr[:, i:i + 2]:
            mask[int(j[0]):int(j[1])] = i
    return mask
