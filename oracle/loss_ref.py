"""ORACLE (test infrastructure only): CPU/GPU-agnostic torch restatement of the reference's
training loss and training step, the caller of the training path.  Pinned
against tests/golden/fx_grad_train_*.npz, which oracle/gen_golden_grad.py produced with the
reference's own LightningTrainer.training_step and loss_function.

  get_mean_error        training/loss.py:8-23
  mask_on_water         training/loss.py:25-35
  loss variable scaler  training/loss.py:37-47
  get_multiscale_loss   training/loss.py:49-74 (Batch branch: node_ptr 2-D after
                        update_batch_multiscale, training/train.py:31-65)
  loss_function         training/loss.py:76-118 (conservation = 0, the config.yaml value;
                        the conservation term is not restated)
  training_step         training/train.py:125-145
"""
import torch

NUM_WATER_VARS = 2


def get_mean_error(diff, type_loss, nodes_dim=0):
    """training/loss.py:8-23"""
    if type_loss == "RMSE":
        return torch.sqrt((diff ** 2).mean(nodes_dim))
    if type_loss == "MAE":
        return diff.abs().mean(nodes_dim)
    raise ValueError(type_loss)


def mask_on_water(diff, water_axis=1):
    """training/loss.py:25-35"""
    return (diff != 0).any(water_axis)


def loss_variable_scaler(velocity_scaler=1, device="cpu", dtype=torch.float32):
    """training/loss.py:37-47"""
    s = torch.ones(NUM_WATER_VARS, dtype=dtype, device=device)
    s[1::NUM_WATER_VARS] = velocity_scaler
    return s


def multiscale_loss(diff, node_ptr, only_where_water=True, type_loss="RMSE", num_graphs=None):
    """training/loss.py:49-74: the finest scale of every graph (node_ptr [G, S+1] for a batch,
    [S+1] for one graph), optionally only rows with a non-zero difference."""
    where = mask_on_water(diff) if only_where_water else torch.ones(diff.shape[0], dtype=torch.bool,
                                                                      device=diff.device)
    if node_ptr.dim() == 2:
        parts = [diff[int(node_ptr[i, 0]):int(node_ptr[i, 1])][where[int(node_ptr[i, 0]):int(node_ptr[i, 1])]]
                 for i in range(num_graphs if num_graphs is not None else node_ptr.shape[0])]
        return get_mean_error(torch.cat(parts), type_loss, 0)
    a, b = int(node_ptr[0]), int(node_ptr[1])
    return get_mean_error(diff[a:b][where[a:b]], type_loss, 0)


def loss_function(preds, real, data, type_loss="RMSE", only_where_water=False, conservation=0,
                  velocity_scaler=1):
    """training/loss.py:76-118 (conservation = 0)."""
    if conservation != 0:
        raise NotImplementedError("the mass-conservation term (config.yaml: conservation 0) is not restated")
    diff = preds - real
    if "node_ptr" in data.keys():
        loss = multiscale_loss(diff, data.node_ptr, only_where_water, type_loss)
    else:
        if only_where_water:
            diff = diff[mask_on_water(diff)]
        loss = get_mean_error(diff, type_loss, 0)
    sc = loss_variable_scaler(velocity_scaler, diff.device, loss.dtype)
    return torch.dot(loss, sc) / sc.sum()


def apply_boundary_condition(x_d, BC, node_BC, type_BC=2):
    """utils/dataset.py:486-497"""
    x_d[node_BC, (int(type_BC) - 1)::NUM_WATER_VARS] = BC
    return x_d


def use_prediction(x, pred, previous_t):
    """utils/dataset.py:508-529"""
    dyn = previous_t * NUM_WATER_VARS
    st = x.shape[1] - dyn
    if previous_t == 1:
        return torch.cat((x[:, :st], pred), 1)
    return torch.cat((x[:, :st], x[:, -dyn + NUM_WATER_VARS:], pred), 1)


def training_step(model, temp, rollout_steps, type_loss="RMSE", only_where_water=True, conservation=0,
                  velocity_scaler=7):
    """training/train.py:125-145 on an already adapted batch `temp` (adapt_batch_training,
    train.py:14-29; the caller passes a fresh one, it is modified in place): R curriculum
    rollout steps -- BC write, forward, prediction fed back, per-step loss -- and their mean.
    Defaults: config.yaml trainer_options."""
    dyn = model.previous_t * model.NUM_WATER_VARS
    roll = []
    for i in range(rollout_steps):
        temp.x[:, -dyn:] = apply_boundary_condition(temp.x[:, -dyn:], temp.BC[:, :, i], temp.node_BC,
                                                    type_BC=temp.type_BC)
        preds = model(temp)
        temp.x = use_prediction(temp.x, preds, model.previous_t)
        roll.append(loss_function(preds, temp.y[:, :, i], temp, type_loss=type_loss,
                                  only_where_water=only_where_water, conservation=conservation,
                                  velocity_scaler=velocity_scaler))
    return torch.stack(roll).mean()
