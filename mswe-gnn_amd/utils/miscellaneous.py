"""Drop-in subset of the reference's ``utils.miscellaneous`` (get_model registry,
utils/miscellaneous.py:15-18).  Evaluation metrics / plotting are outside the hot path."""
from models.gnn import GNN, MSGNN

NUM_WATER_VARS = 2


def get_model(model_name):
    return {'GNN': GNN, 'MSGNN': MSGNN}[model_name]
