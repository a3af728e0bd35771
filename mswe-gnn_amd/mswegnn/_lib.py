"""ctypes binding of the C ABI in include/mswegnn.h (libmswegnn.so, gfx950).

The shared library is built in-tree (mswe-gnn_amd/lib/libmswegnn.so) by
``python mswe-gnn_amd/build_engine.py`` / ``__graft_entry__.build()``.  There is no fallback:
if the library is missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MSW_LIB_VARIANT=trace selects the diagnostic build (tools/trace_kernels.py)
_VARIANT = os.environ.get("MSW_LIB_VARIANT", "")
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib",
                        f"libmswegnn_{_VARIANT}.so" if _VARIANT else "libmswegnn.so")

MSW_OK = 0
MAX_MLP_LAYERS = 4

ACT = {None: 0, "prelu": 1, "relu": 2, "leakyrelu": 3, "elu": 4, "swish": 5, "sigmoid": 6,
       "tanh": 7}

c_float_p = C.POINTER(C.c_float)
c_int64_p = C.POINTER(C.c_int64)
c_int32_p = C.POINTER(C.c_int32)


class MswLinear(C.Structure):
    _fields_ = [("in_features", C.c_int32), ("out_features", C.c_int32),
                ("weight", c_float_p), ("bias", c_float_p),
                ("act", C.c_int32), ("act_param", C.c_float)]


class MswMlp(C.Structure):
    _fields_ = [("n_layers", C.c_int32), ("layer", MswLinear * MAX_MLP_LAYERS)]


class MswSwegnn(C.Structure):
    _fields_ = [("K", C.c_int32), ("normalize", C.c_int32), ("with_filter_matrix", C.c_int32),
                ("with_gradient", C.c_int32), ("upwind_mode", C.c_int32),
                ("edge_features", C.c_int32), ("edge_mlp", MswMlp),
                ("filter", C.POINTER(c_float_p))]


class MswModelDesc(C.Structure):
    _fields_ = [("model_type", C.c_int32), ("hid_features", C.c_int32),
                ("num_scales", C.c_int32), ("previous_t", C.c_int32),
                ("num_node_features", C.c_int32), ("with_WL", C.c_int32),
                ("skip_connections", C.c_int32), ("learned_pooling", C.c_int32),
                ("gnn_act", C.c_int32), ("gnn_act_param", C.c_float),
                ("residual_weights", c_float_p), ("edge_mlp", C.c_int32),
                ("edge_encoder", MswMlp), ("static_encoder", MswMlp),
                ("dynamic_encoder", MswMlp), ("decoder", MswMlp),
                ("num_processors", C.c_int32), ("processors", C.POINTER(MswSwegnn)),
                ("num_unpool", C.c_int32), ("unpool", C.POINTER(MswSwegnn))]


class MswGraphDesc(C.Structure):
    _fields_ = [("num_nodes", C.c_int64), ("num_scales", C.c_int32), ("num_graphs", C.c_int32),
                ("node_ptr", c_int64_p), ("num_edges", C.c_int64), ("edge_index", c_int64_p),
                ("edge_attr", c_float_p), ("num_edge_features", C.c_int32),
                ("edge_ptr", c_int64_p), ("num_intra_edges", C.c_int64),
                ("intra_edge_index", c_int64_p), ("intra_edge_ptr", c_int64_p)]


class MswPlanStats(C.Structure):
    _fields_ = [("num_nodes", C.c_int64), ("num_edges", C.c_int64), ("num_scales", C.c_int32),
                ("hid_features", C.c_int32), ("padded_features", C.c_int32),
                ("kernels_per_step", C.c_int32), ("forward_calls", C.c_int64),
                ("rollout_steps", C.c_int64), ("device_bytes", C.c_int64),
                ("graph_captured", C.c_int32), ("rccl_calls", C.c_int64), ("rccl_steps", C.c_int64)]


class MswExchangeDesc(C.Structure):
    _fields_ = [("num_entries", C.c_int32), ("peer", c_int32_p), ("scale", c_int32_p),
                ("recv_ptr", c_int64_p), ("recv_rows", c_int32_p),
                ("send_ptr", c_int64_p), ("send_rows", c_int32_p)]


MAX_HOPS = 8


class MswSwegnnTrainDesc(C.Structure):
    _fields_ = [("num_nodes", C.c_int64), ("num_edges", C.c_int64), ("F", C.c_int32),
                ("edge_features", C.c_int32), ("K", C.c_int32), ("n_layers", C.c_int32),
                ("width", C.c_int32 * (MAX_MLP_LAYERS + 1)), ("act", C.c_int32 * MAX_MLP_LAYERS),
                ("normalize", C.c_int32), ("with_filter_matrix", C.c_int32),
                ("with_gradient", C.c_int32), ("upwind_mode", C.c_int32),
                ("row", C.c_void_p), ("col", C.c_void_p), ("in_ptr", C.c_void_p), ("in_edge", C.c_void_p),
                ("out_ptr", C.c_void_p), ("out_edge", C.c_void_p),
                ("weight", C.c_void_p * MAX_MLP_LAYERS), ("bias", C.c_void_p * MAX_MLP_LAYERS),
                ("slope", C.c_void_p * MAX_MLP_LAYERS), ("filter", C.c_void_p * (MAX_HOPS + 1))]


class MswSwegnnGrads(C.Structure):
    _fields_ = [("d_x_s", C.c_void_p), ("d_x_d", C.c_void_p), ("d_edge_attr", C.c_void_p),
                ("d_weight", C.c_void_p * MAX_MLP_LAYERS), ("d_bias", C.c_void_p * MAX_MLP_LAYERS),
                ("d_slope", C.c_void_p * MAX_MLP_LAYERS), ("d_filter", C.c_void_p * (MAX_HOPS + 1))]



class MswMlpTrainDesc(C.Structure):
    _fields_ = [("rows", C.c_int64), ("n_layers", C.c_int32), ("width", C.c_int32 * (MAX_MLP_LAYERS + 1)),
                ("act", C.c_int32 * MAX_MLP_LAYERS), ("weight", C.c_void_p * MAX_MLP_LAYERS),
                ("bias", C.c_void_p * MAX_MLP_LAYERS), ("slope", C.c_void_p * MAX_MLP_LAYERS)]


class MswMlpGrads(C.Structure):
    _fields_ = [("d_x", C.c_void_p), ("d_weight", C.c_void_p * MAX_MLP_LAYERS),
                ("d_bias", C.c_void_p * MAX_MLP_LAYERS), ("d_slope", C.c_void_p * MAX_MLP_LAYERS)]


# (name, restype, argtypes) of every entry point declared in include/mswegnn.h
SYMBOLS = [
    ("msw_plan_create", C.c_int, [C.POINTER(MswGraphDesc), C.POINTER(MswModelDesc), C.c_int,
                                  C.POINTER(C.c_void_p)]),
    ("msw_plan_destroy", C.c_int, [C.c_void_p]),
    ("msw_forward", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("msw_rollout", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, c_int32_p, C.c_int32,
                              C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    ("msw_debug_buffer", C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_void_p]),
    ("msw_set_graph_capture", C.c_int, [C.c_void_p, C.c_int]),
    ("msw_set_group_graph", C.c_int, [C.c_void_p, C.c_int]),
    ("msw_plan_get_stats", C.c_int, [C.c_void_p, C.POINTER(MswPlanStats)]),
    ("msw_last_error", C.c_char_p, []),
    ("msw_abi_version", C.c_int, []),
    ("msw_struct_size", C.c_int64, [C.c_char_p]),
    ("msw_bench_kernel", C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, c_int64_p,
                                   C.c_void_p]),
    ("msw_set_trace", C.c_int, [C.c_void_p, C.c_void_p]),
    ("msw_rollout_metrics", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, c_int64_p, C.c_int32,
                                      c_float_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p]),
    ("msw_plan_create_part", C.c_int, [C.POINTER(MswGraphDesc), C.POINTER(MswModelDesc), C.c_int,
                                       C.POINTER(MswExchangeDesc), C.c_int32, C.POINTER(C.c_void_p)]),
    ("msw_comm_unique_id", C.c_int, [C.c_char_p]),
    ("msw_plan_set_comm", C.c_int, [C.c_void_p, C.c_char_p, C.c_int32, C.c_int32]),
    ("msw_group_rollout", C.c_int, [C.POINTER(C.c_void_p), C.c_int32, C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_void_p), c_int32_p, C.POINTER(c_int32_p), c_int32_p,
                                    C.c_int32, C.c_int32, C.POINTER(C.c_void_p), C.c_void_p]),
    ("msw_swegnn_train_workspace", C.c_int, [C.POINTER(MswSwegnnTrainDesc), c_int64_p, c_int64_p]),
    ("msw_swegnn_train_forward", C.c_int, [C.POINTER(MswSwegnnTrainDesc), C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("msw_swegnn_train_backward", C.c_int, [C.POINTER(MswSwegnnTrainDesc), C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.POINTER(MswSwegnnGrads), C.c_void_p, C.c_void_p]),
    ("msw_pool_mean_forward", C.c_int, [C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_void_p]),
    ("msw_pool_mean_backward", C.c_int, [C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p]),
    ("msw_mlp_train_workspace", C.c_int, [C.POINTER(MswMlpTrainDesc), c_int64_p, c_int64_p]),
    ("msw_mlp_train_forward", C.c_int, [C.POINTER(MswMlpTrainDesc), C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p]),
    ("msw_mlp_train_backward", C.c_int, [C.POINTER(MswMlpTrainDesc), C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.POINTER(MswMlpGrads), C.c_void_p, C.c_void_p]),
]

STRUCTS = {"msw_linear": MswLinear, "msw_mlp": MswMlp, "msw_swegnn": MswSwegnn,
           "msw_model_desc": MswModelDesc, "msw_graph_desc": MswGraphDesc,
           "msw_plan_stats": MswPlanStats, "msw_exchange_desc": MswExchangeDesc,
           "msw_swegnn_train_desc": MswSwegnnTrainDesc, "msw_swegnn_grads": MswSwegnnGrads,
           "msw_mlp_train_desc": MswMlpTrainDesc, "msw_mlp_grads": MswMlpGrads}

_lib = None


def lib():
    """Load libmswegnn.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"mSWE-GNN HIP engine not built: {LIB_PATH} is missing "
                "(run `python mswe-gnn_amd/build_engine.py` or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SYMBOLS:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.msw_abi_version() != 1:
            raise RuntimeError("libmswegnn.so ABI version mismatch")
        _lib = L
    return _lib


def lib_info():
    """Path, size, mtime and sha256 of the library this process loads (bench provenance)."""
    import hashlib
    with open(LIB_PATH, "rb") as f:
        data = f.read()
    st = os.stat(LIB_PATH)
    return {"path": os.path.relpath(LIB_PATH, os.path.dirname(os.path.dirname(_HERE))),
            "bytes": st.st_size, "mtime": st.st_mtime, "sha256": hashlib.sha256(data).hexdigest()}


MSW_ERR_UNSUPPORTED = -3


class EngineError(RuntimeError):
    """A negative MSW_ERR_* return code; ``code`` holds it."""

    def __init__(self, code, msg):
        super().__init__(f"mswegnn error {code}: {msg}")
        self.code = code


def check(rc):
    if rc != MSW_OK:
        msg = lib().msw_last_error().decode(errors="replace")
        raise EngineError(rc, msg)
    return rc
