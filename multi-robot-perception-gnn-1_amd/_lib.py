"""ctypes binding of the HIP C-ABI library ``lib/libmrp_gnn.so`` (declared in ``include/mrp_gnn.h``).

The library is built in-tree by ``__graft_entry__.build()`` (or ``python -m mrp_gnn_amd.build``).
There is deliberately no CPU fallback: if the shared object is missing, every compute call
raises.  torch is imported first so that the process already holds torch's HIP runtime
(soname ``libamdhip64.so.7``) and the library binds to that same runtime, making torch's
streams and device pointers valid inside it.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be loaded before the HIP library, see module docstring)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libmrp_gnn.so")

#: Every symbol ``include/mrp_gnn.h`` declares.
EXPORTED_SYMBOLS = (
    "mrp_film_mean_fwd",
    "mrp_film_mean_cat_fwd",
    "mrp_film_mean_bwd",
    "mrp_film_mean_fwd_ex",
    "mrp_film_mean_bwd_ex",
    "mrp_film_mean_bwd_workspace",
    "mrp_compress_fwd",
    "mrp_compress_weight_transpose",
    "mrp_compress_bwd_data",
    "mrp_compress_bwd_weight_workspace",
    "mrp_compress_bwd_weight",
    "mrp_compress_split_pack_bytes",
    "mrp_compress_split_pack",
    "mrp_compress_fwd_split",
    "mrp_compress_bwd_data_split",
    "mrp_compress_bwd_weight_split_workspace",
    "mrp_compress_bwd_weight_split",
    "mrp_edge_hidden_fwd",
    "mrp_edge_logits_fwd",
    "mrp_edge_encoder_pack_bytes",
    "mrp_edge_encoder_pack",
    "mrp_edge_encoder_fwd_split",
    "mrp_edge_encoder_fwd_split_train",
    "mrp_edge_encoder_bwd_workspace",
    "mrp_edge_encoder_bwd",
    "mrp_edge_encoder_bwd_prep",
    "mrp_edge_encoder_bwd_split_workspace",
    "mrp_edge_encoder_bwd_split",
    "mrp_edge_encoder_bwd_fused_workspace",
    "mrp_edge_encoder_bwd_fused",
    "mrp_edge_encoder_bwd_t_workspace",
    "mrp_edge_encoder_bwd_t",
    "mrp_edge_encoder_bwd_pose_workspace",
    "mrp_edge_encoder_bwd_pose",
    "mrp_frame_graph_build",
    "mrp_stream_copy",
    "mrp_stream_join",
    "mrp_tuning_set",
    "mrp_abi_version",
    "mrp_error_string",
)
ABI_VERSION = 21
MAX_NODES = 16

HIP_ERROR_NOT_SUPPORTED = 801  # hipErrorNotSupported: a fused path declines this shape

MODE_FILM_MEAN = 0
MODE_FILM_SUM = 1
MODE_COPY_MEAN = 2
GB_LOGITS = 0x100  # mode flag: gb holds pre-sigmoid logits
GRAPH_CSR = 0
GRAPH_COMPLETE = 1


MAX_REGULAR_K = 8  # largest in-degree the per-edge-slot backward handles


def graph_regular(k: int) -> int:
    """MRP_GRAPH_REGULAR(k): every node has exactly k in-edges."""
    return (k << 8) | 2
MODES = {"film_mean": MODE_FILM_MEAN, "film_sum": MODE_FILM_SUM, "copy_mean": MODE_COPY_MEAN}

class Epilogue(ctypes.Structure):
    """``mrp_agg_epilogue`` (include/mrp_gnn.h): out = agg_scale*a + self_scale*x[v] + x0_scale*x0[v],
    plus an optional copy of x[v] (the first half of a concatenation buffer)."""

    _fields_ = [("agg_scale", ctypes.c_float), ("self_scale", ctypes.c_float), ("x0", ctypes.c_void_p),
                ("x0_node_stride", ctypes.c_int64), ("x0_scale", ctypes.c_float), ("xcopy", ctypes.c_void_p),
                ("xcopy_node_stride", ctypes.c_int64)]


_lock = threading.Lock()
_lib = None

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64


def _declare(lib: ctypes.CDLL) -> None:
    graph = [_P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32]  # indptr..mode
    lib.mrp_film_mean_fwd.argtypes = [_P, _I64, _P] + graph + [_P, _I64, _P]
    lib.mrp_film_mean_fwd.restype = ctypes.c_int
    lib.mrp_film_mean_cat_fwd.argtypes = [_P, _I64, _P] + graph + [_P, _I64, _P]
    lib.mrp_film_mean_cat_fwd.restype = ctypes.c_int
    lib.mrp_film_mean_bwd.argtypes = [_P, _I64, _P, _I64, _P] + graph + [_P, _I64, _P, _I64, _P, _P]
    lib.mrp_film_mean_bwd.restype = ctypes.c_int
    ep = ctypes.POINTER(Epilogue)
    lib.mrp_film_mean_fwd_ex.argtypes = [_P, _I64, _P] + graph + [_P, _I64, ep, _P]
    lib.mrp_film_mean_fwd_ex.restype = ctypes.c_int
    lib.mrp_film_mean_bwd_ex.argtypes = [_P, _I64, _P, _I64, _P] + graph + [_P, _I64, _P, _I64, _P, ep, _P, _I64, _P]
    lib.mrp_film_mean_bwd_ex.restype = ctypes.c_int
    lib.mrp_film_mean_bwd_workspace.argtypes = [_I32, _I32, _I32, _I32, _I32]
    lib.mrp_film_mean_bwd_workspace.restype = ctypes.c_int64
    lib.mrp_tuning_set.argtypes = [ctypes.c_char_p, _I32]
    lib.mrp_tuning_set.restype = ctypes.c_int
    lib.mrp_compress_fwd.argtypes = [_P, _I64, _P, _I64, _I32, _I32, _I32, _P, _P, _P, _I64, _P]
    lib.mrp_compress_fwd.restype = ctypes.c_int
    lib.mrp_compress_weight_transpose.argtypes = [_P, _P, _I32, _P]
    lib.mrp_compress_weight_transpose.restype = ctypes.c_int
    lib.mrp_compress_bwd_data.argtypes = [_P, _I64, _I32, _I32, _I32, _P, _P, _I64, _P, _I64, _P]
    lib.mrp_compress_bwd_data.restype = ctypes.c_int
    lib.mrp_compress_bwd_weight_workspace.argtypes = [_I32, _I32, _I32, _I64]
    lib.mrp_compress_bwd_weight_workspace.restype = ctypes.c_int64
    lib.mrp_compress_bwd_weight.argtypes = [_P, _I64, _P, _I64, _P, _I64, _I32, _I32, _I32, _P, _P, _P, _I64, _P]
    lib.mrp_compress_bwd_weight.restype = ctypes.c_int
    lib.mrp_compress_split_pack_bytes.argtypes = [_I32, _I32]
    lib.mrp_compress_split_pack_bytes.restype = ctypes.c_int64
    lib.mrp_compress_split_pack.argtypes = [_P, _I64, _I32, _I32, _I32, _P, _P]
    lib.mrp_compress_split_pack.restype = ctypes.c_int
    lib.mrp_compress_fwd_split.argtypes = [_P, _I64, _P, _I64, _I32, _I32, _I32, _P, _P, _P, _I64, _P]
    lib.mrp_compress_fwd_split.restype = ctypes.c_int
    lib.mrp_compress_bwd_data_split.argtypes = [_P, _I64, _I32, _I32, _I32, _P, _P, _I64, _P, _I64, _P]
    lib.mrp_compress_bwd_data_split.restype = ctypes.c_int
    lib.mrp_compress_bwd_weight_split_workspace.argtypes = [_I32, _I32, _I32]
    lib.mrp_compress_bwd_weight_split_workspace.restype = ctypes.c_int64
    lib.mrp_compress_bwd_weight_split.argtypes = lib.mrp_compress_bwd_weight.argtypes
    lib.mrp_compress_bwd_weight_split.restype = ctypes.c_int
    lib.mrp_edge_hidden_fwd.argtypes = [_P, _P, _P, _I32, _I32, _P, _P]
    lib.mrp_edge_hidden_fwd.restype = ctypes.c_int
    lib.mrp_edge_logits_fwd.argtypes = [_P, _I32, _I32, _P, _P, _P, _P]
    lib.mrp_edge_logits_fwd.restype = ctypes.c_int
    lib.mrp_edge_encoder_pack_bytes.argtypes = [_I32]
    lib.mrp_edge_encoder_pack_bytes.restype = ctypes.c_int64
    lib.mrp_edge_encoder_pack.argtypes = [_P, _P, _P, _I32, _P, _P]
    lib.mrp_edge_encoder_pack.restype = ctypes.c_int
    lib.mrp_edge_encoder_fwd_split.argtypes = [_P, _P, _P, _I32, _I32, _P, _P]
    lib.mrp_edge_encoder_fwd_split.restype = ctypes.c_int
    lib.mrp_edge_encoder_fwd_split_train.argtypes = [_P, _P, _P, _I32, _I32, _P, _P, _I64, _P]
    lib.mrp_edge_encoder_fwd_split_train.restype = ctypes.c_int
    lib.mrp_edge_encoder_bwd_prep.argtypes = [_P, _I32, _I32, _P, _I64, _P]
    lib.mrp_edge_encoder_bwd_prep.restype = ctypes.c_int
    lib.mrp_edge_encoder_bwd_split_workspace.argtypes = [_I32, _I32]
    lib.mrp_edge_encoder_bwd_split_workspace.restype = ctypes.c_int64
    lib.mrp_edge_encoder_bwd_split.argtypes = [_P, _P, _P, _P, _I32, _I32, _P, _P, _P, _P, _I64, _P]
    lib.mrp_edge_encoder_bwd_split.restype = ctypes.c_int
    lib.mrp_edge_encoder_bwd_fused_workspace.argtypes = [_I32, _I32]
    lib.mrp_edge_encoder_bwd_fused_workspace.restype = ctypes.c_int64
    lib.mrp_edge_encoder_bwd_fused.argtypes = [_P, _P, _P, _P, _P, _I32, _I32, _P, _P, _P, _P, _P, _I64, _P]
    lib.mrp_edge_encoder_bwd_fused.restype = ctypes.c_int
    lib.mrp_edge_encoder_bwd_t_workspace.argtypes = [_I32, _I32]
    lib.mrp_edge_encoder_bwd_t_workspace.restype = ctypes.c_int64
    lib.mrp_edge_encoder_bwd_t.argtypes = [_P, _I64, _P, _I64, _P, _I32, _I32, _P, _P, _P, _I64, _P]
    lib.mrp_edge_encoder_bwd_t.restype = ctypes.c_int
    lib.mrp_edge_encoder_bwd_pose_workspace.argtypes = [_I32, _I32]
    lib.mrp_edge_encoder_bwd_pose_workspace.restype = ctypes.c_int64
    lib.mrp_edge_encoder_bwd_pose.argtypes = [_P, _I64, _P, _I64, _P, _I32, _I32, _P, _P, _I64, _P]
    lib.mrp_edge_encoder_bwd_pose.restype = ctypes.c_int
    lib.mrp_edge_encoder_bwd_workspace.argtypes = [_I32, _I32]
    lib.mrp_edge_encoder_bwd_workspace.restype = ctypes.c_int64
    lib.mrp_edge_encoder_bwd.argtypes = [_P, _P, _P, _P, _I32, _I32, _P, _P, _P, _P, _P]
    lib.mrp_edge_encoder_bwd.restype = ctypes.c_int
    lib.mrp_frame_graph_build.argtypes = [_P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P]
    lib.mrp_frame_graph_build.restype = ctypes.c_int
    lib.mrp_stream_copy.argtypes = [_P, _P, _I64, _P]
    lib.mrp_stream_copy.restype = ctypes.c_int
    lib.mrp_stream_join.argtypes = [_P, _P]
    lib.mrp_stream_join.restype = ctypes.c_int
    lib.mrp_abi_version.argtypes = []
    lib.mrp_abi_version.restype = ctypes.c_int
    lib.mrp_error_string.argtypes = [ctypes.c_int]
    lib.mrp_error_string.restype = ctypes.c_char_p


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and return the HIP library; raise if it has not been built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.isfile(path):
            raise RuntimeError(
                f"mrp_gnn: HIP library not found at {path}. Build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950). "
                "There is no CPU fallback for the aggregation kernels."
            )
        lib = ctypes.CDLL(path)
        _declare(lib)
        got = lib.mrp_abi_version()
        if got != ABI_VERSION:
            raise RuntimeError(f"mrp_gnn: ABI version mismatch: library {got}, bindings {ABI_VERSION}")
        _lib = lib
        return lib


def check(code: int, what: str) -> None:
    if code != 0:
        msg = load_library().mrp_error_string(code)
        text = msg.decode() if msg else "unknown error"
        raise RuntimeError(f"mrp_gnn: {what} failed with HIP error {code}: {text}")
