"""The no-grad GCN layer in ONE launch: ``mrp_gcn_fwd_fused`` (``csrc/gcn_fused.hip``).

Replaces, in the reference's eval path (``torch.no_grad()`` around the model, ``dgl/eval.py:184-199``,
``dgl/training.py:225-240``), the two steps of ``GCN.forward`` (``dgl/model/models.py:219-226``)::

    gamma, beta = edge_encoder(g.edata['pose'])   # models.py:222
    g.update_all(edge_udf, node_udf)               # models.py:223

which the two-launch path runs as ``mrp_edge_encoder_fwd_split`` then ``film_fwd``.  Here the first
workgroups of one grid compute the encoder's logits graph by graph on the matrix cores while the rest
aggregate, each aggregation workgroup waiting only for its own graph's rows; the logits and the
aggregate are bit-identical to the two-launch path (tests/test_gpu_fused.py).

Shapes it serves: complete graphs of 2..8 nodes (the reference's topology, ``dgl/dataloader.py:88-95``),
FiLM-mean, C % 64 == 0, planes of whole 16-byte slices; anything else returns None and the caller
runs the two launches (both HIP; there is no CPU path).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib
from .aggregate import node_stride
from .encoder import PATH_COUNTS, packed_weights
from .graph import GraphCSR

_ENABLED = True


def set_fused_forward(on: bool) -> None:
    """Enable (default) or disable the one-launch no-grad layer (A/B comparisons)."""
    global _ENABLED
    _ENABLED = bool(on)


def fused_forward_enabled() -> bool:
    return _ENABLED


# hand-off words per (device, stream): the call zeroes them itself before its kernel, so a workspace
# is reused across calls on one stream (two streams never share one)
_workspaces = {}
_last_block = {}  # (device, stream) -> (workspace, bytes the last call used)


def _workspace(dev: torch.device, stream: int, nbytes: int) -> torch.Tensor:
    key = (dev.index, stream)
    ws = _workspaces.get(key)
    if ws is None or ws.numel() * 4 < nbytes:
        ws = torch.empty((nbytes + 3) // 4, device=dev, dtype=torch.int32)
        _workspaces[key] = ws
    return ws


def error_word(dev: torch.device, stream: Optional[int] = None) -> int:
    """The last fused launch's error word on ``dev``'s current stream (1 = a hand-off wait timed out;
    never expected): synchronises the device.  Test hook."""
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    hit = _last_block.get((dev.index, stream))
    if hit is None:
        return 0
    ws, nbytes = hit
    torch.cuda.synchronize(dev)
    return int(ws[nbytes // 4 - 64].item())  # the zeroed block's last 256 bytes hold the error word


def gcn_forward_fused(x: torch.Tensor, pose: torch.Tensor, csr: GraphCSR, l1: torch.nn.Linear,
                      l2: torch.nn.Linear, z_out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """FiLM-mean aggregate of ``x`` with gamma/beta = sigmoid(encoder(pose)), one launch; None when the
    shape is not one the fused launch serves.  ``z_out`` (E, 2C), if given, receives the logits."""
    if not _ENABLED or csr.graph_kind != _lib.GRAPH_COMPLETE or not (2 <= csr.max_nodes <= 8):
        return None
    if x.dim() != 4 or x.dtype != torch.float32 or not x.is_cuda:
        return None
    n, C, H, W = x.shape
    P = H * W
    if n != csr.num_nodes or l1.bias is None or tuple(l1.weight.shape) != (C, 9) \
            or tuple(l2.weight.shape) != (2 * C, C) or pose.dim() != 2 or pose.shape[1] != 9:
        return None
    lib = _lib.load_library()
    nbytes = int(lib.mrp_gcn_fwd_fused_workspace_bytes(csr.num_graphs, csr.max_nodes, C, P))
    if nbytes <= 0:
        return None
    xs = node_stride(x)
    if xs is None:
        x = x.contiguous()
        xs = C * P
    E = csr.num_edges
    pose = pose.detach().contiguous().float()
    img = packed_weights(l1, l2)
    b2 = l2.bias.detach().contiguous().float() if l2.bias is not None else None
    z = z_out if z_out is not None else torch.empty((E, 2 * C), device=x.device, dtype=torch.float32)
    if tuple(z.shape) != (E, 2 * C) or not z.is_contiguous() or z.dtype != torch.float32:
        raise ValueError(f"z_out must be a contiguous ({E}, {2 * C}) float32 tensor")
    out = torch.empty((n, C, H, W), device=x.device, dtype=torch.float32)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    ws = _workspace(x.device, stream, nbytes)
    _last_block[(x.device.index, stream)] = (ws, nbytes)
    with torch.cuda.device(x.device):
        code = lib.mrp_gcn_fwd_fused(
            ctypes.c_void_p(x.data_ptr()), xs, ctypes.c_void_p(pose.data_ptr()), ctypes.c_void_p(img.data_ptr()),
            ctypes.c_void_p(b2.data_ptr()) if b2 is not None else None, csr.num_graphs, csr.max_nodes, C, P,
            ctypes.c_void_p(z.data_ptr()), ctypes.c_void_p(out.data_ptr()), C * P, ctypes.c_void_p(ws.data_ptr()),
            ws.numel() * 4, ctypes.c_void_p(stream))
    if code == _lib.HIP_ERROR_NOT_SUPPORTED:
        return None
    _lib.check(code, "mrp_gcn_fwd_fused")
    PATH_COUNTS["fused"] += 1
    return out
