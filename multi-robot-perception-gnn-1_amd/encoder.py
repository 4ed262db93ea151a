"""Edge encoder on the GPU (``dgl/model/models.py:146-154``), restructured for the hot path.

``z = W2 relu(W1 pose + b1) + b2``, ``gamma/beta = sigmoid(z)``:

* ``relu(W1 pose + b1)`` — one HIP kernel (``mrp_edge_hidden_fwd``; K = 9, a streaming write);
* ``h W2^T + b2``        — a plain library GEMM (``torch.addmm`` -> hipBLASLt/rocBLAS, bias in the
  epilogue): the encoder's only dense contraction;
* ``sigmoid``            — not run here: the aggregation kernels take the logits
  (``MRP_AGG_GB_LOGITS``) and apply it while building their tiles.

The hidden layer's backward (training only) is torch ops; it is not on the forward hot path.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def hidden_forward(pose, w1, b1) -> torch.Tensor:
    """relu(pose @ w1.T + b1), (E, C), via the HIP kernel."""
    E = pose.shape[0]
    C = w1.shape[0]
    if pose.dim() != 2 or pose.shape[1] != 9 or tuple(w1.shape) != (C, 9) or tuple(b1.shape) != (C,):
        raise ValueError("edge hidden layer shapes must be pose (E,9), w1 (C,9), b1 (C,)")
    if not pose.is_cuda:
        raise RuntimeError("mrp_gnn: the edge hidden-layer kernel runs only on the GPU; no CPU fallback")
    pose, w1, b1 = (t.contiguous().float() for t in (pose, w1, b1))
    h = torch.empty((E, C), device=pose.device, dtype=torch.float32)
    lib = _lib.load_library()
    with torch.cuda.device(pose.device):
        code = lib.mrp_edge_hidden_fwd(_ptr(pose), _ptr(w1), _ptr(b1), E, C, _ptr(h),
                                       ctypes.c_void_p(torch.cuda.current_stream(pose.device).cuda_stream))
    _lib.check(code, "mrp_edge_hidden_fwd")
    return h


class EdgeHiddenFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pose, w1, b1):
        h = hidden_forward(pose, w1, b1)
        ctx.save_for_backward(pose, w1, h)
        return h

    @staticmethod
    def backward(ctx, gh):
        pose, w1, h = ctx.saved_tensors
        dpre = gh * (h > 0)
        dw1 = dpre.t().mm(pose.float())
        db1 = dpre.sum(0)
        dpose = dpre.mm(w1) if ctx.needs_input_grad[0] else None
        return dpose, dw1, db1


def edge_logits(enc_layers: torch.nn.Sequential, pose: torch.Tensor) -> torch.Tensor:
    """Pre-sigmoid FiLM logits z (E, 2C) from the reference-layout ``nn.Sequential``
    (layers 0 and 2 are the Linears)."""
    l1, l2 = enc_layers[0], enc_layers[2]
    h = EdgeHiddenFunction.apply(pose, l1.weight, l1.bias)
    return torch.addmm(l2.bias, h, l2.weight.t())
