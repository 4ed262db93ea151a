"""Fused edge encoder on the GPU: the FiLM parameters of ``edge_encoder.forward``
(``dgl/model/models.py:146-154``) from one HIP kernel (``mrp_edge_encoder_fwd``).

Forward: ``sigmoid(W2 relu(W1 pose + b1) + b2)`` -> (E, 2C), hidden activations kept on chip,
second Linear on the fp32 MFMA.  Backward (training only) recomputes the hidden activations and
uses library GEMMs (``torch.matmul`` on rocBLAS): it is not on the forward hot path.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def encoder_forward(pose, w1, b1, w2, b2) -> torch.Tensor:
    E = pose.shape[0]
    C = w1.shape[0]
    if pose.shape[1] != 9 or tuple(w1.shape) != (C, 9) or tuple(w2.shape) != (2 * C, C):
        raise ValueError("edge encoder shapes must be pose (E,9), w1 (C,9), w2 (2C,C)")
    if not pose.is_cuda:
        raise RuntimeError("mrp_gnn: the fused edge encoder runs only on the GPU; no CPU fallback")
    pose, w1, b1, w2, b2 = (t.contiguous().float() for t in (pose, w1, b1, w2, b2))
    out = torch.empty((E, 2 * C), device=pose.device, dtype=torch.float32)
    lib = _lib.load_library()
    with torch.cuda.device(pose.device):
        code = lib.mrp_edge_encoder_fwd(_ptr(pose), _ptr(w1), _ptr(b1), _ptr(w2), _ptr(b2), E, C, _ptr(out),
                                        ctypes.c_void_p(torch.cuda.current_stream(pose.device).cuda_stream))
    _lib.check(code, "mrp_edge_encoder_fwd")
    return out


class EdgeEncoderFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pose, w1, b1, w2, b2):
        out = encoder_forward(pose, w1, b1, w2, b2)
        ctx.save_for_backward(pose, w1, b1, w2, out)
        return out

    @staticmethod
    def backward(ctx, gout):
        pose, w1, b1, w2, out = ctx.saved_tensors
        pose = pose.float()
        h_pre = torch.addmm(b1, pose, w1.t())
        h = torch.relu(h_pre)
        dz = gout * out * (1.0 - out)  # sigmoid'
        dw2 = dz.t().mm(h)
        db2 = dz.sum(0)
        dh = dz.mm(w2) * (h_pre > 0)
        dw1 = dh.t().mm(pose)
        db1 = dh.sum(0)
        dpose = dh.mm(w1) if ctx.needs_input_grad[0] else None
        return dpose, dw1, db1, dw2, db2


def fused_film_params(enc_layers: torch.nn.Sequential, pose: torch.Tensor) -> torch.Tensor:
    """(E, 2C) FiLM parameters from the reference-layout ``nn.Sequential`` (layers 0 and 2)."""
    l1, l2 = enc_layers[0], enc_layers[2]
    return EdgeEncoderFunction.apply(pose, l1.weight, l1.bias, l2.weight, l2.bias)
