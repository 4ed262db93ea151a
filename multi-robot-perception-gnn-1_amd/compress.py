"""The 1x1 compress convolution after the concatenation (``dgl/model/models.py:165-171,183,189``:
``conv1``/``conv2 = nn.Conv2d(2C, C, kernel_size=1)``) as library GEMMs on the fp32 MFMA.

A 1x1 convolution over NCHW is, per node n, ``Y_n = W X_n + b`` with W (C, 2C) shared and X_n the
node's (2C, H*W) block — a strided-batched GEMM with a broadcast A operand.  Measured on MI355X
(``tools/exp_compress*.py``): at Nt=256, C=512, 32x32 the batched GEMM takes 2159 us forward and
2012 us for the input gradient against 2674 / 2363 us for MIOpen's convolution (127 vs 106 TF/s of
the 157 TF/s fp32 MFMA peak); the weight gradient stays MIOpen's (no (Nt, C, 2C) temporary).
Same fp32 arithmetic as the convolution, different summation order: ≤ 1e-5 relative.
The module keeps the reference's ``nn.Conv2d`` parameters (``conv1.weight`` (C, 2C, 1, 1),
``conv1.bias``), so ``state_dict`` keys are unchanged.
"""
from __future__ import annotations

import torch


class Compress1x1Function(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, weight, bias):
        n, k, H, W = h.shape
        c = weight.shape[0]
        h = h.contiguous()
        w2 = weight.reshape(c, k)
        x = h.view(n, k, H * W)
        if bias is not None:
            y = torch.baddbmm(bias.view(1, c, 1), w2.expand(n, c, k), x)
        else:
            y = torch.bmm(w2.expand(n, c, k), x)
        ctx.save_for_backward(h, weight)
        ctx.has_bias = bias is not None
        return y.view(n, c, H, W)

    @staticmethod
    def backward(ctx, gy):
        h, weight = ctx.saved_tensors
        n, k, H, W = h.shape
        c = weight.shape[0]
        gy = gy.contiguous()
        dh = dw = db = None
        if ctx.needs_input_grad[0]:
            dh = torch.bmm(weight.reshape(c, k).t().expand(n, k, c), gy.view(n, c, H * W)).view(n, k, H, W)
        if ctx.needs_input_grad[1]:
            dw = torch.nn.grad.conv2d_weight(h, weight.shape, gy)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = gy.sum((0, 2, 3))
        return dh, dw, db


def compress_1x1(conv: torch.nn.Conv2d, h: torch.Tensor) -> torch.Tensor:
    """``conv(h)`` for the reference's 1x1 compress conv; batched GEMM on the GPU."""
    if not h.is_cuda or conv.kernel_size != (1, 1) or conv.stride != (1, 1) or conv.groups != 1 \
            or conv.padding not in ((0, 0), "valid") or conv.dilation != (1, 1) or h.dtype != torch.float32:
        return conv(h)
    return Compress1x1Function.apply(h, conv.weight, conv.bias)
