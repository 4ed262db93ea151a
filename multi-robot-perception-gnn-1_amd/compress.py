"""The 1x1 compress convolution after the concatenation (``dgl/model/models.py:165-171,183,189``:
``conv1``/``conv2 = nn.Conv2d(2C, C, kernel_size=1)``) as library GEMMs on the fp32 MFMA.

A 1x1 convolution over NCHW is, per node n, ``Y_n = W X_n + b`` with W (C, 2C) shared and X_n the
node's (2C, H*W) block — a strided-batched GEMM with a broadcast A operand.  Measured on MI355X
(``tools/exp_compress*.py``): at Nt=256, C=512, 32x32 the batched GEMM takes 2159 us forward and
2012 us for the input gradient against 2674 / 2363 us for MIOpen's convolution (127 vs 106 TF/s of
the 157 TF/s fp32 MFMA peak).  The weight gradient ``dW = sum_n dy_n h_n^T`` (``weight_grad_1x1``,
``tools/exp_compress_wgrad.py``, against MIOpen's weight-gradient convolution with its NCHW -> NHWC
transposes): on planes of >= 1024 pixels a batched GEMM into an (Nt, C, 2C) temporary + a sum over
nodes (configs[1] 1.04 vs 1.28 ms, headline size 2.06 vs 2.60 ms); on smaller planes, where K = H W
is too short for that, channel-major copies of dy and h and ONE GEMM with K = Nt H W (configs[2]
0.96 vs 1.06 ms, [3] 0.51 vs 0.54, [4] 1.07 vs 1.12).
Same fp32 arithmetic as the convolution, different summation order: ≤ 1e-5 relative.
The module keeps the reference's ``nn.Conv2d`` parameters (``conv1.weight`` (C, 2C, 1, 1),
``conv1.bias``), so ``state_dict`` keys are unchanged.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


# the batched-GEMM weight gradient: planes of at least this many pixels, temporaries up to this size
WGRAD_BMM_MIN_PLANE = 1024
WGRAD_BMM_MAX_TEMP = 1 << 30


def weight_grad_1x1(h: torch.Tensor, wshape, gy: torch.Tensor) -> torch.Tensor:
    """``torch.nn.grad.conv2d_weight(h, wshape, gy)`` for a 1x1 conv over (N, K, H, W) input h and
    (N, C, H, W) output gradient gy (both contiguous fp32), by the faster route for the plane size."""
    n, k, H, W = h.shape
    c = wshape[0]
    P = H * W
    if P >= WGRAD_BMM_MIN_PLANE and n * c * k * 4 <= WGRAD_BMM_MAX_TEMP:
        return torch.bmm(gy.reshape(n, c, P), h.reshape(n, k, P).transpose(1, 2)).sum(0).view(wshape)
    a = gy.reshape(n, c, P).permute(1, 0, 2).reshape(c, n * P)
    bt = h.reshape(n, k, P).permute(1, 0, 2).reshape(k, n * P)
    return torch.mm(a, bt.t()).view(wshape)


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
            dw = weight_grad_1x1(h, weight.shape, gy)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = gy.sum((0, 2, 3))
        return dh, dw, db


def compress_1x1(conv: torch.nn.Conv2d, h: torch.Tensor) -> torch.Tensor:
    """``conv(h)`` for the reference's 1x1 compress conv; batched GEMM on the GPU."""
    if not h.is_cuda or conv.kernel_size != (1, 1) or conv.stride != (1, 1) or conv.groups != 1 \
            or conv.padding not in ((0, 0), "valid") or conv.dilation != (1, 1) or h.dtype != torch.float32:
        return conv(h)
    return Compress1x1Function.apply(h, conv.weight, conv.bias)


def _weight_packed(conv: torch.nn.Conv2d) -> torch.Tensor:
    """The conv weight (C, 2C, 1, 1) in the fused kernel's k4-packed stage layout
    (``mrp_compress_weight_pack``); cached on the module per weight version."""
    from .aggregate import _ptr, _stream
    w = conv.weight
    key = (w.data_ptr(), w._version, w.device)
    hit = getattr(conv, "_mrp_wp", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    C = w.shape[0]
    src = w.detach().reshape(C, 2 * C).contiguous()
    wp = torch.empty(2 * C * C, device=w.device, dtype=torch.float32)
    with torch.cuda.device(w.device):
        _lib.check(_lib.load_library().mrp_compress_weight_pack(_ptr(src), _ptr(wp), C, _stream(w.device)),
                   "mrp_compress_weight_pack")
    conv._mrp_wp = (key, wp)
    return wp


def fused_compress_supported(conv: torch.nn.Conv2d, x: torch.Tensor, csr) -> bool:
    """Whether ``mrp_compress_film_fwd`` covers this layer: fp32 CUDA features, a plain 1x1
    Conv2d(2C, C), complete graphs of 2..8 nodes, H W % 16 == 0, C % 128 == 0."""
    if x.dim() != 4:
        return False
    n, C, H, W = x.shape
    if (not x.is_cuda or x.dtype != torch.float32 or conv.kernel_size != (1, 1) or conv.groups != 1
            or conv.stride != (1, 1) or conv.dilation != (1, 1) or conv.padding not in ((0, 0), "valid")
            or tuple(conv.weight.shape[:2]) != (C, 2 * C) or conv.weight.dtype != torch.float32):
        return False
    return csr.graph_kind == _lib.GRAPH_COMPLETE and 2 <= csr.max_nodes <= 8 and (H * W) % 16 == 0 and C % 128 == 0


def compress_film_fused(conv: torch.nn.Conv2d, x: torch.Tensor, gb, csr, mode: int):
    """``conv(torch.cat((x, film_mean(x, gb)), 1))`` (``models.py:181-184``) in ONE kernel
    (``mrp_compress_film_fwd``): the aggregate is computed inside the 1x1 GEMM's operand producer and
    the (N, 2C, H, W) concatenation never reaches HBM.  Forward only (no autograd).  Returns None
    when the kernel does not cover the shape (non-complete graphs, N > 8, P % 16, C % 128): the
    caller then runs the cat kernel + batched GEMM."""
    if not fused_compress_supported(conv, x, csr):
        return None
    n, C, H, W = x.shape
    from .aggregate import _ptr, _stream, node_stride
    xs = node_stride(x)
    if xs is None:
        x = x.contiguous()
        xs = C * H * W
    lib = _lib.load_library()
    if gb is not None:
        gb = gb.reshape(csr.num_edges, C, 2)
        if not gb.is_contiguous() or gb.dtype != torch.float32:
            gb = gb.contiguous().float()
        if mode & _lib.GB_LOGITS:
            # one elementwise pass to post-sigmoid pairs (the kernels' own sigmoid: same bits as the
            # logits path) instead of 2 x E x C sigmoids in every workgroup of a channel column
            gate = torch.empty_like(gb)
            with torch.cuda.device(x.device):
                _lib.check(lib.mrp_film_gate(_ptr(gb), _ptr(gate), gb.numel(), _stream(x.device)), "mrp_film_gate")
            gb, mode = gate, mode & ~_lib.GB_LOGITS
    wt = _weight_packed(conv)
    bias = conv.bias.detach() if conv.bias is not None else None
    if bias is not None and (bias.dtype != torch.float32 or not bias.is_contiguous()):
        bias = bias.float().contiguous()
    y = torch.empty((n, C, H, W), device=x.device, dtype=torch.float32)
    with torch.cuda.device(x.device):
        code = lib.mrp_compress_film_fwd(_ptr(x), xs, _ptr(gb), csr.num_graphs, csr.max_nodes, csr.graph_kind,
                                         csr.num_nodes, csr.num_edges, C, H * W, mode, _ptr(wt), _ptr(bias),
                                         _ptr(y), C * H * W, _stream(x.device))
    if code == _lib.HIP_ERROR_NOT_SUPPORTED:
        return None
    _lib.check(code, "mrp_compress_film_fwd")
    return y


def dual_compress_supported(conv: torch.nn.Conv2d, x: torch.Tensor) -> bool:
    """Whether ``mrp_compress_dual_fwd`` covers this layer (any graph): fp32 CUDA features, a plain
    1x1 Conv2d(2C, C), C % 128 == 0, H W % 16 == 0."""
    if x.dim() != 4:
        return False
    n, C, H, W = x.shape
    return (x.is_cuda and x.dtype == torch.float32 and conv.kernel_size == (1, 1) and conv.groups == 1
            and conv.stride == (1, 1) and conv.dilation == (1, 1) and conv.padding in ((0, 0), "valid")
            and tuple(conv.weight.shape[:2]) == (C, 2 * C) and conv.weight.dtype == torch.float32
            and C % 128 == 0 and (H * W) % 16 == 0)


def compress_dual(conv: torch.nn.Conv2d, x: torch.Tensor, agg: torch.Tensor):
    """``conv(torch.cat((x, agg), 1))`` for a 1x1 ``Conv2d(2C, C)`` without the concatenation:
    ``mrp_compress_dual_fwd`` (fp32 MFMA, operands staged by LDS-DMA).  Forward only.  None when the
    kernel does not cover the shape (C % 128, H W % 16, alignment)."""
    n, C, H, W = x.shape
    if not dual_compress_supported(conv, x) or agg.shape != x.shape or agg.dtype != torch.float32:
        return None
    from .aggregate import _ptr, _stream, node_stride
    xs, gs = node_stride(x), node_stride(agg)
    if xs is None:
        x = x.contiguous()
        xs = C * H * W
    if gs is None:
        agg = agg.contiguous()
        gs = C * H * W
    wt = _weight_packed(conv)
    bias = conv.bias.detach() if conv.bias is not None else None
    if bias is not None and (bias.dtype != torch.float32 or not bias.is_contiguous()):
        bias = bias.float().contiguous()
    y = torch.empty((n, C, H, W), device=x.device, dtype=torch.float32)
    lib = _lib.load_library()
    with torch.cuda.device(x.device):
        code = lib.mrp_compress_dual_fwd(_ptr(x), xs, _ptr(agg), gs, n, C, H * W, _ptr(wt), _ptr(bias), _ptr(y),
                                         C * H * W, _stream(x.device))
    if code == _lib.HIP_ERROR_NOT_SUPPORTED:
        return None
    _lib.check(code, "mrp_compress_dual_fwd")
    return y



class FilmCompressFunction(torch.autograd.Function):
    """``conv(torch.cat((x, film_mean(x, gb)), 1))`` (``models.py:181-184``) with autograd and without
    the concatenation: forward = the aggregation kernel into its own (N, C, H, W) output, then the
    two-source MFMA compress (``mrp_compress_dual_fwd``) reading x and the aggregate in place.
    Backward: ``d cat = W^T dy`` (one batched GEMM into an (N, 2C, H, W) buffer, as the cat path's),
    then ONE aggregation-backward pass with the first half as the base of x's gradient (so x's two
    gradient terms are never added by a separate kernel), and the weight gradient as two half-width
    GEMMs (x and the aggregate are separate tensors here).  Saves, per layer, the concatenation's
    second copy of x (written by the cat kernel, read by the GEMM) and keeps the aggregate instead of
    the 2C-channel buffer for backward."""

    @staticmethod
    def forward(ctx, x, gb, weight, bias, conv, csr, mode: int):
        from .aggregate import film_mean_forward_into
        agg = torch.empty(x.shape, device=x.device, dtype=torch.float32)
        film_mean_forward_into(x, gb, csr, mode, agg)
        y = compress_dual(conv, x, agg)
        if y is None:
            raise RuntimeError("mrp_compress_dual_fwd does not cover this shape (callers check "
                               "dual_compress_supported first)")
        ctx.save_for_backward(x, gb, agg, weight)
        ctx.csr, ctx.mode, ctx.has_bias = csr, mode, bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        from .aggregate import film_mean_backward
        x, gb, agg, weight = ctx.saved_tensors
        n, C, H, W = x.shape
        gy = gy.contiguous()
        need_x, need_gb = ctx.needs_input_grad[0], gb is not None and ctx.needs_input_grad[1]
        dx = dgb = dw = db = None
        if need_x or need_gb:
            dcat = torch.bmm(weight.reshape(C, 2 * C).t().expand(n, 2 * C, C), gy.view(n, C, H * W))
            dcat = dcat.view(n, 2 * C, H, W)
            dx, dgb = film_mean_backward(dcat[:, C:], x, gb, ctx.csr, ctx.mode, need_x, need_gb,
                                         grad_x_base=dcat[:, :C] if need_x else None)
            if dgb is not None:
                dgb = dgb.view(gb.shape).to(gb.dtype)
        if ctx.needs_input_grad[2]:
            half = (C, C, 1, 1)
            dw = torch.cat((weight_grad_1x1(x.contiguous(), half, gy), weight_grad_1x1(agg, half, gy)), 1)
        if ctx.has_bias and ctx.needs_input_grad[3]:
            db = gy.sum((0, 2, 3))
        return dx, dgb, dw, db, None, None, None


def film_compress(conv: torch.nn.Conv2d, x: torch.Tensor, gb, csr, mode: int) -> torch.Tensor:
    """Autograd form of ``conv(torch.cat((x, film_mean(x, gb)), 1))`` without the concatenation
    (``FilmCompressFunction``); the caller checks ``dual_compress_supported(conv, x)``."""
    if gb is not None:
        gb = gb.reshape(csr.num_edges, x.shape[1], 2)
    return FilmCompressFunction.apply(x, gb, conv.weight, conv.bias, conv, csr, mode)
