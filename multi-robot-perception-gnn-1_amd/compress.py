"""The 1x1 compress convolution after the concatenation (``dgl/model/models.py:163-165,181-184,186-189``:
``h = conv(torch.cat((h, g_h), 1))`` with ``conv = nn.Conv2d(2C, C, kernel_size=1)``) and both of its
gradients on hand-written matrix-core kernels (``include/mrp_gnn.h``).

Per node n a 1x1 convolution over NCHW is ``y[n] = W [x[n]; a[n]] + b`` with W (C, 2C) shared, so:

* forward:      one GEMM whose K rows come from two tensors (x and the aggregate) — the (N, 2C, H, W)
  concatenation is never written;
* data grad:    ``[dx[n]; da[n]] = W^T dy[n]``, written straight into x's gradient half and the
  aggregate's gradient (which the aggregation backward then consumes) — no (N, 2C, H, W) buffer;
* weight grad:  ``dW = sum_n dy[n] [x[n]; a[n]]^T`` and ``db = sum dy`` in one split-K kernel with a
  fixed-order sum of its partial tiles (deterministic), no (N, C, 2C) temporary, no layout copies.

Arithmetic (:func:`set_compress_path`): ``"split"`` (default) runs all three products on the bf16
matrix cores with every fp32 operand split exactly into three bf16 parts and six partial products per
product (``mrp_compress_fwd_split`` / ``_bwd_data_split`` / ``_bwd_weight_split``, as accurate as an
fp32 GEMM: the omitted terms are below 2^-25 of each product; the weight gradient where C % 64 == 0);
``"hip"`` runs all three on the fp32 MFMA (``mrp_compress_fwd`` / ``_bwd_data`` / ``_bwd_weight``, exact
fp32 products).  Both are checked against float64 (``tests/stack_ref``).  The split weight images are
built once per weight version (:func:`packed_weight`).

The module keeps the reference's ``nn.Conv2d`` parameters (``conv1.weight`` (C, 2C, 1, 1),
``conv1.bias``), so ``state_dict`` keys are unchanged.

Shapes the kernels do not tile (C % 32 != 0, H W % 4 != 0 — and, for the weight gradient only,
H W % 32 != 0 — none of them a reference configuration: the reference's planes are
``image_size/32`` squares, 8 x 8 at its default) run the same kernels on zero-padded operands
(:func:`_fwd`, :func:`_bwd_data`, :func:`_bwd_weight`); ``set_compress_path("library")`` runs
torch's own GEMMs everywhere, for A/B measurements only.
"""
from __future__ import annotations

import weakref

import torch

from . import _lib

_PATH = ["split"]
# products the "split" path runs on the split-bf16 kernels (the rest on the fp32 MFMA): "fwd", "dgrad",
# "wgrad" (set_compress_path(..., split_ops=...); for A/B and accuracy studies)
_SPLIT_OPS = {"fwd", "dgrad", "wgrad"}


def _split(op: str) -> bool:
    return _PATH[0] == "split" and op in _SPLIT_OPS


def set_compress_path(path: str, split_ops=None) -> None:
    """``"split"`` (default): forward, data gradient and weight gradient on the split-bf16 matrix
    cores (``compress_split.hip``, fp32-accurate; the weight gradient falls back to the fp32 MFMA
    where C % 64 or H W % 32 is not 0); ``split_ops`` narrows which of "fwd" / "dgrad" / "wgrad" take
    the split kernels; ``"hip"``: all three on
    the fp32 MFMA (``compress_gemm.hip``); ``"library"``: the cat kernel + torch's library GEMMs (the
    round-2 path), for A/B measurement."""
    if path not in ("split", "hip", "library"):
        raise ValueError("compress path must be 'split', 'hip' or 'library'")
    _PATH[0] = path
    if split_ops is not None:
        ops = set(split_ops)
        if not ops <= {"fwd", "dgrad", "wgrad"}:
            raise ValueError("split_ops: a subset of {'fwd', 'dgrad', 'wgrad'}")
        _SPLIT_OPS.clear()
        _SPLIT_OPS.update(ops)


# packed split-bf16 images of a compress weight, per weight tensor: id -> (weakref, {"fwd" | "bwd":
# (key, image)}), dropped when the tensor dies (tensors compare elementwise, so no WeakKeyDictionary).
# The key holds the data pointer and autograd version, so an optimizer step (an in-place update under
# no_grad) triggers a repack; writes through ``.data`` bypass the version counter: call
# :func:`clear_packed_weights` after those.  Kept outside the modules (not pickled, not deep-copied).
_packed = {}


def clear_packed_weights() -> None:
    _packed.clear()
    _padded_w.clear()


def packed_weight(weight: torch.Tensor, kind: str) -> torch.Tensor:
    """``mrp_compress_split_pack`` image of the (C, 2C[, 1, 1]) weight: ``"fwd"`` packs W (M = C,
    K = 2C) for the forward, ``"bwd"`` packs W^T (M = 2C, K = C) for the data gradient."""
    from .aggregate import _ptr, _stream
    key = (weight.data_ptr(), weight._version, weight.device.index)
    entry = _packed.get(id(weight))
    slot = entry[1] if entry is not None and entry[0]() is weight else None
    if slot is not None and kind in slot and slot[kind][0] == key:
        return slot[kind][1]
    C = weight.shape[0]
    w = _weight2d(weight)
    M, K, trans = (C, 2 * C, 0) if kind == "fwd" else (2 * C, C, 1)
    lib = _lib.load_library()
    img = torch.empty((int(lib.mrp_compress_split_pack_bytes(M, K)) + 3) // 4, device=w.device, dtype=torch.float32)
    with torch.cuda.device(w.device):
        _lib.check(lib.mrp_compress_split_pack(_ptr(w), 2 * C, trans, M, K, _ptr(img), _stream(w.device)),
                   "mrp_compress_split_pack")
    if slot is None:
        slot = {}
        wid = id(weight)
        _packed[wid] = (weakref.ref(weight, lambda _r, wid=wid: _packed.pop(wid, None)), slot)
    slot[kind] = (key, img)
    return img


def compress_path() -> str:
    return _PATH[0]


def _nstride(t: torch.Tensor):
    """Node stride of an (N, C, H, W) fp32 tensor laid out as the kernels need (each node's C H W
    block contiguous, 16-byte aligned, stride % 4 == 0), else None."""
    from .aggregate import node_stride
    s = node_stride(t)
    if s is None or s % 4 != 0 or t.data_ptr() % 16 != 0:
        return None
    return s


def _node_major(t: torch.Tensor):
    s = _nstride(t)
    if s is None:
        t = t.contiguous()
        s = t.shape[1] * t.shape[2] * t.shape[3]
    return t, s


def _weight2d(weight: torch.Tensor) -> torch.Tensor:
    C = weight.shape[0]
    w = weight.detach().reshape(C, weight.shape[1])
    if not w.is_contiguous() or w.dtype != torch.float32:
        w = w.float().contiguous()
    return w


def conv_is_plain_1x1(conv: torch.nn.Conv2d, C: int) -> bool:
    return (conv.kernel_size == (1, 1) and conv.stride == (1, 1) and conv.groups == 1 and conv.dilation == (1, 1)
            and conv.padding in ((0, 0), "valid") and tuple(conv.weight.shape[:2]) == (C, 2 * C)
            and conv.weight.dtype == torch.float32)


def kernels_supported(C: int, P: int) -> bool:
    """The forward and data-gradient kernels: C % 32 == 0, P % 4 == 0 (``include/mrp_gnn.h``)."""
    return C > 0 and P > 0 and C % 32 == 0 and P % 4 == 0


def compress_forward(weight: torch.Tensor, bias, x: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
    """``conv(torch.cat((x, a), 1))`` for a (C, 2C, 1, 1) weight without the concatenation
    (``mrp_compress_fwd``); x and a are (N, C, H, W), e.g. views of a cat buffer's halves."""
    from .aggregate import _ptr, _stream
    n, C, H, W = x.shape
    x, xs = _node_major(x)
    a, as_ = _node_major(a)
    w = _weight2d(weight)
    b = bias.detach() if bias is not None else None
    if b is not None and (b.dtype != torch.float32 or not b.is_contiguous()):
        b = b.float().contiguous()
    y = torch.empty((n, C, H, W), device=x.device, dtype=torch.float32)
    lib = _lib.load_library()
    with torch.cuda.device(x.device):
        if _split("fwd"):
            img = packed_weight(weight, "fwd")
            _lib.check(lib.mrp_compress_fwd_split(_ptr(x), xs, _ptr(a), as_, n, C, H * W, _ptr(img), _ptr(b), _ptr(y),
                                                  C * H * W, _stream(x.device)), "mrp_compress_fwd_split")
        else:
            _lib.check(lib.mrp_compress_fwd(_ptr(x), xs, _ptr(a), as_, n, C, H * W, _ptr(w), _ptr(b), _ptr(y),
                                            C * H * W, _stream(x.device)), "mrp_compress_fwd")
    return y


def compress_backward_data(weight: torch.Tensor, gy: torch.Tensor, gx: torch.Tensor = None, ga: torch.Tensor = None):
    """(gx, ga) = (W[:, :C]^T gy, W[:, C:]^T gy) per node (``mrp_compress_bwd_data``), written into
    the given (N, C, H, W) outputs (e.g. the halves of a cat buffer's gradient) or new tensors."""
    from .aggregate import _ptr, _stream
    n, C, H, W = gy.shape
    lib = _lib.load_library()
    gy, gs = _node_major(gy)
    gx = torch.empty((n, C, H, W), device=gy.device, dtype=torch.float32) if gx is None else gx
    ga = torch.empty((n, C, H, W), device=gy.device, dtype=torch.float32) if ga is None else ga
    gxs, gas = _nstride(gx), _nstride(ga)
    if gxs is None or gas is None:
        raise ValueError("compress_backward_data: outputs must be node-major fp32, 16-byte aligned")
    st = _stream(gy.device)
    with torch.cuda.device(gy.device):
        if _split("dgrad"):
            img = packed_weight(weight, "bwd")
            _lib.check(lib.mrp_compress_bwd_data_split(_ptr(gy), gs, n, C, H * W, _ptr(img), _ptr(gx), gxs, _ptr(ga),
                                                       gas, st), "mrp_compress_bwd_data_split")
            return gx, ga
        w = _weight2d(weight)
        wt = torch.empty((2 * C, C), device=gy.device, dtype=torch.float32)
        _lib.check(lib.mrp_compress_weight_transpose(_ptr(w), _ptr(wt), C, st), "mrp_compress_weight_transpose")
        _lib.check(lib.mrp_compress_bwd_data(_ptr(gy), gs, n, C, H * W, _ptr(wt), _ptr(gx), gxs, _ptr(ga), gas, st),
                   "mrp_compress_bwd_data")
    return gx, ga


def compress_backward_weight(gy: torch.Tensor, x: torch.Tensor, a: torch.Tensor, want_bias: bool = True,
                             weight: torch.Tensor = None, bias: torch.Tensor = None, want_weight: bool = True):
    """(dW (C, 2C, 1, 1), db (C) or None) = (sum_n gy[n] [x[n]; a[n]]^T, sum gy)
    (``mrp_compress_bwd_weight``); None when the kernel declines the shape (H W % 32 != 0).  Given
    the parameters, the results are written straight into a gradient all-reducer's buckets when
    one holds them (``dist.grad_out_like``) — only for a gradient that is wanted, and the slots are
    given back (``dist.release_grad_out``) when the kernel declines the shape."""
    from .aggregate import _ptr, _stream
    from .dist import grad_out_like, release_grad_out
    n, C, H, W = gy.shape
    lib = _lib.load_library()
    gy, gs = _node_major(gy)
    x, xs = _node_major(x)
    a, as_ = _node_major(a)
    claimed = []
    dw = grad_out_like(weight) if want_weight and weight is not None and weight.dim() == 4 else None
    if dw is not None:
        claimed.append((weight, dw))
    else:
        dw = torch.empty((C, 2 * C, 1, 1), device=gy.device, dtype=torch.float32)
    db = None
    if want_bias:
        db = grad_out_like(bias) if bias is not None else None
        if db is not None:
            claimed.append((bias, db))
        else:
            db = torch.empty((C,), device=gy.device, dtype=torch.float32)
    P = H * W
    split = _split("wgrad") and C % 64 == 0 and P % 32 == 0
    if split:
        nbytes = int(lib.mrp_compress_bwd_weight_split_workspace(n, C, P))
        fn, name = lib.mrp_compress_bwd_weight_split, "mrp_compress_bwd_weight_split"
    else:
        nbytes = int(lib.mrp_compress_bwd_weight_workspace(n, C, P, max(gs, xs, as_)))
        fn, name = lib.mrp_compress_bwd_weight, "mrp_compress_bwd_weight"
    done = False
    try:  # claimed bucket slots go back unless the kernel wrote them (declined shape, error, exception)
        ws = torch.empty((nbytes + 3) // 4, device=gy.device, dtype=torch.float32) if nbytes > 0 else None
        with torch.cuda.device(gy.device):
            code = fn(_ptr(gy), gs, _ptr(x), xs, _ptr(a), as_, n, C, P, _ptr(dw), _ptr(db), _ptr(ws), nbytes,
                      _stream(gy.device))
        if code == _lib.HIP_ERROR_NOT_SUPPORTED:
            return None
        _lib.check(code, name)
        done = True
        return dw, db
    finally:
        if not done:
            for p, v in claimed:
                release_grad_out(p, v)


# ---- torch library GEMMs: the A/B comparison path and the shapes the kernels decline -------------

def _lib_forward(weight, bias, x, a):
    n, C, H, W = x.shape
    cat = torch.cat((x, a), 1).reshape(n, 2 * C, H * W)
    w2 = weight.reshape(C, 2 * C)
    y = torch.baddbmm(bias.view(1, C, 1), w2.expand(n, C, 2 * C), cat) if bias is not None else \
        torch.bmm(w2.expand(n, C, 2 * C), cat)
    return y.view(n, C, H, W)


def _lib_backward_data(weight, gy):
    n, C, H, W = gy.shape
    d = torch.bmm(weight.reshape(C, 2 * C).t().expand(n, 2 * C, C), gy.reshape(n, C, H * W)).view(n, 2 * C, H, W)
    return d[:, :C], d[:, C:]


def _lib_backward_weight(gy, x, a, want_bias):
    n, C, H, W = gy.shape
    cat = torch.cat((x, a), 1)
    g2 = gy.reshape(n, C, H * W).permute(1, 0, 2).reshape(C, -1)
    h2 = cat.reshape(n, 2 * C, H * W).permute(1, 0, 2).reshape(2 * C, -1)
    return torch.mm(g2, h2.t()).view(C, 2 * C, 1, 1), (gy.sum((0, 2, 3)) if want_bias else None)


# ---- shapes the kernels do not tile: the same kernels on zero-padded operands ---------------------
# C rounded up to 32 and H W to 4 (forward, data gradient) or 32 (weight gradient): padded channels
# carry zero features and zero weight rows / columns, padded pixels zero features and zero gradients,
# so every padded term of every sum is a product with an exact zero and the results are the leading
# blocks of the padded ones.

def _round(n: int, m: int) -> int:
    return (n + m - 1) // m * m


# padded (weight, bias) per weight tensor, keyed like the packed images: id -> (weakref, key, wp, bp)
_padded_w = {}


def _padded_params(weight: torch.Tensor, bias):
    key = (weight.data_ptr(), weight._version, weight.device.index) + \
        ((bias.data_ptr(), bias._version) if bias is not None else ())
    hit = _padded_w.get(id(weight))
    if hit is not None and hit[0]() is weight and hit[1] == key:
        return hit[2], hit[3]
    C = weight.shape[0]
    Cp = _round(C, 32)
    w = _weight2d(weight)
    with torch.no_grad():
        wp = torch.zeros((Cp, 2 * Cp, 1, 1), device=w.device, dtype=torch.float32)
        wp[:C, :C, 0, 0] = w[:, :C]
        wp[:C, Cp:Cp + C, 0, 0] = w[:, C:]
        bp = None
        if bias is not None:
            bp = torch.zeros((Cp,), device=w.device, dtype=torch.float32)
            bp[:C] = bias.detach()
    wid = id(weight)
    _padded_w[wid] = (weakref.ref(weight, lambda _r, wid=wid: _padded_w.pop(wid, None)), key, wp, bp)
    return wp, bp


def _pad_planes(t: torch.Tensor, Cp: int, Pp: int) -> torch.Tensor:
    """(N, C, H, W) -> (N, Cp, Pp, 1) with t in the leading (C, H W) block, zeros elsewhere."""
    n, C, H, W = t.shape
    out = torch.zeros((n, Cp, Pp, 1), device=t.device, dtype=torch.float32)
    out.view(n, Cp, Pp)[:, :C, : H * W] = t.reshape(n, C, H * W)
    return out


def _unpad_planes(t: torch.Tensor, C: int, H: int, W: int) -> torch.Tensor:
    n, Cp, Pp, _ = t.shape
    return t.view(n, Cp, Pp)[:, :C, : H * W].contiguous().view(n, C, H, W)


def _fwd(weight, bias, x, a):
    n, C, H, W = x.shape
    if kernels_supported(C, H * W):
        return compress_forward(weight, bias, x, a)
    Cp, Pp = _round(C, 32), _round(H * W, 4)
    wp, bp = _padded_params(weight, bias)
    y = compress_forward(wp, bp, _pad_planes(x, Cp, Pp), _pad_planes(a, Cp, Pp))
    return _unpad_planes(y, C, H, W)


def _bwd_data(weight, gy):
    n, C, H, W = gy.shape
    if kernels_supported(C, H * W):
        return compress_backward_data(weight, gy)
    Cp, Pp = _round(C, 32), _round(H * W, 4)
    wp, _ = _padded_params(weight, None)
    gx, ga = compress_backward_data(wp, _pad_planes(gy, Cp, Pp))
    return _unpad_planes(gx, C, H, W), _unpad_planes(ga, C, H, W)


def _bwd_weight(gy, x, a, want_bias, weight, bias, want_weight=True):
    n, C, H, W = gy.shape
    if kernels_supported(C, H * W):
        r = compress_backward_weight(gy, x, a, want_bias, weight, bias, want_weight=want_weight)
        if r is not None:
            return r
    Cp, Pp = _round(C, 32), _round(H * W, 32)
    r = compress_backward_weight(*(_pad_planes(t, Cp, Pp) for t in (gy, x, a)), want_bias)
    if r is None:
        raise RuntimeError(f"mrp_gnn: the compress weight-gradient kernels declined the padded shape C={Cp}, HW={Pp}")
    dwp, dbp = r
    dw = torch.cat((dwp[:C, :C], dwp[:C, Cp:Cp + C]), 1)
    return dw, (dbp[:C].contiguous() if dbp is not None else None)


class CompressFunction(torch.autograd.Function):
    """``conv(torch.cat((x, a), 1))`` with autograd, x and a separate (N, C, H, W) tensors."""

    @staticmethod
    def forward(ctx, x, a, weight, bias):
        hip = _PATH[0] != "library"
        y = _fwd(weight, bias, x, a) if hip else _lib_forward(weight, bias, x, a)
        ctx.save_for_backward(x, a, weight)
        ctx.hip, ctx.has_bias = hip, bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, a, weight = ctx.saved_tensors
        gx = ga = dw = db = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            gx, ga = _bwd_data(weight, gy) if ctx.hip else _lib_backward_data(weight, gy)
        if ctx.needs_input_grad[2] or (ctx.has_bias and ctx.needs_input_grad[3]):
            dw, db = _bwd_weight(gy, x, a, ctx.has_bias, None, None) if ctx.hip else \
                _lib_backward_weight(gy, x, a, ctx.has_bias)
        return gx, ga, dw, db


class LibraryCompressFunction(torch.autograd.Function):
    """``conv(h)`` over a (N, 2C, H, W) concatenation buffer on torch's library GEMMs (the round-2
    path: batched GEMM forward and data gradient, one GEMM with K = N H W for the weight gradient)."""

    @staticmethod
    def forward(ctx, h, weight, bias):
        n, k, H, W = h.shape
        C = weight.shape[0]
        h = h.contiguous()
        w2 = weight.reshape(C, k)
        y = torch.baddbmm(bias.view(1, C, 1), w2.expand(n, C, k), h.view(n, k, H * W)) if bias is not None else \
            torch.bmm(w2.expand(n, C, k), h.view(n, k, H * W))
        ctx.save_for_backward(h, weight)
        ctx.has_bias = bias is not None
        return y.view(n, C, H, W)

    @staticmethod
    def backward(ctx, gy):
        h, weight = ctx.saved_tensors
        n, k, H, W = h.shape
        C = weight.shape[0]
        gy = gy.contiguous()
        dh = dw = db = None
        if ctx.needs_input_grad[0]:
            dh = torch.bmm(weight.reshape(C, k).t().expand(n, k, C), gy.view(n, C, H * W)).view(n, k, H, W)
        if ctx.needs_input_grad[1]:
            g2 = gy.reshape(n, C, H * W).permute(1, 0, 2).reshape(C, -1)
            h2 = h.reshape(n, k, H * W).permute(1, 0, 2).reshape(k, -1)
            dw = torch.mm(g2, h2.t()).view(weight.shape)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = gy.sum((0, 2, 3))
        return dh, dw, db


def compress_1x1(conv: torch.nn.Conv2d, h: torch.Tensor) -> torch.Tensor:
    """``conv(h)`` for the reference's 1x1 compress conv over a (N, 2C, H, W) concatenation h: the
    matrix-core kernels read its two halves in place (``set_compress_path('library')``: torch's
    library GEMMs)."""
    C = h.shape[1] // 2
    if not h.is_cuda or h.dtype != torch.float32 or h.shape[1] != 2 * C or not conv_is_plain_1x1(conv, C):
        return conv(h)
    if _PATH[0] == "library":
        return LibraryCompressFunction.apply(h, conv.weight, conv.bias)
    return CompressFunction.apply(h[:, :C], h[:, C:], conv.weight, conv.bias)


class FilmCompressFunction(torch.autograd.Function):
    """``conv(torch.cat((x, film_mean(x, gb)), 1))`` (``models.py:181-184``) with autograd and without
    the concatenation: forward = the aggregation kernel into its own (N, C, H, W) output, then the
    two-source compress.  Backward: ``[gx; ga] = W^T dy`` by the data-gradient kernel, ONE
    aggregation-backward pass with ga as its grad_out and gx as the base of x's gradient (x's two
    gradient terms are never added by a separate kernel), and the weight gradient from x and the
    saved aggregate.  Saves x, gb and the aggregate — not a 2C-channel buffer."""

    @staticmethod
    def forward(ctx, x, gb, weight, bias, csr, mode: int):
        from .aggregate import film_mean_forward_into
        n, C, H, W = x.shape
        agg = torch.empty(x.shape, device=x.device, dtype=torch.float32)
        film_mean_forward_into(x, gb, csr, mode, agg)
        hip = _PATH[0] != "library"
        y = _fwd(weight, bias, x, agg) if hip else _lib_forward(weight, bias, x, agg)
        ctx.save_for_backward(x, gb, agg, weight, bias)
        ctx.csr, ctx.mode, ctx.has_bias, ctx.hip = csr, mode, bias is not None, hip
        return y

    @staticmethod
    def backward(ctx, gy):
        from .aggregate import film_mean_backward
        x, gb, agg, weight, bias = ctx.saved_tensors
        need_x, need_gb = ctx.needs_input_grad[0], gb is not None and ctx.needs_input_grad[1]
        dx = dgb = dw = db = None
        if need_x or need_gb:
            gx, ga = _bwd_data(weight, gy) if ctx.hip else _lib_backward_data(weight, gy)
            dx, dgb = film_mean_backward(ga, x, gb, ctx.csr, ctx.mode, need_x, need_gb,
                                         grad_x_base=gx if need_x else None)
            if dgb is not None:
                dgb = dgb.view(gb.shape).to(gb.dtype)
        if ctx.needs_input_grad[2] or (ctx.has_bias and ctx.needs_input_grad[3]):
            dw, db = _bwd_weight(gy, x, agg, ctx.has_bias and ctx.needs_input_grad[3], weight, bias,
                                 want_weight=ctx.needs_input_grad[2]) if ctx.hip else \
                _lib_backward_weight(gy, x, agg, ctx.has_bias)
            if not ctx.needs_input_grad[2]:
                dw = None
        return dx, dgb, dw, db, None, None


def film_compress_supported(conv: torch.nn.Conv2d, x: torch.Tensor) -> bool:
    """Whether :func:`film_compress` takes this layer: fp32 CUDA (N, C, H, W) features and a plain 1x1
    ``Conv2d(2C, C)`` (the matrix-core kernels, or torch's GEMMs for shapes they decline)."""
    return x.dim() == 4 and x.is_cuda and x.dtype == torch.float32 and conv_is_plain_1x1(conv, x.shape[1])


def film_compress(conv: torch.nn.Conv2d, x: torch.Tensor, gb, csr, mode: int) -> torch.Tensor:
    """Autograd form of ``conv(torch.cat((x, film_mean(x, gb)), 1))`` without the concatenation
    (:class:`FilmCompressFunction`); the caller checks :func:`film_compress_supported`."""
    if gb is not None:
        gb = gb.reshape(csr.num_edges, x.shape[1], 2)
    return FilmCompressFunction.apply(x, gb, conv.weight, conv.bias, csr, mode)
