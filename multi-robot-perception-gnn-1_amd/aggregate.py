"""FiLM-mean message passing on the GPU: the replacement for ``g.update_all(edge_udf, node_udf)``.

Reference semantics (``dgl/model/models.py:207-211,223``)::

    m_e   = gamma_e * x[src(e)] + beta_e        # edge_udf, gamma/beta broadcast over H x W
    out_v = mean_{e: dst(e) = v} m_e            # node_udf over v's mailbox; zeros if deg v = 0

``gb`` is the edge encoder's sigmoid output viewed ``(E, C, 2)`` (gamma = ``[..., 0]``,
beta = ``[..., 1]``, ``models.py:154-155``) and is read in place, never split or copied.

Everything here dispatches to the HIP library through its C ABI; a CPU tensor raises.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib
from .graph import GraphCSR


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def node_stride(t: torch.Tensor) -> Optional[int]:
    """Node stride of a (N, C, H, W) fp32 tensor whose per-node C*H*W block is contiguous,
    else None (then the caller makes it contiguous)."""
    if t.dim() != 4 or t.dtype != torch.float32:
        return None
    n, c, h, w = t.shape
    if n == 0 or c * h * w == 0:
        return c * h * w
    s = t.stride()
    if (w == 1 or s[3] == 1) and (h == 1 or s[2] == w) and (c == 1 or s[1] == h * w) and (n == 1 or s[0] >= c * h * w):
        return s[0] if n > 1 else c * h * w
    return None


def _as_node_major(t: torch.Tensor):
    s = node_stride(t)
    if s is None:
        t = t.contiguous()
        s = t.shape[1] * t.shape[2] * t.shape[3]
    return t, s


def _require_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                "mrp_gnn: the FiLM-mean aggregation runs only on the GPU (HIP, gfx950); got a "
                f"{t.device} tensor. There is no CPU fallback.")


def _stream(dev: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def film_mean_forward_into(x: torch.Tensor, gb: Optional[torch.Tensor], csr: GraphCSR, mode: int,
                           out: torch.Tensor, epilogue: Optional["EpilogueSpec"] = None) -> torch.Tensor:
    """Run the forward kernel into ``out`` (N, C, H, W) — which may be a strided view such as
    the second half of a ``torch.cat((h, g_h), 1)`` buffer.  No autograd."""
    return _forward(x, gb, csr, mode, out, epilogue=epilogue)


def film_mean_cat_forward_into(x: torch.Tensor, gb: Optional[torch.Tensor], csr: GraphCSR, mode: int,
                               cat: torch.Tensor) -> torch.Tensor:
    """``cat[:, :C] = x; cat[:, C:] = film_mean(x)`` for a (N, 2C, H, W) buffer, one kernel pass
    (``mrp_film_mean_cat_fwd``).  No autograd."""
    C = x.shape[1]
    if cat.dim() != 4 or tuple(cat.shape) != (x.shape[0], 2 * C) + tuple(x.shape[2:]):
        raise ValueError(f"cat must be {(x.shape[0], 2 * C) + tuple(x.shape[2:])} fp32")
    return _forward(x, gb, csr, mode, cat[:, C:], epilogue=EpilogueSpec(xcopy=cat[:, :C]))


class EpilogueSpec:
    """What the forward writes per destination v (``mrp_agg_epilogue``, include/mrp_gnn.h):
    ``out[v] = agg_scale * a + self_scale * x[v] + x0_scale * x0[v]``, optionally also ``xcopy[v] = x[v]``.

    * residual ``h = g_h + h`` (``dgl/model/dgl_models.py:36-37``): ``self_scale=1``;
    * initial-feature mix ``(1 - alpha) a + alpha x0`` (GCN2-style; not in the reference):
      ``agg_scale=1-alpha, x0=h0, x0_scale=alpha``;
    * ``torch.cat((x, a), 1)`` (``dgl/model/models.py:182``): ``xcopy`` = the first half."""

    def __init__(self, agg_scale: float = 1.0, self_scale: float = 0.0, x0: Optional[torch.Tensor] = None,
                 x0_scale: float = 0.0, xcopy: Optional[torch.Tensor] = None):
        self.agg_scale = float(agg_scale)
        self.self_scale = float(self_scale)
        self.x0 = x0
        self.x0_scale = float(x0_scale)
        self.xcopy = xcopy

    def is_plain(self) -> bool:
        return self.agg_scale == 1.0 and self.self_scale == 0.0 and self.x0 is None and self.xcopy is None


def _epilogue_struct(ep: Optional[EpilogueSpec], shape):
    """(ctypes Epilogue or None, tensors to keep alive)."""
    if ep is None or ep.is_plain():
        return None, ()
    keep = []
    x0p, x0s, xcp, xcs = 0, 0, 0, 0
    if ep.x0 is not None:
        if tuple(ep.x0.shape) != tuple(shape):
            raise ValueError(f"x0 must have the node features' shape {tuple(shape)}")
        _require_device(ep.x0)
        x0, x0s = _as_node_major(ep.x0.float() if ep.x0.dtype != torch.float32 else ep.x0)
        keep.append(x0)
        x0p = x0.data_ptr()
    if ep.xcopy is not None:
        xcs = node_stride(ep.xcopy)
        if xcs is None or tuple(ep.xcopy.shape) != tuple(shape):
            raise ValueError("xcopy must be (N, C, H, W) fp32 with a contiguous block per node")
        _require_device(ep.xcopy)
        xcp = ep.xcopy.data_ptr()
    st = _lib.Epilogue(ep.agg_scale, ep.self_scale, x0p, x0s, ep.x0_scale, xcp, xcs)
    return st, keep


def _forward(x, gb, csr, mode, out, epilogue=None):
    _require_device(x, out)
    n, C, H, W = x.shape
    x, xs = _as_node_major(x)
    os_ = node_stride(out)
    if os_ is None or tuple(out.shape) != (n, C, H, W):
        raise ValueError(f"out must be {(n, C, H, W)} fp32 with a contiguous block per node")
    if (mode & ~_lib.GB_LOGITS) != _lib.MODE_COPY_MEAN:
        if gb is None:
            raise ValueError("gamma/beta tensor required for FiLM modes")
        gb = gb.reshape(csr.num_edges, C, 2)
        if not gb.is_contiguous() or gb.dtype != torch.float32:
            gb = gb.contiguous().float()
        _require_device(gb)
    else:
        gb = None
    if n != csr.num_nodes:
        raise ValueError(f"x has {n} nodes, graph has {csr.num_nodes}")
    ep, _keep = _epilogue_struct(epilogue, x.shape)
    lib = _lib.load_library()
    with torch.cuda.device(x.device):
        code = lib.mrp_film_mean_fwd_ex(
            _ptr(x), xs, _ptr(gb), _ptr(csr.indptr), _ptr(csr.src), _ptr(csr.eid), _ptr(csr.graph_off),
            csr.num_graphs, csr.max_nodes, csr.graph_kind, csr.num_nodes, csr.num_edges, C, H * W, mode,
            _ptr(out), os_, ctypes.byref(ep) if ep is not None else None, _stream(x.device))
    _lib.check(code, "mrp_film_mean_fwd_ex")
    return out


def film_mean_backward(grad_out: torch.Tensor, x: torch.Tensor, gb: Optional[torch.Tensor], csr: GraphCSR,
                       mode: int, need_dx: bool, need_dgb: bool, grad_x_base: Optional[torch.Tensor] = None,
                       epilogue: Optional[EpilogueSpec] = None):
    """(grad_x or None, grad_gb (E, C, 2) or None) for the forward above; ``grad_x_base`` (N, C, H, W),
    if given, is added into grad_x by the kernel.  ``epilogue``: the forward's (its agg_scale and
    self_scale enter here; the gradient of x0 is x0_scale * grad_out, formed by the caller)."""
    _require_device(grad_out, x)
    n, C, H, W = x.shape
    grad_out, gs = _as_node_major(grad_out)
    bs = 0
    if grad_x_base is not None:
        grad_x_base, bs = _as_node_major(grad_x_base)
    dx = torch.empty((n, C, H, W), device=x.device, dtype=torch.float32) if need_dx else None
    dgb = torch.empty((csr.num_edges, C, 2), device=x.device, dtype=torch.float32) if need_dgb else None
    xs = 0
    if need_dgb and (mode & ~_lib.GB_LOGITS) != _lib.MODE_COPY_MEAN:
        x, xs = _as_node_major(x)
    if gb is not None:
        # the kernel reads fp32 (gamma, beta) pairs: the same conversion as the forward
        gb = gb.reshape(csr.num_edges, C, 2)
        if not gb.is_contiguous() or gb.dtype != torch.float32:
            gb = gb.contiguous().float()
    ep = None
    if epilogue is not None and (epilogue.agg_scale != 1.0 or epilogue.self_scale != 0.0):
        ep = _lib.Epilogue(epilogue.agg_scale, epilogue.self_scale, 0, 0, 0.0, 0, 0)
    lib = _lib.load_library()
    ws = None
    if need_dgb:  # scratch for the plane-split k-NN backward (the library never allocates)
        nbytes = int(lib.mrp_film_mean_bwd_workspace(csr.num_graphs, csr.max_nodes, csr.graph_kind, C, H * W))
        if nbytes > 0:
            ws = torch.empty(nbytes // 4 + 1, device=x.device, dtype=torch.float32)
    with torch.cuda.device(x.device):
        code = lib.mrp_film_mean_bwd_ex(
            _ptr(grad_out), gs, _ptr(x), xs, _ptr(gb), _ptr(csr.indptr), _ptr(csr.src), _ptr(csr.eid),
            _ptr(csr.graph_off), csr.num_graphs, csr.max_nodes, csr.graph_kind, csr.num_nodes, csr.num_edges, C,
            H * W, mode,
            _ptr(dx), (C * H * W) if dx is not None else 0, _ptr(grad_x_base), bs, _ptr(dgb),
            ctypes.byref(ep) if ep is not None else None, _ptr(ws), ws.numel() * 4 if ws is not None else 0,
            _stream(x.device))
    _lib.check(code, "mrp_film_mean_bwd_ex")
    return dx, dgb


class FilmMeanFunction(torch.autograd.Function):
    """Autograd wrapper: forward = ``mrp_film_mean_fwd_ex``, backward = ``mrp_film_mean_bwd_ex``.
    ``mode`` may carry ``_lib.GB_LOGITS`` (gb = pre-sigmoid logits; the gradient is then d logits).
    ``scales`` = (agg_scale, self_scale, x0_scale) of the epilogue (``EpilogueSpec``); x0 may be None."""

    @staticmethod
    def forward(ctx, x, gb, x0, csr: GraphCSR, mode: int, scales=(1.0, 0.0, 0.0)):
        out = torch.empty(x.shape, device=x.device, dtype=torch.float32)
        ep = EpilogueSpec(scales[0], scales[1], x0, scales[2])
        film_mean_forward_into(x, gb, csr, mode, out, epilogue=ep)
        ctx.save_for_backward(x, gb)
        ctx.csr = csr
        ctx.mode = mode
        ctx.scales = scales
        ctx.x0_dtype = x0.dtype if x0 is not None else None
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, gb = ctx.saved_tensors
        need_dx = ctx.needs_input_grad[0]
        need_dgb = gb is not None and ctx.needs_input_grad[1]
        ep = EpilogueSpec(ctx.scales[0], ctx.scales[1])
        dx, dgb = film_mean_backward(grad_out, x, gb, ctx.csr, ctx.mode, need_dx, need_dgb, epilogue=ep)
        if dgb is not None:
            dgb = dgb.view(gb.shape).to(gb.dtype)
        dx0 = None
        if ctx.needs_input_grad[2]:
            dx0 = (grad_out * ctx.scales[2]).to(ctx.x0_dtype)
        return dx, dgb, dx0, None, None, None


def _mode_flags(mode, logits: bool) -> int:
    m = _lib.MODES[mode] if isinstance(mode, str) else int(mode)
    if m != _lib.MODE_COPY_MEAN and logits:
        m |= _lib.GB_LOGITS
    return m


def _check_x(x):
    if x.dim() != 4:
        raise ValueError(f"node features must be (N, C, H, W), got {tuple(x.shape)}")
    if x.dtype != torch.float32:
        raise TypeError("node features must be float32 (the reference path is fp32)")
    _require_device(x)


def film_mean(x: torch.Tensor, gb: Optional[torch.Tensor], csr: GraphCSR, mode="film_mean",
              logits: bool = False) -> torch.Tensor:
    """``mean_e(gamma_e * x_src + beta_e)`` per destination node (see module docstring).

    x: (N, C, H, W) fp32 on a ROCm device; gb: (E, 2C) or (E, C, 2) interleaved gamma/beta
    (ignored for ``mode='copy_mean'``), or their pre-sigmoid logits with ``logits=True`` (the
    encoder's Sigmoid then runs inside the kernel); csr: ``RobotGraph.csr(device)``.
    """
    _check_x(x)
    m = _mode_flags(mode, logits)
    if (m & ~_lib.GB_LOGITS) == _lib.MODE_COPY_MEAN:
        gb = None
    return FilmMeanFunction.apply(x, gb, None, csr, m)


def film_mean_residual(x: torch.Tensor, gb: Optional[torch.Tensor], csr: GraphCSR, mode="film_mean",
                       logits: bool = False) -> torch.Tensor:
    """``x + film_mean(x, ...)`` in one pass — the residual combination ``h = g_h + h`` of
    ``dgl/model/dgl_models.py:36-37`` (x[v] is already in registers: no extra traffic)."""
    _check_x(x)
    m = _mode_flags(mode, logits)
    if (m & ~_lib.GB_LOGITS) == _lib.MODE_COPY_MEAN:
        gb = None
    return FilmMeanFunction.apply(x, gb, None, csr, m, (1.0, 1.0, 0.0))


def film_mean_mix(x: torch.Tensor, gb: Optional[torch.Tensor], csr: GraphCSR, x0: torch.Tensor, alpha: float,
                  mode="film_mean", logits: bool = False) -> torch.Tensor:
    """``(1 - alpha) * film_mean(x, ...) + alpha * x0`` in one pass: the initial-feature mix of a
    GCN2-style layer (BASELINE configs[3]'s "GCN2Conv"; not in the reference, parity unpinned)."""
    _check_x(x)
    m = _mode_flags(mode, logits)
    if (m & ~_lib.GB_LOGITS) == _lib.MODE_COPY_MEAN:
        gb = None
    return FilmMeanFunction.apply(x, gb, x0, csr, m, (1.0 - float(alpha), 0.0, float(alpha)))


class FilmMeanCatFunction(torch.autograd.Function):
    """``torch.cat((x, film_mean(x, gb)), 1)`` without the concatenation pass for the aggregate
    (``dgl/model/models.py:181-182,187-188``): the kernel writes the aggregate into the second half of
    the (N, 2C, H, W) buffer and x, whose slices it holds anyway, into the first; backward hands the
    kernel the second half of the incoming gradient as grad_out and the first half as the base of
    x's gradient."""

    @staticmethod
    def forward(ctx, x, gb, csr: GraphCSR, mode: int):
        n, C, H, W = x.shape
        buf = torch.empty((n, 2 * C, H, W), device=x.device, dtype=torch.float32)
        film_mean_cat_forward_into(x, gb, csr, mode, buf)  # the kernel also writes x into buf[:, :C]
        ctx.save_for_backward(x, gb)
        ctx.csr = csr
        ctx.mode = mode
        return buf

    @staticmethod
    def backward(ctx, grad_buf):
        x, gb = ctx.saved_tensors
        C = x.shape[1]
        need_dx = ctx.needs_input_grad[0]
        need_dgb = gb is not None and ctx.needs_input_grad[1]
        dx, dgb = film_mean_backward(grad_buf[:, C:], x, gb, ctx.csr, ctx.mode, need_dx, need_dgb,
                                     grad_x_base=grad_buf[:, :C] if need_dx else None)
        if dgb is not None:
            dgb = dgb.view(gb.shape).to(gb.dtype)
        return dx, dgb, None, None


def film_mean_cat(x: torch.Tensor, gb: Optional[torch.Tensor], csr: GraphCSR, mode="film_mean",
                  logits: bool = False) -> torch.Tensor:
    """``torch.cat((x, film_mean(x, gb, csr, mode, logits)), dim=1)`` in one kernel pass."""
    if x.dim() != 4 or x.dtype != torch.float32:
        raise ValueError("node features must be (N, C, H, W) float32")
    _require_device(x)
    m = _mode_flags(mode, logits)
    if (m & ~_lib.GB_LOGITS) == _lib.MODE_COPY_MEAN:
        gb = None
    return FilmMeanCatFunction.apply(x, gb, csr, m)
