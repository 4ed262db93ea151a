"""Edge encoder on the GPU (``dgl/model/models.py:146-154``), restructured for the hot path.

``z = W2 relu(W1 pose + b1) + b2``, ``gamma/beta = sigmoid(z)``; the sigmoid is not run here: the
aggregation kernels take the logits (``MRP_AGG_GB_LOGITS``) and apply it while building their tiles.

Both Linears run on the bf16 matrix cores at fp32 accuracy (every fp32 operand split exactly into
three bf16 parts, six partial products; ``csrc/encoder_split.hip``), the weights split and laid out
once per weight version (:func:`packed_weights`):

* inference (no gradient wanted): ONE kernel, ``mrp_edge_encoder_fwd_split`` — h never written;
* training (:class:`EdgeEncoderSplitFunction`, E % 32 == 0 and C % 32 == 0 — every reference
  configuration): the same kernel also writes h^T for the backward; the backward's two GEMMs
  (``dh^T = W2^T dz^T``, ``dW2 = dz^T h`` with db2) run on the split-bf16 weight-gradient kernel of
  ``compress_split.hip`` on two streams, the ReLU mask, dW1 and db1 in one HIP pass.

Other shapes train through :class:`EdgeEncoderFunction`: ``mrp_edge_hidden_fwd`` (K = 9, a streaming
write) + ``mrp_edge_logits_fwd`` (fp32 MFMA, 64 x 64 tiles, bias in the epilogue; C % 32 != 0 or
``set_logits_path("library")``: ``torch.addmm``), the backward GEMMs on torch (two streams) and the
small reductions in one HIP pass (``mrp_edge_encoder_bwd``).
"""
from __future__ import annotations

import collections
import ctypes
import weakref

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


_LOGITS_PATH = "split"


def set_logits_path(path: str) -> None:
    """"split" (default): ``mrp_edge_encoder_fwd_split`` (split-bf16 matrix cores) when no gradient is
    wanted and the split training path otherwise; "hip": ``mrp_edge_hidden_fwd`` +
    ``mrp_edge_logits_fwd`` (fp32 MFMA); "library": the hidden kernel + ``torch.addmm`` (comparison runs)."""
    global _LOGITS_PATH
    if path not in ("split", "hip", "library"):
        raise ValueError(f"unknown logits path {path!r}")
    _LOGITS_PATH = path


# packed split-bf16 weight images, per second-Linear module: (key, tensor).  The key holds the data
# pointers and autograd versions of W1, b1, W2: an optimizer step (an in-place update under no_grad)
# bumps a version and the image is rebuilt on the next call.  Writes through ``.data`` bypass the
# version counter: call :func:`clear_packed_weights` after those.  Kept outside the modules (not
# pickled, not deep-copied).
_packed = weakref.WeakKeyDictionary()


def clear_packed_weights() -> None:
    _packed.clear()
    _w2t_cache.clear()
    _w2t_img_cache.clear()


def packed_weights(l1: torch.nn.Linear, l2: torch.nn.Linear) -> torch.Tensor:
    """The ``mrp_edge_encoder_pack`` image of (W1, b1, W2), rebuilt when a weight changed."""
    w1, b1, w2 = l1.weight, l1.bias, l2.weight
    key = tuple((t.data_ptr(), t._version, t.device.index) for t in (w1, b1, w2))
    hit = _packed.get(l2)
    if hit is not None and hit[0] == key:
        return hit[1]
    C = w1.shape[0]
    lib = _lib.load_library()
    nbytes = int(lib.mrp_edge_encoder_pack_bytes(C))
    img = torch.empty((nbytes + 3) // 4, device=w1.device, dtype=torch.float32)
    w1c, b1c, w2c = (t.detach().contiguous().float() for t in (w1, b1, w2))
    with torch.cuda.device(w1.device):
        _lib.check(lib.mrp_edge_encoder_pack(_ptr(w1c), _ptr(b1c), _ptr(w2c), C, _ptr(img),
                                             ctypes.c_void_p(torch.cuda.current_stream(w1.device).cuda_stream)),
                   "mrp_edge_encoder_pack")
    _packed[l2] = (key, img)
    return img


def encoder_forward_split(pose, l1: torch.nn.Linear, l2: torch.nn.Linear):
    """z = relu(pose W1^T + b1) W2^T + b2, (E, 2C), in one launch on the split-bf16 matrix cores
    (``mrp_edge_encoder_fwd_split``); None when the kernel declines the shape (C % 32 != 0)."""
    C = l1.weight.shape[0]
    if not pose.is_cuda:
        raise RuntimeError("mrp_gnn: the edge encoder kernel runs only on the GPU; no CPU fallback")
    if C % 32 != 0 or tuple(l1.weight.shape) != (C, 9) or tuple(l2.weight.shape) != (2 * C, C) \
            or l1.bias is None or not image_supported(C):
        return None
    img = packed_weights(l1, l2)
    pose = pose.detach().contiguous().float()
    b2 = l2.bias.detach().contiguous().float() if l2.bias is not None else None
    E = pose.shape[0]
    z = torch.empty((E, 2 * C), device=pose.device, dtype=torch.float32)
    lib = _lib.load_library()
    with torch.cuda.device(pose.device):
        code = lib.mrp_edge_encoder_fwd_split(_ptr(pose), _ptr(img), _ptr(b2) if b2 is not None else None, E, C,
                                              _ptr(z), ctypes.c_void_p(torch.cuda.current_stream(pose.device).cuda_stream))
    if code == _lib.HIP_ERROR_NOT_SUPPORTED:
        return None
    _lib.check(code, "mrp_edge_encoder_fwd_split")
    return z


def logits_forward(h, w2, b2) -> torch.Tensor:
    """z = h @ w2.T + b2, (E, 2C)."""
    E, C = h.shape
    if tuple(w2.shape) != (2 * C, C) or tuple(b2.shape) != (2 * C,):
        raise ValueError("edge logits shapes must be h (E,C), w2 (2C,C), b2 (2C,)")
    if not h.is_cuda:
        raise RuntimeError("mrp_gnn: the edge logits kernel runs only on the GPU; no CPU fallback")
    h, w2, b2 = (t.contiguous().float() for t in (h, w2, b2))
    if _LOGITS_PATH == "library" or C % 32 != 0:
        return torch.addmm(b2, h, w2.t())
    z = torch.empty((E, 2 * C), device=h.device, dtype=torch.float32)
    lib = _lib.load_library()
    with torch.cuda.device(h.device):
        code = lib.mrp_edge_logits_fwd(_ptr(h), E, C, _ptr(w2), _ptr(b2), _ptr(z),
                                       ctypes.c_void_p(torch.cuda.current_stream(h.device).cuda_stream))
    _lib.check(code, "mrp_edge_logits_fwd")
    return z


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


_side_streams = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    s = _side_streams.get(dev)
    if s is None:
        s = _side_streams[dev] = torch.cuda.Stream(device=dev)
    return s


def _grad_out(param, shape, dev):
    """The gradient buffer of ``param``: its slot in a gradient all-reducer's bucket when one holds
    it (``dist.grad_out_like``: written in place, adopted by autograd without a copy), else new."""
    from .dist import grad_out_like
    g = grad_out_like(param) if param is not None else None
    return g if g is not None else torch.empty(shape, device=dev)


def encoder_backward_reductions(dz, dh, h, pose, b2=None, w1=None, b1=None):
    """(db2 (2C,), dw1 (C, 9), db1 (C,)) via ``mrp_edge_encoder_bwd`` (see module docstring)."""
    E, C = h.shape
    dev = h.device
    db2 = _grad_out(b2, (2 * C,), dev)
    dw1 = _grad_out(w1, (C, 9), dev)
    db1 = _grad_out(b1, (C,), dev)
    lib = _lib.load_library()
    ws = torch.empty(max(int(lib.mrp_edge_encoder_bwd_workspace(E, C)) // 4, 1), device=dev)
    with torch.cuda.device(dev):
        code = lib.mrp_edge_encoder_bwd(_ptr(dz), _ptr(dh), _ptr(h), _ptr(pose), E, C, _ptr(db2), _ptr(dw1),
                                        _ptr(db1), _ptr(ws), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    _lib.check(code, "mrp_edge_encoder_bwd")
    return db2, dw1, db1


class EdgeEncoderFunction(torch.autograd.Function):
    """z = relu(pose W1^T + b1) W2^T + b2 (``models.py:146-149`` without the Sigmoid)."""

    @staticmethod
    def forward(ctx, pose, w1, b1, w2, b2):
        pose = pose.contiguous().float()
        h = hidden_forward(pose, w1, b1)
        z = logits_forward(h, w2, b2)
        ctx.save_for_backward(pose, w1, w2, h, b1, b2)
        return z

    @staticmethod
    def backward(ctx, dz):
        pose, w1, w2, h, b1, b2 = ctx.saved_tensors
        dz = dz.contiguous()
        need = ctx.needs_input_grad
        cur = torch.cuda.current_stream(dz.device)
        dw2 = None
        if need[3]:
            dw2 = _grad_out(w2, tuple(w2.shape), dz.device)
            side = _side_stream(dz.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):  # dW2 = dz^T h beside dh = dz W2
                torch.mm(dz.t(), h, out=dw2)
            dz.record_stream(side)
            h.record_stream(side)
        dh = dz.mm(w2) if (need[0] or need[1] or need[2]) else None
        if dw2 is not None:
            cur.wait_stream(_side_stream(dz.device))
            dw2.record_stream(cur)
        db2 = dw1 = db1 = None
        if dh is not None or need[4]:
            db2, dw1, db1 = encoder_backward_reductions(dz, dh if dh is not None else dz[:, : h.shape[1]], h, pose,
                                                        b2 if need[4] else None, w1 if need[1] else None,
                                                        b1 if need[2] else None)
        dpose = (dh * (h > 0)).mm(w1) if need[0] else None
        return (dpose, dw1 if need[1] else None, db1 if need[2] else None, dw2,
                db2 if need[4] else None)


#: calls per encoder path ("split": mrp_edge_encoder_fwd_split,
#: "split_train": EdgeEncoderSplitFunction, "autograd": EdgeEncoderFunction) — lets tests assert which
#: kernels a forward actually ran
PATH_COUNTS = collections.Counter()


_w2t_cache = weakref.WeakKeyDictionary()
_w2t_img_cache = weakref.WeakKeyDictionary()

#: the single-stream fused encoder backward (``mrp_edge_encoder_bwd_fused``) when every parameter
#: gradient and no pose gradient is wanted; False: the two-stream form (A/B comparisons)
_BWD_FUSED = True


def set_fused_backward(on: bool) -> None:
    global _BWD_FUSED
    _BWD_FUSED = bool(on)


def transposed_w2(l2: torch.nn.Linear) -> torch.Tensor:
    """W2^T (C, 2C) row-major — the dh^T GEMM's row operand — cached per weight version like the
    packed images (cleared by :func:`clear_packed_weights`)."""
    w2 = l2.weight
    key = (w2.data_ptr(), w2._version, w2.device.index)
    hit = _w2t_cache.get(l2)
    if hit is not None and hit[0] == key:
        return hit[1]
    t = w2.detach().float().t().contiguous()
    _w2t_cache[l2] = (key, t)
    return t


def packed_w2t(l2: torch.nn.Linear) -> torch.Tensor:
    """W2^T's packed split-bf16 image (``mrp_compress_split_pack(w2, C, 1, C, 2C)``) — the dh^T product's
    row operand in ``mrp_edge_encoder_bwd_fused`` — cached per weight version like :func:`transposed_w2`."""
    w2 = l2.weight
    key = (w2.data_ptr(), w2._version, w2.device.index)
    hit = _w2t_img_cache.get(l2)
    if hit is not None and hit[0] == key:
        return hit[1]
    C = w2.shape[1]
    lib = _lib.load_library()
    nbytes = int(lib.mrp_compress_split_pack_bytes(C, 2 * C))
    img = torch.empty((nbytes + 3) // 4, device=w2.device, dtype=torch.float32)
    w2c = w2.detach().contiguous().float()
    with torch.cuda.device(w2.device):
        _lib.check(lib.mrp_compress_split_pack(_ptr(w2c), C, 1, C, 2 * C, _ptr(img),
                                               ctypes.c_void_p(torch.cuda.current_stream(w2.device).cuda_stream)),
                   "mrp_compress_split_pack")
    _w2t_img_cache[l2] = (key, img)
    return img


def image_supported(C: int) -> bool:
    """The packed split-bf16 weight image exists for C: C % 32 == 0 and the image under 2^31 bytes
    (``mrp_edge_encoder_pack`` declines C > 13344)."""
    return C > 0 and C % 32 == 0 and 0 < int(_lib.load_library().mrp_edge_encoder_pack_bytes(C)) < (1 << 31)


def split_train_supported(E: int, C: int) -> bool:
    """The split-bf16 training path's shapes: C % 32 == 0 and E % 32 == 0 (its backward GEMMs walk
    the edges in 32-edge stages), the weight image under 2^31 bytes and every operand (z, dz^T, h^T:
    E x 2C floats at most) addressable with 32-bit offsets; the reference configurations all qualify
    (E = B N (N - 1) or B N k).  Other shapes train through :class:`EdgeEncoderFunction`."""
    return (E > 0 and C > 0 and C % 32 == 0 and E % 32 == 0 and E * 2 * C * 4 < (1 << 31)
            and image_supported(C))


class EdgeEncoderSplitFunction(torch.autograd.Function):
    """z = relu(pose W1^T + b1) W2^T + b2 (``models.py:146-149`` without the Sigmoid) on the split-bf16
    matrix cores, forward and backward (``include/mrp_gnn.h``, the encoder's training path):

    * forward: ``mrp_edge_encoder_fwd_split_train`` — the inference kernel, which also writes h^T;
    * backward: on a side stream ``mrp_edge_encoder_bwd_prep`` (dz^T) and ``mrp_edge_encoder_bwd_split``
      for dW2 = dz^T h (db2 = the row sums of dz^T on the same pass); beside it ``_bwd_split`` for
      dh^T = W2^T dz^T and ``mrp_edge_encoder_bwd_t`` (the ReLU mask, dW1, db1).  Gradients are written straight into a
      gradient all-reducer's buckets when one holds the parameters (``dist.grad_out_like``)."""

    @staticmethod
    def forward(ctx, pose, w1, b1, w2, b2, img, l2):
        E, C = pose.shape[0], w1.shape[0]
        pose = pose.detach().contiguous().float()
        b2c = b2.detach().contiguous().float() if b2 is not None else None
        z = torch.empty((E, 2 * C), device=pose.device, dtype=torch.float32)
        hT = torch.empty((C, E), device=pose.device, dtype=torch.float32)
        lib = _lib.load_library()
        with torch.cuda.device(pose.device):
            _lib.check(lib.mrp_edge_encoder_fwd_split_train(
                _ptr(pose), _ptr(img), _ptr(b2c) if b2c is not None else None, E, C, _ptr(z), _ptr(hT), E,
                ctypes.c_void_p(torch.cuda.current_stream(pose.device).cuda_stream)), "mrp_edge_encoder_fwd_split_train")
        ctx.save_for_backward(pose, w1, b1, w2, b2, hT)
        # W2^T (and its packed image) are built in backward, only for the products that run:
        # a forward whose backward never runs, or runs without dh^T, packs nothing
        ctx.l2 = l2
        return z

    @staticmethod
    def backward(ctx, dz):
        pose, w1, b1, w2, b2, hT = ctx.saved_tensors
        need = ctx.needs_input_grad
        dz = dz.contiguous().float()
        E, C = pose.shape[0], w1.shape[0]
        dev = dz.device
        cur = torch.cuda.current_stream(dev)
        lib = _lib.load_library()
        nbytes = int(lib.mrp_edge_encoder_bwd_split_workspace(E, C))

        def workspace():
            return torch.empty((nbytes + 3) // 4, device=dev) if nbytes > 0 else None

        if not need[0] and need[1] and need[2] and need[3] and need[4] and _BWD_FUSED:
            # every parameter gradient, no pose gradient (the reference's case: poses are data): the
            # three-launch single-stream form, dh^T never materialised
            dw1, db1 = _grad_out(w1, (C, 9), dev), _grad_out(b1, (C,), dev)
            dw2, db2 = _grad_out(w2, (2 * C, C), dev), _grad_out(b2, (2 * C,), dev)
            wsf = torch.empty((int(lib.mrp_edge_encoder_bwd_fused_workspace(E, C)) + 3) // 4, device=dev)
            with torch.cuda.device(dev):
                w2t, w2t_img = transposed_w2(ctx.l2), packed_w2t(ctx.l2)
                _lib.check(lib.mrp_edge_encoder_bwd_fused(
                    _ptr(dz), _ptr(w2t), _ptr(w2t_img) if w2t_img is not None else None, _ptr(hT), _ptr(pose), E, C,
                    _ptr(dw1), _ptr(db1), _ptr(dw2), _ptr(db2),
                    _ptr(wsf), wsf.numel() * 4, ctypes.c_void_p(cur.cuda_stream)), "mrp_edge_encoder_bwd_fused")
            return None, dw1, db1, dw2, db2, None, None
        dw2 = db2 = side = None
        with torch.cuda.device(dev):
            if need[3] or need[4]:  # dz^T, then dW2 = dz^T h with db2 as its row sums, on the side stream
                dw2 = _grad_out(w2, (2 * C, C), dev) if need[3] else torch.empty((2 * C, C), device=dev)
                db2 = _grad_out(b2, (2 * C,), dev) if need[4] else None
                dzT = torch.empty((2 * C, E), device=dev)
                wsa = workspace()
                side = _side_stream(dev)
                side.wait_stream(cur)
                ss = ctypes.c_void_p(side.cuda_stream)
                _lib.check(lib.mrp_edge_encoder_bwd_prep(_ptr(dz), E, C, _ptr(dzT), E, ss), "mrp_edge_encoder_bwd_prep")
                _lib.check(lib.mrp_edge_encoder_bwd_split(
                    None, _ptr(dzT), None, _ptr(hT), E, C, None, _ptr(dw2), _ptr(db2) if db2 is not None else None,
                    _ptr(wsa) if wsa is not None else None, nbytes, ss), "mrp_edge_encoder_bwd_split")
                for t in (dz, hT, dzT, wsa, dw2, db2):
                    if t is not None:
                        t.record_stream(side)
            dw1 = db1 = dhT = None
            if need[0] or need[1] or need[2]:  # dh^T = W2^T dz^T, then the ReLU mask, dW1, db1
                w2t = transposed_w2(ctx.l2)
                st = ctypes.c_void_p(cur.cuda_stream)
                dhT = torch.empty((C, E), device=dev)
                wsb = workspace()
                _lib.check(lib.mrp_edge_encoder_bwd_split(
                    _ptr(dz), None, _ptr(w2t), None, E, C, _ptr(dhT), None, None,
                    _ptr(wsb) if wsb is not None else None, nbytes, st), "mrp_edge_encoder_bwd_split")
                if need[1] or need[2]:
                    dw1 = _grad_out(w1, (C, 9), dev) if need[1] else None
                    db1 = _grad_out(b1, (C,), dev) if need[2] else None
                    wst = torch.empty(max(int(lib.mrp_edge_encoder_bwd_t_workspace(E, C)) // 4, 1), device=dev)
                    _lib.check(lib.mrp_edge_encoder_bwd_t(
                        _ptr(dhT), E, _ptr(hT), E, _ptr(pose), E, C, _ptr(dw1) if dw1 is not None else None,
                        _ptr(db1) if db1 is not None else None, _ptr(wst), wst.numel() * 4, st), "mrp_edge_encoder_bwd_t")
            if side is not None:
                cur.wait_stream(side)
        dpose = (dhT * (hT > 0)).t().mm(w1.float()) if need[0] else None
        return dpose, dw1, db1, dw2 if need[3] else None, db2, None, None


def edge_logits(enc_layers: torch.nn.Sequential, pose: torch.Tensor) -> torch.Tensor:
    """Pre-sigmoid FiLM logits z (E, 2C) from the reference-layout ``nn.Sequential``
    (layers 0 and 2 are the Linears)."""
    l1, l2 = enc_layers[0], enc_layers[2]
    if not pose.is_cuda:
        raise RuntimeError("mrp_gnn: the edge encoder kernels run only on the GPU; no CPU fallback")
    params = (pose, l1.weight, l1.bias, l2.weight, l2.bias)
    inference = not (torch.is_grad_enabled() and any(t.requires_grad for t in params))
    if _LOGITS_PATH == "split" and inference:
        z = encoder_forward_split(pose, l1, l2)
        if z is not None:
            PATH_COUNTS["split"] += 1
            return z
    C = l1.weight.shape[0]
    if _LOGITS_PATH == "split" and split_train_supported(pose.shape[0], C) and l1.bias is not None \
            and tuple(l1.weight.shape) == (C, 9) and tuple(l2.weight.shape) == (2 * C, C):
        PATH_COUNTS["split_train"] += 1
        return EdgeEncoderSplitFunction.apply(pose, l1.weight, l1.bias, l2.weight, l2.bias,
                                              packed_weights(l1, l2), l2)
    PATH_COUNTS["autograd"] += 1
    return EdgeEncoderFunction.apply(*params)
