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
  ``compress_split.hip`` (one launch of both, or two streams), the ReLU mask, dW1 and db1 in one HIP
  pass, the pose gradient (when poses require grad) on ``mrp_edge_encoder_bwd_pose``;
* any other E or C (:class:`EdgeEncoderPaddedFunction`, and inference with C % 32 != 0): the same
  kernels on operands zero-padded to multiples of 32 (:func:`padded_weights`) — every padded term a
  product with an exact zero, so z and the gradients are the leading blocks of the padded results.

:class:`EdgeEncoderFunction` (``mrp_edge_hidden_fwd`` + ``mrp_edge_logits_fwd`` in fp32, the backward
GEMMs on torch) serves only the comparison paths (``set_logits_path("hip" | "library")``) and shapes
past the split kernels' 32-bit offsets (E x 2C >= 2^29 floats after padding).
"""
from __future__ import annotations

import collections
import ctypes
import os
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
    _padded.clear()
    _ready.clear()


def _pack(w1, b1, w2) -> torch.Tensor:
    C = w1.shape[0]
    lib = _lib.load_library()
    nbytes = int(lib.mrp_edge_encoder_pack_bytes(C))
    img = torch.empty((nbytes + 3) // 4, device=w1.device, dtype=torch.float32)
    w1c, b1c, w2c = (t.detach().contiguous().float() for t in (w1, b1, w2))
    with torch.cuda.device(w1.device):
        _lib.check(lib.mrp_edge_encoder_pack(_ptr(w1c), _ptr(b1c), _ptr(w2c), C, _ptr(img),
                                             ctypes.c_void_p(torch.cuda.current_stream(w1.device).cuda_stream)),
                   "mrp_edge_encoder_pack")
    return img


def packed_weights(l1: torch.nn.Linear, l2: torch.nn.Linear) -> torch.Tensor:
    """The ``mrp_edge_encoder_pack`` image of (W1, b1, W2), rebuilt when a weight changed."""
    w1, b1, w2 = l1.weight, l1.bias, l2.weight
    key = tuple((t.data_ptr(), t._version, t.device.index) for t in (w1, b1, w2))
    hit = _packed.get(l2)
    if hit is not None and hit[0] == key:
        return hit[1]
    img = _pack(w1, b1, w2)
    _packed[l2] = (key, img)
    _track_image(img)
    return img


# The inference encoder on its own stream (one per device), ordered after the producers of what it
# reads rather than after everything queued before it: its inputs — the poses, b2 and the packed
# weight image — each carry the event recorded on the caller's stream when this module first saw them
# in their current state (tensor object and autograd version; the image: when it was packed), and the
# caller's stream waits for the encoder before the aggregation that reads its logits.  So the encoder
# of a batch whose inputs are ready runs beside the aggregation of the previous batch (an HBM-bound
# kernel) instead of after it.  Every write to those inputs that bumps the version counter is ordered
# (a new event); writes that bypass it (``.data``, foreign kernels) need ``clear_packed_weights()``, as
# for the packed images.  Not under stream capture (one stream there).  set_encoder_stream(False):
# the caller's stream.
_ENC_STREAM = os.environ.get("MRP_ENCODER_STREAM", "1") != "0"
# below this many E x C products the encoder is a few microseconds of GPU work and the stream's
# bookkeeping (its waits and the join, ~10 us of host time) would cost more than the overlap saves
_ENC_STREAM_MIN_WORK = 1 << 18
_enc_streams = {}
_waited = {}       # device index -> ids of readiness events the encoder stream already waits behind
_recorded = {}     # device index -> {id(tensor): weakref} already recorded on the encoder stream
_ready = {}        # id(tensor) -> (weakref, version, event)
_image_ready = {}  # id(packed image) -> (weakref, event recorded after its pack kernel)


def set_encoder_stream(on: bool) -> None:
    global _ENC_STREAM
    _ENC_STREAM = bool(on)


def _record(dev: torch.device) -> torch.cuda.Event:
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    return ev


def _track_image(img: torch.Tensor) -> None:
    """The event after a packed image's pack kernel (dropped with the image)."""
    iid = id(img)
    _image_ready[iid] = (weakref.ref(img, lambda _r, iid=iid: _image_ready.pop(iid, None)), _record(img.device))


def _ready_event(t: torch.Tensor) -> torch.cuda.Event:
    """The event after which ``t`` (in its current version) is complete on the caller's stream."""
    hit = _ready.get(id(t))
    if hit is not None and hit[0]() is t and hit[1] == t._version:
        return hit[2]
    ev = _record(t.device)
    tid = id(t)
    _ready[tid] = (weakref.ref(t, lambda _r, tid=tid: _ready.pop(tid, None)), t._version, ev)
    return ev


_ENC_PRIORITY = -1  # the highest the runtime offers (torch: lower is higher); 0 = normal
# the caller's stream joins the encoder's through a device-scope event (mrp_stream_join) instead of
# torch's wait_stream, whose event carries a system-scope release (False: torch's, lab A/B)
_FAST_JOIN = True


def set_fast_join(on: bool) -> None:
    global _FAST_JOIN
    _FAST_JOIN = bool(on)


def set_encoder_stream_priority(priority: int) -> None:
    """Priority of the encoder stream (lab A/B): at normal priority its workgroups queue behind the
    aggregation's thousands and it finishes late; high priority lets it through first."""
    global _ENC_PRIORITY
    _ENC_PRIORITY = int(priority)
    _enc_streams.clear()


def _enc_stream(dev: torch.device) -> torch.cuda.Stream:
    s = _enc_streams.get(dev.index)
    if s is None:
        lo, hi = torch.cuda.Stream.priority_range()  # (lowest, highest), e.g. (0, -1)
        prio = max(min(_ENC_PRIORITY, lo), hi)
        s = _enc_streams[dev.index] = torch.cuda.Stream(device=dev, priority=prio)
    return s


def encoder_forward_split(pose, l1: torch.nn.Linear, l2: torch.nn.Linear):
    """z = relu(pose W1^T + b1) W2^T + b2, (E, 2C), in one launch on the split-bf16 matrix cores
    (``mrp_edge_encoder_fwd_split``), on the encoder stream (see above); C % 32 != 0 runs on the
    zero-padded weights (:func:`padded_weights`) and keeps z's 2C leading columns.  None when no
    weight image exists for the shape (C beyond ``mrp_edge_encoder_pack``'s bound, layers not the
    reference's)."""
    C = l1.weight.shape[0]
    if not pose.is_cuda:
        raise RuntimeError("mrp_gnn: the edge encoder kernel runs only on the GPU; no CPU fallback")
    if tuple(l1.weight.shape) != (C, 9) or tuple(l2.weight.shape) != (2 * C, C) or l1.bias is None or C == 0:
        return None
    # readiness is tracked on the tensors the caller holds (detach() makes a new tensor object per call,
    # sharing the version counter)
    if C % 32 == 0 and image_supported(C):
        img = packed_weights(l1, l2)
        b2 = l2.bias.detach().contiguous().float() if l2.bias is not None else None
        b2_src = l2.bias
        Cp = C
    elif image_supported(_pad32(C)):
        rec = padded_weights(l1, l2)
        img, b2, Cp = rec.img, rec.b2, rec.Cp
        b2_src = b2
    else:
        return None
    pose_src = pose
    pose = pose.detach().contiguous().float()
    E = pose.shape[0]
    dev = pose.device
    cur = torch.cuda.current_stream(dev)
    side = _enc_begin(dev, E * C, ((pose_src, pose), (b2_src, b2)), img)
    run = side if side is not None else cur
    lib = _lib.load_library()
    with torch.cuda.device(dev), torch.cuda.stream(run):
        z = torch.empty((E, 2 * Cp), device=dev, dtype=torch.float32)
        code = lib.mrp_edge_encoder_fwd_split(_ptr(pose), _ptr(img), _ptr(b2) if b2 is not None else None, E, Cp,
                                              _ptr(z), ctypes.c_void_p(run.cuda_stream))
        if code == _lib.HIP_ERROR_NOT_SUPPORTED:
            return None
        _lib.check(code, "mrp_edge_encoder_fwd_split")
        if Cp != C:
            z = z[:, : 2 * C].contiguous()
    _enc_end(dev, side, (z,), ((pose_src, pose), (None, img), (None, b2)))
    return z


def _enc_begin(dev: torch.device, work: int, reads, img):
    """The stream the encoder runs on: its own, after the readiness events of ``reads`` ((caller's
    tensor, tensor the kernel reads) pairs) and of the packed image; or None for the caller's stream
    (small encoders, stream capture, set_encoder_stream(False))."""
    if not _ENC_STREAM or work < _ENC_STREAM_MIN_WORK or torch.cuda.is_current_stream_capturing():
        return None
    side = _enc_stream(dev)
    waited = _waited.setdefault(dev.index, {})

    def wait(ev):
        # the encoder stream's waits are in its own order: one it already passed need not be repeated
        if waited.get(id(ev)) is not ev:
            side.wait_event(ev)
            waited[id(ev)] = ev
            if len(waited) > 64:
                waited.clear()
                waited[id(ev)] = ev

    for src, t in reads:
        if t is None:
            continue
        # a converted copy (non-contiguous or non-fp32 input) was made just now on the caller's stream
        same = src is not None and t.data_ptr() == src.data_ptr() and t.dtype == src.dtype
        wait(_ready_event(src) if same else _record(dev))
    hit = _image_ready.get(id(img))
    if hit is not None and hit[0]() is img:
        wait(hit[1])
    else:  # an image packed before this module tracked it: after everything queued so far
        side.wait_stream(torch.cuda.current_stream(dev))
    return side


def _enc_end(dev: torch.device, side, outs, reads) -> None:
    """The caller's stream (and whatever it runs next: the aggregation, an optimizer step writing the
    weights) joins the encoder stream; the encoder's outputs and inputs are not recycled by the caching
    allocator before both streams are past them."""
    if side is None:
        return
    cur = torch.cuda.current_stream(dev)
    if _FAST_JOIN:
        _lib.check(_lib.load_library().mrp_stream_join(ctypes.c_void_p(cur.cuda_stream),
                                                       ctypes.c_void_p(side.cuda_stream)), "mrp_stream_join")
    else:
        cur.wait_stream(side)
    for t in outs:
        t.record_stream(cur)
    rec = _recorded.setdefault(dev.index, {})
    for src, t in reads:
        if t is None:
            continue
        if src is not None and src.data_ptr() == t.data_ptr():
            t = src
        hit = rec.get(id(t))
        if hit is None or hit() is not t:  # the block keeps its recorded streams for its lifetime
            t.record_stream(side)
            tid = id(t)
            rec[tid] = weakref.ref(t, lambda _r, tid=tid, rec=rec: rec.pop(tid, None))


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
#: "split_train": EdgeEncoderSplitFunction, "split_padded": EdgeEncoderPaddedFunction,
#: "autograd": EdgeEncoderFunction) — lets tests assert which
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


def _pack_w2t(w2: torch.Tensor) -> torch.Tensor:
    C = w2.shape[1]
    lib = _lib.load_library()
    nbytes = int(lib.mrp_compress_split_pack_bytes(C, 2 * C))
    img = torch.empty((nbytes + 3) // 4, device=w2.device, dtype=torch.float32)
    w2c = w2.detach().contiguous().float()
    with torch.cuda.device(w2.device):
        _lib.check(lib.mrp_compress_split_pack(_ptr(w2c), C, 1, C, 2 * C, _ptr(img),
                                               ctypes.c_void_p(torch.cuda.current_stream(w2.device).cuda_stream)),
                   "mrp_compress_split_pack")
    return img


def packed_w2t(l2: torch.nn.Linear) -> torch.Tensor:
    """W2^T's packed split-bf16 image (``mrp_compress_split_pack(w2, C, 1, C, 2C)``) — the dh^T product's
    row operand in ``mrp_edge_encoder_bwd_fused`` — cached per weight version like :func:`transposed_w2`."""
    w2 = l2.weight
    key = (w2.data_ptr(), w2._version, w2.device.index)
    hit = _w2t_img_cache.get(l2)
    if hit is not None and hit[0] == key:
        return hit[1]
    img = _pack_w2t(w2)
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
        # on the caller's stream: beside the previous step's backward (2 workgroups per CU at 245
        # registers) the encoder's workgroups slowed the layer's training step 0.54 -> 0.60 ms (round 6)
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
        params = (None, w1, b1, w2, b2)
        dev = dz.device

        def out(i, shape):
            return _grad_out(params[i], shape, dev)
        return split_backward(dz.contiguous().float(), pose, hT, w1, ctx.needs_input_grad, out,
                              lambda: transposed_w2(ctx.l2), lambda: packed_w2t(ctx.l2)) + (None, None)


def pose_grad(dhT: torch.Tensor, hT: torch.Tensor, w1: torch.Tensor) -> torch.Tensor:
    """dpose (E, 9) = (dh^T (.) [h^T > 0])^T W1 on ``mrp_edge_encoder_bwd_pose`` (h^T, dh^T: (C, E))."""
    C, E = hT.shape
    dev = hT.device
    dpose = torch.empty((E, 9), device=dev)
    lib = _lib.load_library()
    nbytes = int(lib.mrp_edge_encoder_bwd_pose_workspace(E, C))
    ws = torch.empty((nbytes + 3) // 4, device=dev) if nbytes > 0 else None
    w1c = w1.detach().contiguous().float()
    with torch.cuda.device(dev):
        _lib.check(lib.mrp_edge_encoder_bwd_pose(
            _ptr(dhT), dhT.stride(0), _ptr(hT), hT.stride(0), _ptr(w1c), E, C, _ptr(dpose),
            _ptr(ws) if ws is not None else None, nbytes, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
            "mrp_edge_encoder_bwd_pose")
    return dpose


def split_backward(dz, pose, hT, w1, need, out, w2t_get, w2t_img_get):
    """The split-bf16 backward of ``z = relu(pose W1^T + b1) W2^T + b2`` (E % 32 == 0, C % 32 == 0):
    ``need`` = needs_input_grad of (pose, w1, b1, w2, b2); ``out(i, shape)`` the buffer of parameter
    gradient i (1..4); ``w2t_get`` / ``w2t_img_get`` build W2^T and its packed image on demand.
    Returns (dpose, dw1, db1, dw2, db2)."""
    E, C = pose.shape[0], hT.shape[0]
    dev = dz.device
    cur = torch.cuda.current_stream(dev)
    lib = _lib.load_library()
    nbytes = int(lib.mrp_edge_encoder_bwd_split_workspace(E, C))

    def workspace():
        return torch.empty((nbytes + 3) // 4, device=dev) if nbytes > 0 else None

    if not need[0] and need[1] and need[2] and need[3] and need[4] and _BWD_FUSED:
        # every parameter gradient, no pose gradient (the reference's case: poses are data): the
        # three-launch single-stream form, dh^T never materialised
        dw1, db1 = out(1, (C, 9)), out(2, (C,))
        dw2, db2 = out(3, (2 * C, C)), out(4, (2 * C,))
        wsf = torch.empty((int(lib.mrp_edge_encoder_bwd_fused_workspace(E, C)) + 3) // 4, device=dev)
        with torch.cuda.device(dev):
            w2t, w2t_img = w2t_get(), w2t_img_get()
            _lib.check(lib.mrp_edge_encoder_bwd_fused(
                _ptr(dz), _ptr(w2t), _ptr(w2t_img) if w2t_img is not None else None, _ptr(hT), _ptr(pose), E, C,
                _ptr(dw1), _ptr(db1), _ptr(dw2), _ptr(db2),
                _ptr(wsf), wsf.numel() * 4, ctypes.c_void_p(cur.cuda_stream)), "mrp_edge_encoder_bwd_fused")
        return None, dw1, db1, dw2, db2
    dw2 = db2 = side = None
    with torch.cuda.device(dev):
        if need[3] or need[4]:  # dz^T, then dW2 = dz^T h with db2 as its row sums, on the side stream
            dw2 = out(3, (2 * C, C)) if need[3] else torch.empty((2 * C, C), device=dev)
            db2 = out(4, (2 * C,)) if need[4] else None
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
            w2t = w2t_get()
            st = ctypes.c_void_p(cur.cuda_stream)
            dhT = torch.empty((C, E), device=dev)
            wsb = workspace()
            _lib.check(lib.mrp_edge_encoder_bwd_split(
                _ptr(dz), None, _ptr(w2t), None, E, C, _ptr(dhT), None, None,
                _ptr(wsb) if wsb is not None else None, nbytes, st), "mrp_edge_encoder_bwd_split")
            if need[1] or need[2]:
                dw1 = out(1, (C, 9)) if need[1] else None
                db1 = out(2, (C,)) if need[2] else None
                wst = torch.empty(max(int(lib.mrp_edge_encoder_bwd_t_workspace(E, C)) // 4, 1), device=dev)
                _lib.check(lib.mrp_edge_encoder_bwd_t(
                    _ptr(dhT), E, _ptr(hT), E, _ptr(pose), E, C, _ptr(dw1) if dw1 is not None else None,
                    _ptr(db1) if db1 is not None else None, _ptr(wst), wst.numel() * 4, st), "mrp_edge_encoder_bwd_t")
        if side is not None:
            cur.wait_stream(side)
    dpose = pose_grad(dhT, hT, w1) if need[0] else None
    return dpose, dw1, db1, dw2 if need[3] else None, db2


def _pad32(n: int) -> int:
    return (n + 31) // 32 * 32


class _PaddedWeights:
    """The encoder's weights zero-padded to C32 = C rounded up to 32 (W1 (C32, 9), b1 (C32), W2
    (2 C32, C32) with W2 in its top-left (2C, C) corner, b2 (2 C32)) and their packed image: the
    split kernels on these compute z's 2C columns exactly (every padded term a product with an exact
    zero) in the first 2C columns of a (E, 2 C32) result."""

    __slots__ = ("key", "C", "Cp", "w1", "b1", "w2", "b2", "img", "_w2t", "_w2t_img", "__weakref__")

    def w2t(self):
        if self._w2t is None:
            self._w2t = self.w2.t().contiguous()
        return self._w2t

    def w2t_img(self):
        if self._w2t_img is None:
            self._w2t_img = _pack_w2t(self.w2)
        return self._w2t_img


_padded = weakref.WeakKeyDictionary()


def padded_weights(l1: torch.nn.Linear, l2: torch.nn.Linear) -> "_PaddedWeights":
    """The zero-padded weights of an encoder whose C is not a multiple of 32 (or whose edge count is
    not), rebuilt when a weight changes (the keys of :func:`packed_weights`)."""
    w1, b1, w2, b2 = l1.weight, l1.bias, l2.weight, l2.bias
    key = tuple((t.data_ptr(), t._version, t.device.index) for t in (w1, b1, w2) + ((b2,) if b2 is not None else ()))
    hit = _padded.get(l2)
    if hit is not None and hit.key == key:
        return hit
    C = w1.shape[0]
    Cp = _pad32(C)
    dev = w1.device
    r = _PaddedWeights()
    r.key, r.C, r.Cp, r._w2t, r._w2t_img = key, C, Cp, None, None
    with torch.no_grad():
        r.w1 = torch.zeros((Cp, 9), device=dev)
        r.w1[:C] = w1
        r.b1 = torch.zeros((Cp,), device=dev)
        r.b1[:C] = b1
        r.w2 = torch.zeros((2 * Cp, Cp), device=dev)
        r.w2[: 2 * C, :C] = w2
        r.b2 = torch.zeros((2 * Cp,), device=dev)
        if b2 is not None:
            r.b2[: 2 * C] = b2
    r.img = _pack(r.w1, r.b1, r.w2)
    _track_image(r.img)
    _padded[l2] = r
    return r


def padded_supported(E: int, C: int) -> bool:
    """The padded split path's shapes: the padded operands (E32 x 2 C32 floats at most) addressable
    with 32-bit offsets and the padded weight image under 2^31 bytes."""
    Ep, Cp = _pad32(E), _pad32(C)
    return E > 0 and C > 0 and Ep * 2 * Cp * 4 < (1 << 31) and image_supported(Cp)


class EdgeEncoderPaddedFunction(torch.autograd.Function):
    """The split-bf16 training path (:class:`EdgeEncoderSplitFunction`'s kernels) for shapes it does not
    tile: E and C rounded up to 32 with zero pose rows, zero weight rows/columns (``padded_weights``)
    and zero gradient rows; z and every gradient are the leading blocks of the padded results."""

    @staticmethod
    def forward(ctx, pose, w1, b1, w2, b2, rec):
        E, C, Cp = pose.shape[0], rec.C, rec.Cp
        Ep = _pad32(E)
        dev = pose.device
        pp = torch.zeros((Ep, 9), device=dev)
        pp[:E] = pose.detach()
        zp = torch.empty((Ep, 2 * Cp), device=dev)
        hT = torch.empty((Cp, Ep), device=dev)
        lib = _lib.load_library()
        with torch.cuda.device(dev):
            _lib.check(lib.mrp_edge_encoder_fwd_split_train(
                _ptr(pp), _ptr(rec.img), _ptr(rec.b2), Ep, Cp, _ptr(zp), _ptr(hT), Ep,
                ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "mrp_edge_encoder_fwd_split_train")
        ctx.save_for_backward(pp, hT)
        ctx.rec, ctx.E = rec, E
        ctx.has_b2 = b2 is not None
        return zp[:E, : 2 * C].contiguous()

    @staticmethod
    def backward(ctx, dz):
        pp, hT = ctx.saved_tensors
        rec, E = ctx.rec, ctx.E
        C, Cp = rec.C, rec.Cp
        dev = dz.device
        need = list(ctx.needs_input_grad[:5])
        need[4] = need[4] and ctx.has_b2
        dzp = torch.zeros((pp.shape[0], 2 * Cp), device=dev)
        dzp[:E, : 2 * C] = dz
        dpose, dw1, db1, dw2, db2 = split_backward(dzp, pp, hT, rec.w1, need,
                                                   lambda i, shape: torch.empty(shape, device=dev),
                                                   rec.w2t, rec.w2t_img)
        return (dpose[:E] if dpose is not None else None,
                dw1[:C].contiguous() if dw1 is not None else None,
                db1[:C].contiguous() if db1 is not None else None,
                dw2[: 2 * C, :C].contiguous() if dw2 is not None else None,
                db2[: 2 * C].contiguous() if db2 is not None else None, None)


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
    C, E = l1.weight.shape[0], pose.shape[0]
    if _LOGITS_PATH == "split" and l1.bias is not None and tuple(l1.weight.shape) == (C, 9) \
            and tuple(l2.weight.shape) == (2 * C, C):
        if split_train_supported(E, C):
            PATH_COUNTS["split_train"] += 1
            return EdgeEncoderSplitFunction.apply(pose, l1.weight, l1.bias, l2.weight, l2.bias,
                                                  packed_weights(l1, l2), l2)
        if padded_supported(E, C):
            PATH_COUNTS["split_padded"] += 1
            return EdgeEncoderPaddedFunction.apply(pose, l1.weight, l1.bias, l2.weight, l2.bias,
                                                   padded_weights(l1, l2))
    PATH_COUNTS["autograd"] += 1
    return EdgeEncoderFunction.apply(*params)
