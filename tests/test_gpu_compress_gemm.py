"""The matrix-core compress kernels — fp32 MFMA (``csrc/compress_gemm.hip``: ``mrp_compress_fwd``,
``mrp_compress_bwd_data``, ``mrp_compress_bwd_weight``) and split-bf16 (``csrc/compress_split.hip``:
``mrp_compress_fwd_split``, ``mrp_compress_bwd_data_split``) — against a float64 restatement of the
reference's 1x1 conv over the concatenation (``dgl/model/models.py:163-165,182-184``).

Bound: the error against float64 must be within max(1e-5, 4 x the error of torch's own fp32 GEMM of
the same product) — i.e. as accurate as an fp32 computation of the reference op, whatever the
summation order (``tests/stack_ref.within``)."""
import contextlib

import pytest
import torch

import mrp_gnn_amd as m
from stack_ref import within

pytestmark = pytest.mark.gpu


def _ref(w, b, x, a, gy, dtype):
    """(y, gx, ga, gw, gb) of conv(cat(x, a)) in dtype, by einsum."""
    C = x.shape[1]
    w2 = w.reshape(C, 2 * C).to(dtype)
    cat = torch.cat((x, a), 1).to(dtype)
    y = torch.einsum("oc,nchw->nohw", w2, cat) + b.to(dtype)[None, :, None, None]
    g = gy.to(dtype)
    gcat = torch.einsum("oc,nohw->nchw", w2, g)
    gw = torch.einsum("nohw,nchw->oc", g, cat)
    return y, gcat[:, :C], gcat[:, C:], gw.reshape(C, 2 * C, 1, 1), g.sum((0, 2, 3))


@contextlib.contextmanager
def _path(path):
    """"split" (per-shape workgroup), "split2" (128-row workgroups forced), "hip" (fp32 MFMA)."""
    prev = m.compress.compress_path()
    lib = m.load_library()
    m.compress.set_compress_path("split" if path.startswith("split") else path)
    if path == "split2":
        assert lib.mrp_tuning_set(b"gemm_split", 2) == 0
    try:
        yield
    finally:
        m.compress.set_compress_path(prev)
        lib.mrp_tuning_set(b"gemm_split", -1)


PATHS = ["split", "split2", "hip"]


def _check(ours, f32, f64, what):
    ok, errs = within(ours, f32, f64)
    assert ok, f"{what}: error {errs[0]:.3g} vs fp32 restatement {errs[1]:.3g}"


SHAPES = [(16, 64, 8, 8), (5, 96, 4, 4), (3, 32, 2, 2), (10, 128, 16, 16), (64, 256, 8, 8), (7, 160, 4, 8),
          (2, 32, 32, 32), (9, 224, 2, 6), (1, 32, 1, 4), (33, 96, 8, 8)]


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("n,C,H,W", SHAPES)
def test_compress_gemm_matches_float64(cuda_device, n, C, H, W, path):
    torch.manual_seed(n * 131 + C)
    dev = cuda_device
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    b = torch.randn(C, device=dev)
    x = torch.randn(n, C, H, W, device=dev)
    a = torch.randn(n, C, H, W, device=dev)
    gy = torch.randn(n, C, H, W, device=dev)
    with _path(path):
        y = m.compress.compress_forward(w, b, x, a)
        gx, ga = m.compress.compress_backward_data(w, gy)
        r = m.compress.compress_backward_weight(gy, x, a)
    r64 = _ref(w, b, x, a, gy, torch.float64)
    r32 = _ref(w, b, x, a, gy, torch.float32)
    for name, o, f32, f64 in zip(("y", "gx", "ga"), (y, gx, ga), r32, r64):
        _check(o, f32, f64, name)
    if H * W % 32 != 0:
        assert r is None  # the weight-gradient kernel declines planes that are not whole 32-pixel stages
        return
    for name, o, f32, f64 in zip(("gw", "gb"), r, r32[3:], r64[3:]):
        _check(o, f32, f64, name)


def _no_library_gemm(monkeypatch):
    """Make torch's GEMM forms of the compress (the A/B comparison path) fail if anything calls them."""
    def boom(*_a, **_k):
        raise AssertionError("a library GEMM ran on the product path")
    for name in ("_lib_forward", "_lib_backward_data", "_lib_backward_weight"):
        monkeypatch.setattr(m.compress, name, boom)


@pytest.mark.parametrize("path", ["split", "hip"])
@pytest.mark.parametrize("n,C,H,W", [(6, 48, 8, 8), (4, 64, 3, 5), (5, 64, 4, 4), (3, 100, 7, 7), (2, 1, 1, 1),
                                     (4, 96, 6, 6), (2, 33, 9, 9)])
def test_compress_function_declined_shapes(cuda_device, monkeypatch, n, C, H, W, path):
    """CompressFunction on shapes the kernels do not tile (C % 32, H W % 4, or H W % 32 for the weight
    gradient): the same kernels on zero-padded operands — never torch's GEMMs — and
    every output and gradient against float64."""
    _no_library_gemm(monkeypatch)
    torch.manual_seed(n + C + H)
    dev = cuda_device
    w = (torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5).requires_grad_(True)
    b = torch.randn(C, device=dev, requires_grad=True)
    x = torch.randn(n, C, H, W, device=dev, requires_grad=True)
    a = torch.randn(n, C, H, W, device=dev, requires_grad=True)
    gy = torch.randn(n, C, H, W, device=dev)
    with _path(path):
        for step in range(2):  # the second after an in-place weight update: padded weights rebuilt
            for t in (w, b, x, a):
                t.grad = None
            y = m.compress.CompressFunction.apply(x, a, w, b)
            y.backward(gy)
            r64 = _ref(w.detach(), b.detach(), x.detach(), a.detach(), gy, torch.float64)
            r32 = _ref(w.detach(), b.detach(), x.detach(), a.detach(), gy, torch.float32)
            for name, o, f32, f64 in zip(("y", "gx", "ga", "gw", "gb"), (y, x.grad, a.grad, w.grad, b.grad), r32, r64):
                _check(o, f32, f64, f"{name} (step {step})")
            with torch.no_grad():
                w.mul_(-0.5)
                b.add_(1.0)


@pytest.mark.parametrize("path", PATHS)
def test_compress_gemm_cat_buffer_halves(cuda_device, path):
    """Operands and outputs as the two halves of (N, 2C, H, W) buffers (node stride 2 C P)."""
    torch.manual_seed(3)
    n, C, H, W = 12, 96, 8, 8
    dev = cuda_device
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    b = torch.randn(C, device=dev)
    cat = torch.randn(n, 2 * C, H, W, device=dev)
    x, a = cat[:, :C], cat[:, C:]
    gy = torch.randn(n, C, H, W, device=dev)
    gcat = torch.full((n, 2 * C, H, W), float("nan"), device=dev)
    with _path(path):
        y = m.compress.compress_forward(w, b, x, a)
        m.compress.compress_backward_data(w, gy, gcat[:, :C], gcat[:, C:])
        gw, gb = m.compress.compress_backward_weight(gy, x, a)
    r64 = _ref(w, b, x.contiguous(), a.contiguous(), gy, torch.float64)
    r32 = _ref(w, b, x.contiguous(), a.contiguous(), gy, torch.float32)
    _check(y, r32[0], r64[0], "y")
    _check(gcat, torch.cat(r32[1:3], 1), torch.cat(r64[1:3], 1), "gcat")
    _check(gw, r32[3], r64[3], "gw")
    _check(gb, r32[4], r64[4], "gb")


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("n,C,H,W", [(128, 512, 32, 32), (256, 1280, 8, 8), (64, 2048, 8, 8), (128, 1024, 16, 16)])
def test_compress_gemm_config_sizes(cuda_device, n, C, H, W, path):
    """The BASELINE configs' per-GPU layer shapes (configs[1..4]): forward, both gradients."""
    torch.manual_seed(C)
    dev = cuda_device
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    b = torch.randn(C, device=dev)
    x = torch.randn(n, C, H, W, device=dev)
    a = torch.randn(n, C, H, W, device=dev)
    gy = torch.randn(n, C, H, W, device=dev)
    with _path(path):
        y = m.compress.compress_forward(w, b, x, a)
        gx, ga = m.compress.compress_backward_data(w, gy)
        gw, gb = m.compress.compress_backward_weight(gy, x, a)
    r64 = _ref(w, b, x, a, gy, torch.float64)
    r32 = _ref(w, b, x, a, gy, torch.float32)
    del x, a
    for name, o, f32, f64 in zip(("y", "gx", "ga", "gw", "gb"), (y, gx, ga, gw, gb), r32, r64):
        _check(o, f32, f64, name)


@pytest.mark.parametrize("path", PATHS)
def test_compress_gemm_deterministic(cuda_device, path):
    torch.manual_seed(5)
    n, C, H, W = 64, 256, 8, 8
    dev = cuda_device
    x = torch.randn(n, C, H, W, device=dev)
    a = torch.randn(n, C, H, W, device=dev)
    gy = torch.randn(n, C, H, W, device=dev)
    w = torch.randn(C, 2 * C, 1, 1, device=dev)
    with _path(path):
        first = m.compress.compress_backward_weight(gy, x, a)
        fy = m.compress.compress_forward(w, None, x, a)
        fd = m.compress.compress_backward_data(w, gy)
        for _ in range(3):
            again = m.compress.compress_backward_weight(gy, x, a)
            assert torch.equal(first[0], again[0]) and torch.equal(first[1], again[1])
            assert torch.equal(fy, m.compress.compress_forward(w, None, x, a))
            d = m.compress.compress_backward_data(w, gy)
            assert torch.equal(fd[0], d[0]) and torch.equal(fd[1], d[1])


def test_split_pack_follows_weight_updates(cuda_device):
    """The packed split-bf16 weight images are rebuilt after an in-place (optimizer-style) update and
    after clear_packed_weights() for writes through .data; the ABI declines unsupported shapes."""
    torch.manual_seed(9)
    n, C, H, W = 8, 64, 8, 8
    dev = cuda_device
    w = torch.nn.Parameter(torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5)
    b = torch.randn(C, device=dev)
    x, a, gy = (torch.randn(n, C, H, W, device=dev) for _ in range(3))
    with _path("split"):
        y0 = m.compress.compress_forward(w, b, x, a)
        with torch.no_grad():
            w.mul_(-2.0)
        y1 = m.compress.compress_forward(w, b, x, a)
        _check(y1, *(_ref(w.detach(), b, x, a, gy, t)[0] for t in (torch.float32, torch.float64)), "y after update")
        w.data.mul_(0.5)
        m.compress.clear_packed_weights()
        g1 = m.compress.compress_backward_data(w, gy)
        r32, r64 = (_ref(w.detach(), b, x, a, gy, t) for t in (torch.float32, torch.float64))
        _check(g1[0], r32[1], r64[1], "gx after .data write")
    assert not torch.equal(y0, y1)
    lib = m.load_library()
    assert lib.mrp_compress_split_pack_bytes(48, 96) == 0 and lib.mrp_compress_split_pack_bytes(64, 128) == 64 * 128 * 6


def test_compress_gemm_empty_and_unsupported(cuda_device):
    dev = cuda_device
    lib = m.load_library()
    w = torch.randn(8, 16, 1, 1, device=dev)
    w64 = torch.randn(64, 128, 1, 1, device=dev)
    x = torch.randn(0, 64, 8, 8, device=dev)
    assert m.compress.compress_forward(w64, None, x, x).shape == (0, 64, 8, 8)
    gw, gb = m.compress.compress_backward_weight(torch.randn(0, 64, 8, 8, device=dev), x, x)
    assert torch.count_nonzero(gw) == 0 and torch.count_nonzero(gb) == 0
    # P % 4 != 0 or C % 32 != 0: declined (the Python layer runs torch's GEMMs instead)
    from mrp_gnn_amd.aggregate import _ptr
    z = torch.zeros(2, 32, 3, 5, device=dev)
    w32 = torch.randn(32, 64, device=dev)
    assert lib.mrp_compress_fwd(_ptr(z), 480, _ptr(z), 480, 2, 32, 15, _ptr(w32), None, _ptr(z), 480, None) == \
        m._lib.HIP_ERROR_NOT_SUPPORTED
    z = torch.zeros(2, 8, 4, 4, device=dev)
    assert lib.mrp_compress_fwd(_ptr(z), 128, _ptr(z), 128, 2, 8, 16, _ptr(w), None, _ptr(z), 128, None) == \
        m._lib.HIP_ERROR_NOT_SUPPORTED
