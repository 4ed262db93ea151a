"""The split-bf16 compress kernel forms the library builds (``csrc/compress_split.hip``): forward / data
gradient (knob ``gemm_split``): 2 = 128-row workgroups on 32x32x16 MFMAs (the fallback where M % 256 != 0),
7 = 256-row workgroups on 16x16x32 MFMAs (the default where M % 256 == 0) — each forced on every shape
and held to float64 with the fp32 yardstick, across ragged M and column tails, the shortest K (two 16-k
stages) and planes smaller than a column tile; every launch of a kernel must repeat the last bit for bit
at a BASELINE config size (the guard against an LDS-DMA ordering race: a read that overtakes the DMA it
depends on gives rare, shifting errors).  Weight gradient (knob ``split_nt``): 3 = both operands split
in the kernel, 4 = dy split once (split_rows + gemm_nt_psa), bit-identical dW at the same split.
Round 4's other forms are lab code (tools/lab_forms.hip)."""
import contextlib

import pytest
import torch

import mrp_gnn_amd as m

pytestmark = pytest.mark.gpu



@contextlib.contextmanager
def _form(v):
    lib = m.load_library()
    prev = m.compress.compress_path()
    m.compress.set_compress_path("split")
    assert lib.mrp_tuning_set(b"gemm_split", v) == 0
    try:
        yield
    finally:
        lib.mrp_tuning_set(b"gemm_split", -1)
        m.compress.set_compress_path(prev)


@pytest.mark.parametrize("form", [2, 7])
def test_config1_size_repeats_bit_identical(cuda_device, form):
    """configs[1]'s layer shape (128 nodes, C = 512, 32 x 32): forward, data gradient and weight
    gradient launched repeatedly on the same inputs give the same bits every time."""
    torch.manual_seed(11)
    dev = cuda_device
    n, C, H, W = 128, 512, 32, 32
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    b = torch.randn(C, device=dev)
    x, a, gy = (torch.randn(n, C, H, W, device=dev) for _ in range(3))
    with _form(form):
        y0 = m.compress.compress_forward(w, b, x, a)
        d0 = m.compress.compress_backward_data(w, gy)
        w0 = m.compress.compress_backward_weight(gy, x, a)
        for _ in range(4):
            assert torch.equal(m.compress.compress_forward(w, b, x, a), y0)
            d = m.compress.compress_backward_data(w, gy)
            assert torch.equal(d[0], d0[0]) and torch.equal(d[1], d0[1])
            g = m.compress.compress_backward_weight(gy, x, a)
            assert torch.equal(g[0], w0[0]) and torch.equal(g[1], w0[1])


@pytest.mark.parametrize("n,C,H,W", [(3, 32, 2, 2), (5, 64, 4, 4), (7, 160, 4, 8), (2, 256, 8, 8), (9, 288, 2, 6),
                                     (33, 96, 8, 8), (4, 512, 16, 16), (1, 256, 1, 4), (17, 320, 4, 4),
                                     (16, 1280, 8, 8)])
@pytest.mark.parametrize("form", [2, 7])
def test_forms_vs_float64(cuda_device, form, n, C, H, W):
    """Form 7 (16x16x32 MFMAs, the default where M % 256 == 0) and form 2 (32x32x16, the fallback),
    each forced on every shape (ragged M tiles and column tails, the shortest K, planes smaller than a
    column tile): forward and data gradient against float64 with the fp32 yardstick, repeated launches
    bit-identical."""
    import stack_ref
    torch.manual_seed(n * 5 + C)
    dev = cuda_device
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    b = torch.randn(C, device=dev)
    x, a, gy = (torch.randn(n, C, H, W, device=dev) for _ in range(3))
    with _form(form):
        y = m.compress.compress_forward(w, b, x, a)
        gx, ga = m.compress.compress_backward_data(w, gy)
        assert torch.equal(y, m.compress.compress_forward(w, b, x, a))
        d = m.compress.compress_backward_data(w, gy)
        assert torch.equal(d[0], gx) and torch.equal(d[1], ga)
    cat = torch.cat((x, a), 1)
    w2 = w.reshape(C, 2 * C)
    y32 = torch.einsum("oc,nchw->nohw", w2, cat) + b.view(1, C, 1, 1)
    y64 = torch.einsum("oc,nchw->nohw", w2.double(), cat.double()) + b.double().view(1, C, 1, 1)
    ok, errs = stack_ref.within(y, y32, y64)
    assert ok, ("y", errs)
    g32 = torch.einsum("oc,nohw->nchw", w2, gy)
    g64 = torch.einsum("oc,nohw->nchw", w2.double(), gy.double())
    ok, errs = stack_ref.within(torch.cat((gx, ga), 1), g32, g64)
    assert ok, ("grad", errs)


@pytest.mark.parametrize("form", [3, 4])
@pytest.mark.parametrize("n,C,H,W", [(16, 64, 8, 8), (10, 128, 16, 16), (64, 256, 8, 8), (7, 160, 4, 8), (2, 32, 32, 32),
                                     (33, 96, 8, 8), (8, 512, 8, 8), (3, 320, 16, 16), (128, 512, 32, 32),
                                     (1024, 512, 4, 8), (256, 1280, 8, 8)])
def test_weight_gradient_forms_vs_float64(cuda_device, form, n, C, H, W):
    """The weight gradient on each NT kernel form (split_nt 3: 32-k stages on 16x16x32 MFMAs, both
    operands split in the kernel; 4 (the default where C >= 1024): dy split once into a packed image,
    split_rows + gemm_nt_psa) against float64 with the fp32 yardstick, repeated launches bit-identical;
    forms 3 and 4 compute the same products in the same order per output (bit-identical dW at equal
    splits; form 4's bias sums dy in other groups)."""
    import stack_ref
    torch.manual_seed(n * 13 + C)
    dev = cuda_device
    x, a, gy = (torch.randn(n, C, H, W, device=dev) for _ in range(3))
    lib = m.load_library()
    prev = m.compress.compress_path()
    m.compress.set_compress_path("split")
    assert lib.mrp_tuning_set(b"split_nt", form) == 0
    try:
        gw, gb = m.compress.compress_backward_weight(gy, x, a)
        again = m.compress.compress_backward_weight(gy, x, a)
        if form == 4:
            assert lib.mrp_tuning_set(b"split_nt", 3) == 0
            assert torch.equal(gw, m.compress.compress_backward_weight(gy, x, a)[0])
    finally:
        lib.mrp_tuning_set(b"split_nt", -1)
        m.compress.set_compress_path(prev)
    assert torch.equal(gw, again[0]) and torch.equal(gb, again[1])
    cat = torch.cat((x, a), 1)
    w64 = torch.einsum("nohw,nchw->oc", gy.double(), cat.double()).reshape(C, 2 * C, 1, 1)
    w32 = torch.einsum("nohw,nchw->oc", gy, cat).reshape(C, 2 * C, 1, 1)
    ok, errs = stack_ref.within(gw, w32, w64)
    assert ok, ("gw", errs)
    ok, errs = stack_ref.within(gb, gy.sum((0, 2, 3)), gy.double().sum((0, 2, 3)))
    assert ok, ("gb", errs)

