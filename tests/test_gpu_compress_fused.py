"""The fused aggregation + 1x1 compress kernel (``mrp_compress_film_fwd``; ``models.py:181-184``:
``conv1(torch.cat((h, gcn1(h)), 1))`` with the concatenation never written).

* Selector weights make the GEMM exact (0/1 products, fp32 accumulation of zeros): W = [0 | I]
  returns the aggregate, which must be bit-identical to ``film_mean`` (the same rounding sequence);
  W = [I | 0] returns x itself.
* Random weights: within max(1e-5, 4 x the fp32 restatement's error) of the float64 result
  (``tests/stack_ref.py``), as every other GEMM-bearing path.
* The GCN stack in eval mode (no autograd) takes the concatenation-free path (forced on here; by default on
  planes of >= models.FUSED_MIN_PLANE pixels); its output matches the unfused (cat kernel + batched GEMM)
  path to fp32 GEMM rounding.
* Both workgroup shapes: BM = 256 output channels (C % 256 == 0) and BM = 128 (C = 128, 384).
"""
import types

import numpy as np
import pytest
import torch

import mrp_gnn_amd as m
import stack_ref
from mrp_gnn_amd.compress import compress_film_fused

pytestmark = pytest.mark.gpu


def frames(B, N, C, H, seed):
    rng = np.random.RandomState(seed)
    gs = [m.frame_graph(np.concatenate([rng.uniform(-10, 10, (N, 3)), rng.standard_normal((N, 4))], 1)
                        .astype(np.float32)) for _ in range(B)]
    g = m.batch(gs)
    torch.manual_seed(seed)
    g.ndata["image"] = torch.randn(g.num_nodes(), C, H, H)
    return g


def conv_with(C, weight, bias=None):
    conv = torch.nn.Conv2d(2 * C, C, 1)
    with torch.no_grad():
        conv.weight.copy_(weight.reshape(C, 2 * C, 1, 1))
        conv.bias.copy_(torch.zeros(C) if bias is None else bias)
    return conv


@pytest.mark.parametrize("N,C,H", [(8, 128, 4), (5, 256, 8), (8, 128, 16), (2, 128, 4), (7, 384, 8), (3, 512, 16)])
@pytest.mark.parametrize("logits", [True, False])
def test_selector_weights_exact(cuda_device, N, C, H, logits):
    g = frames(3, N, C, H, seed=N + C + H).to(cuda_device)
    x = g.ndata["image"]
    torch.manual_seed(7)
    gb = (torch.randn if logits else torch.rand)(g.num_edges(), C, 2, device=cuda_device)
    csr = g.csr(cuda_device)
    mode = m._lib.MODE_FILM_MEAN | (m._lib.GB_LOGITS if logits else 0)
    eye, zero = torch.eye(C), torch.zeros(C, C)
    agg = m.film_mean(x, gb, csr, logits=logits)
    y = compress_film_fused(conv_with(C, torch.cat((zero, eye), 1)).to(cuda_device), x, gb, csr, mode)
    assert y is not None
    assert torch.equal(y, agg)
    y = compress_film_fused(conv_with(C, torch.cat((eye, zero), 1)).to(cuda_device), x, gb, csr, mode)
    assert torch.equal(y, x)


@pytest.mark.parametrize("B,N,C,H", [(4, 8, 512, 32), (6, 8, 1280, 8), (2, 8, 2048, 8), (5, 6, 256, 16)])
def test_random_weights_vs_float64(cuda_device, B, N, C, H):
    g = frames(B, N, C, H, seed=B * N + C)
    gd = g.to(cuda_device)
    x = gd.ndata["image"]
    torch.manual_seed(3)
    conv = torch.nn.Conv2d(2 * C, C, 1).to(cuda_device)
    z = torch.randn(g.num_edges(), C, 2, device=cuda_device)
    csr = gd.csr(cuda_device)
    y = compress_film_fused(conv, x, z, csr, m._lib.MODE_FILM_MEAN | m._lib.GB_LOGITS)
    assert y is not None
    src, dst = (t.to(cuda_device) for t in g.edges())

    def ref(dtype):
        xx = x.to(dtype)
        a = stack_ref.aggregate(xx, torch.sigmoid(z.to(dtype)), src, dst)
        return stack_ref.conv1x1(torch.cat((xx, a), 1), conv.weight.detach().to(dtype), conv.bias.detach().to(dtype))

    ok, e = stack_ref.within(y, ref(torch.float32), ref(torch.float64))
    assert ok, e


def test_unsupported_shapes_decline(cuda_device):
    g = frames(2, 8, 96, 4, seed=1).to(cuda_device)  # C % 128 != 0
    conv = torch.nn.Conv2d(192, 96, 1).to(cuda_device)
    z = torch.randn(g.num_edges(), 96, 2, device=cuda_device)
    assert compress_film_fused(conv, g.ndata["image"], z, g.csr(cuda_device), 0x100) is None
    gk = m.batch([m.frame_graph(np.random.RandomState(0).rand(10, 7).astype(np.float32), knn=3)])  # k-NN
    gk.ndata["image"] = torch.randn(10, 128, 4, 4)
    gk = gk.to(cuda_device)
    conv = torch.nn.Conv2d(256, 128, 1).to(cuda_device)
    z = torch.randn(gk.num_edges(), 128, 2, device=cuda_device)
    assert compress_film_fused(conv, gk.ndata["image"], z, gk.csr(cuda_device), 0x100) is None


def test_stack_eval_takes_fused_path(cuda_device):
    C = 256
    opt = types.SimpleNamespace(feature_dim=C, compress_gcn=True, multi_gcn=True)
    torch.manual_seed(0)
    net = m.GCNBlock(opt).to(cuda_device)
    g = frames(4, 8, C, 8, seed=2).to(cuda_device)
    x = g.ndata["image"]
    prev = m.models.fused_compress_setting()
    try:
        with torch.no_grad():
            m.models.set_fused_compress(True)
            fused = net(g, x)
            m.models.set_fused_compress(False)
            unfused = net(g, x)
    finally:
        m.models.set_fused_compress(prev)
    assert float((fused - unfused).abs().max() / unfused.abs().max()) <= 2e-6
    # with autograd the stack runs the unfused kernels (the fused kernel has no backward)
    out = net(g, x.clone().requires_grad_(True))
    assert out.grad_fn is not None


@pytest.mark.parametrize("C", [16, 128, 256])
def test_weight_pack_layout(cuda_device, C):
    """mrp_compress_weight_pack: wp[h][s][lk][m][k4] = w[m][h C + 16 s + 4 k4 + lk] (include/mrp_gnn.h)."""
    from mrp_gnn_amd.compress import _weight_packed
    conv = torch.nn.Conv2d(2 * C, C, 1).to(cuda_device)
    wp = _weight_packed(conv).cpu()
    w = conv.weight.detach().cpu().reshape(C, 2, C // 16, 4, 4)  # [m][h][s][k4][lk]
    ref = w.permute(1, 2, 4, 0, 3).reshape(-1)
    assert torch.equal(wp, ref)
    # cached per weight version; an in-place update repacks
    assert _weight_packed(conv) is _weight_packed(conv)
    with torch.no_grad():
        conv.weight.mul_(2)
    assert torch.equal(_weight_packed(conv).cpu(), ref * 2)


@pytest.mark.parametrize("n,C,H", [(128, 512, 8), (37, 128, 4), (8, 256, 16), (5, 384, 4)])
def test_dual_compress(cuda_device, n, C, H):
    """mrp_compress_dual_fwd: conv(cat(x, agg)) from two sources, any node count (partial last
    group of 8).  Selector weights make it exact; random weights within the GEMM yardstick."""
    from mrp_gnn_amd.compress import compress_dual
    torch.manual_seed(n + C)
    x = torch.randn(n, C, H, H, device=cuda_device)
    agg = torch.randn(n, C, H, H, device=cuda_device)
    eye, zero = torch.eye(C), torch.zeros(C, C)
    y = compress_dual(conv_with(C, torch.cat((zero, eye), 1)).to(cuda_device), x, agg)
    assert y is not None and torch.equal(y, agg)
    y = compress_dual(conv_with(C, torch.cat((eye, zero), 1)).to(cuda_device), x, agg)
    assert torch.equal(y, x)
    conv = torch.nn.Conv2d(2 * C, C, 1).to(cuda_device)
    y = compress_dual(conv, x, agg)
    w, b = conv.weight.detach(), conv.bias.detach()
    ok, e = stack_ref.within(y, stack_ref.conv1x1(torch.cat((x, agg), 1), w, b),
                             stack_ref.conv1x1(torch.cat((x, agg), 1).double(), w.double(), b.double()))
    assert ok, e


def test_dual_equals_fused(cuda_device):
    """The two-pass path (aggregate kernel, then the dual GEMM) gives the fused kernel's bits: the same
    aggregate and the same MFMA K order."""
    from mrp_gnn_amd.compress import compress_dual
    g = frames(4, 8, 256, 8, seed=11).to(cuda_device)
    x = g.ndata["image"]
    z = torch.randn(g.num_edges(), 256, 2, device=cuda_device)
    csr = g.csr(cuda_device)
    conv = torch.nn.Conv2d(512, 256, 1).to(cuda_device)
    mode = m._lib.MODE_FILM_MEAN | m._lib.GB_LOGITS
    fused = compress_film_fused(conv, x, z, csr, mode)
    agg = m.film_mean(x, z, csr, logits=True)
    assert torch.equal(compress_dual(conv, x, agg), fused)


def test_dual_equals_fused_configs1_size_repeated(cuda_device):
    """configs[1]'s shape (B=16, N=8, C=512, 32x32: 4096 workgroups in flight), five launches: every
    launch gives the fused kernel's bits.  A stage read before its LDS-DMA landed (the producers'
    vmcnt wait) shows up here as NaN or run-to-run differences; small grids hid it."""
    from mrp_gnn_amd.compress import compress_dual
    g = frames(16, 8, 512, 32, seed=12).to(cuda_device)
    x = g.ndata["image"]
    z = torch.randn(g.num_edges(), 512, 2, device=cuda_device)
    csr = g.csr(cuda_device)
    conv = torch.nn.Conv2d(1024, 512, 1).to(cuda_device)
    mode = m._lib.MODE_FILM_MEAN | m._lib.GB_LOGITS
    fused = compress_film_fused(conv, x, z, csr, mode)
    assert torch.isfinite(fused).all()
    agg = m.film_mean(x, z, csr, logits=True)
    for _ in range(5):
        assert torch.equal(compress_dual(conv, x, agg), fused)


def test_stack_eval_fused_mode(cuda_device):
    """set_fused_compress("fused"): the single fused kernel in the eval stack, equal to the two-pass
    path bit for bit (same aggregate, same MFMA order)."""
    C = 256
    opt = types.SimpleNamespace(feature_dim=C, compress_gcn=True, multi_gcn=True)
    torch.manual_seed(1)
    net = m.GCNBlock(opt).to(cuda_device)
    g = frames(3, 8, C, 8, seed=4).to(cuda_device)
    x = g.ndata["image"]
    prev = m.models.fused_compress_setting()
    try:
        with torch.no_grad():
            m.models.set_fused_compress("fused")
            a = net(g, x)
            m.models.set_fused_compress(True)
            b = net(g, x)
    finally:
        m.models.set_fused_compress(prev)
    assert torch.equal(a, b)


@pytest.mark.parametrize("B,N,C,H", [(3, 8, 256, 8), (2, 5, 128, 16), (2, 8, 128, 32)])
def test_training_concatenation_free_layer(cuda_device, B, N, C, H):
    """With autograd and set_training_compress(True) the layer trains through FilmCompressFunction
    (aggregate kernel + two-source GEMM forward; W^T dy, one aggregation-backward pass with the x half
    as its base, two half-width weight-gradient GEMMs): the output, the input gradient and every
    parameter gradient agree with the cat kernel + batched GEMM path to fp32 GEMM rounding."""
    opt = types.SimpleNamespace(feature_dim=C, compress_gcn=True, multi_gcn=True)
    torch.manual_seed(5)
    net = m.GCNBlock(opt).to(cuda_device)
    g = frames(B, N, C, H, seed=B + N + C + H).to(cuda_device)
    x0 = g.ndata["image"]
    G = torch.randn_like(x0)
    res = []
    try:
        for setting in (True, False):
            m.models.set_training_compress(setting)
            net.zero_grad()
            x = x0.clone().requires_grad_(True)
            y = net(g, x)
            (y * G).sum().backward()
            res.append((y.detach(), x.grad, {k: p.grad.clone() for k, p in net.named_parameters()}))
    finally:
        m.models.set_training_compress(False)
    (ya, dxa, pa), (yb, dxb, pb) = res

    def rel(a, b):
        return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))

    assert rel(ya, yb) <= 2e-6
    assert rel(dxa, dxb) <= 1e-5
    for k in pb:
        assert rel(pa[k], pb[k]) <= 1e-5, k
