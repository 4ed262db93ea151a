"""Every BASELINE.json config at its full per-GPU shape on the HIP path, forward and backward, against
a float64 restatement of the same stack (``tests/stack_ref.py``), plus the same stacks at reduced
size against the CPU oracle.

Tolerance: the aggregation alone is held to max|d| / max|ref| <= 1e-5 elsewhere
(``test_gpu_parity.py``).  A stack also contains the encoder GEMM (K = C) and the 1x1 compress GEMMs
(K = 2C = 2560 / 4096 terms here), whose summation order differs between libraries; so a stack result
is accepted when its error against the float64 stack is within max(1e-5, 4 x the error of the same
restatement computed in fp32) — the HIP path is as accurate as an fp32 run of the reference's ops.

Configs (BASELINE.json ``configs``):
  [1] B=16, N=8 complete, C=512, 32x32, 2 layers (multi_gcn + compress)
  [2] B=32, N=8 complete, C=1280, 8x8, gcn1 -> cat -> conv1 (gcn_compress)
  [3] B=8 per GPU (32 over 4), N=8 complete, C=2048, 8x8, 2 layers (multi_gcn + compress)
  [4] B=8 per GPU (64 over 8), N=16 k-NN(4), C=1024, 16x16, 3 layers
"""
import types

import numpy as np
import pytest
import torch

import mrp_gnn_amd as m
import oracle
import stack_ref
from conftest import rel_err

pytestmark = pytest.mark.gpu


def frames(B, N, C, H, W, seed, knn=None):
    rng = np.random.RandomState(seed)
    gs = []
    for _ in range(B):
        poses = np.concatenate([rng.uniform(-10, 10, (N, 3)), rng.standard_normal((N, 4))], 1).astype(np.float32)
        gs.append(m.frame_graph(poses, knn=knn))
    g = m.batch(gs)
    torch.manual_seed(seed)
    g.ndata["image"] = torch.randn(g.num_nodes(), C, H, W)
    return g


def model(C, layers, combine="cat_compress", seed=0):
    torch.manual_seed(seed)
    opt = types.SimpleNamespace(feature_dim=C, compress_gcn=combine == "cat_compress", multi_gcn=False,
                                gcn_layers=layers, gcn_combine=combine, gcn2_alpha=0.25)
    return m.GCNStack(opt)


def check_config(dev, B, N, C, H, layers, knn=None, combine="cat_compress"):
    g = frames(B, N, C, H, H, seed=B * 7 + N + C, knn=knn).to(dev)
    net = model(C, layers, combine).to(dev)
    params = {k: v.detach() for k, v in net.named_parameters()}
    x = g.ndata["image"].detach().clone().requires_grad_(True)
    out = net(g, x)
    torch.manual_seed(1)
    G = torch.randn_like(out)
    out.backward(G)
    src, dst = (t.to(dev) for t in g.edges())
    pose = g.edata["pose"]
    kw = dict(layers=layers, combine=combine, alpha=0.25)
    f64 = stack_ref.run(params, x, pose, src, dst, G, torch.float64, **kw)
    f32 = stack_ref.run(params, x, pose, src, dst, G, torch.float32, **kw)
    ok, e = stack_ref.within(out, f32[0], f64[0])
    assert ok, ("forward", e)
    ok, e = stack_ref.within(x.grad, f32[1], f64[1])
    assert ok, ("dx", e)
    for k, p in net.named_parameters():
        ok, e = stack_ref.within(p.grad, f32[2][k], f64[2][k])
        assert ok, (k, e)


def test_config2_full_size(cuda_device):
    """configs[2]: 8-robot airsim graph, C=1280 (MobileNetV2), 8x8, B=32, gcn1 -> cat -> conv1."""
    check_config(cuda_device, B=32, N=8, C=1280, H=8, layers=1)


def test_config3_full_size(cuda_device):
    """configs[3]: 8-robot warehouse, C=2048 (ResNet50), 8x8, 8 graphs per GPU, 2 layers + compress."""
    check_config(cuda_device, B=8, N=8, C=2048, H=8, layers=2)


def test_config4_full_size(cuda_device):
    """configs[4]: 16-robot k-NN(4), C=1024, 16x16, 8 graphs per GPU, 3 GCN layers (the k-NN frames are
    MRP_GRAPH_REGULAR(4): per-edge-slot forward and backward)."""
    check_config(cuda_device, B=8, N=16, C=1024, H=16, layers=3, knn=4)


@pytest.mark.parametrize("B,N,C,H,layers,knn", [(3, 5, 48, 7, 2, None), (2, 8, 100, 6, 1, None),
                                                 (2, 10, 40, 5, 2, 3)])
def test_odd_shapes_stay_on_hip_kernels(cuda_device, monkeypatch, B, N, C, H, layers, knn):
    """A user of the reference with ``feature_dim`` and plane sizes no BASELINE config has (C % 32 != 0,
    H W % 4 != 0): the encoder and the compress run the hand-written kernels on zero-padded operands
    (no library GEMM: the comparison forms are patched to fail), forward and every gradient against
    float64."""
    def boom(*_a, **_k):
        raise AssertionError("a library GEMM ran on the product path")
    for name in ("_lib_forward", "_lib_backward_data", "_lib_backward_weight"):
        monkeypatch.setattr(m.compress, name, boom)
    before = m.encoder.PATH_COUNTS["autograd"]
    check_config(cuda_device, B=B, N=N, C=C, H=H, layers=layers, knn=knn)
    assert m.encoder.PATH_COUNTS["autograd"] == before  # the fp32 encoder (library backward) never ran


def test_config1_full_size(cuda_device):
    """configs[1]: 8-robot warehouse, ResNet18 C=512 at H/8 x W/8 = 32x32, batch 16, 2 layers (multi_gcn +
    compress, ``dgl/model/models.py:180-189``) — the grid sizes the benchmark runs (forward, dx and
    every parameter gradient against float64)."""
    check_config(cuda_device, B=16, N=8, C=512, H=32, layers=2)


def test_config0_own_shape_vs_oracle(cuda_device):
    """configs[0]: the reference's CPU-runnable case (``dgl/training.py:28,176-218``) at its own shape —
    B = 8 complete 4-robot graphs, C = 64, 32 x 32, one GCN layer (``dgl/model/models.py:207-226``) —
    through the drop-in ``GCN`` on the HIP path, against the CPU oracle (``oracle.gcn_forward`` and
    torch autograd through it) at the north-star 1e-5:
      * the aggregation fed the oracle's own gamma/beta: bit-identical (each destination's sum over its 3
        sources is sequential in source order, as in the reference's mailbox mean);
      * the no-grad forward (the split-bf16 encoder, as bench.py's configs[0] record times it) and the
        training forward;
      * dx and the four edge-encoder parameter gradients (also held to float64 with the fp32 yardstick)."""
    B, N, C, H = 8, 4, 64, 32
    g = frames(B, N, C, H, H, seed=77)
    torch.manual_seed(0)
    gcn = m.GCN(types.SimpleNamespace(feature_dim=C))
    params = {k: v.detach().clone() for k, v in gcn.edge_encoder.named_parameters()}
    src, dst = (t.numpy() for t in g.edges())
    x, pose = g.ndata["image"], g.edata["pose"]
    # CPU oracle: forward and autograd through the reference op sequence
    p_ref = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    x_ref = x.clone().requires_grad_(True)
    ref = oracle.gcn_forward(p_ref, x_ref, pose, src, dst)
    torch.manual_seed(1)
    G = torch.randn_like(ref)
    ref.backward(G)
    gb_ref = oracle.edge_encoder_forward(params, pose)

    gd = g.to(cuda_device)
    gcn = gcn.to(cuda_device)
    xd = gd.ndata["image"]
    # the aggregation alone on the oracle's gamma/beta: the reference's rounding sequence
    agg = m.film_mean(xd, gb_ref.to(cuda_device), gd.csr(cuda_device)).cpu()
    assert torch.equal(agg, oracle.film_aggregate(x, gb_ref, src, dst))
    with torch.no_grad():
        out_eval = gcn(gd, xd).cpu()
    assert rel_err(out_eval.numpy(), ref.detach().numpy()) <= 1e-5
    xr = xd.detach().clone().requires_grad_(True)
    out = gcn(gd, xr)
    out.backward(G.to(cuda_device))
    assert rel_err(out.detach().cpu().numpy(), ref.detach().numpy()) <= 1e-5
    assert rel_err(xr.grad.cpu().numpy(), x_ref.grad.numpy()) <= 1e-5
    # float64 yardstick for the parameter gradients (GEMM sums: any order is as good as fp32's)
    sd, dd = (t.to(cuda_device).long() for t in g.edges())

    def layer_grads(dtype):
        p = {k: v.to(cuda_device, dtype).requires_grad_(True) for k, v in params.items()}
        a = stack_ref.aggregate(xd.to(dtype), stack_ref.edge_gb(p, "", gd.edata["pose"]), sd, dd)
        a.backward(G.to(cuda_device, dtype))
        return {k: v.grad for k, v in p.items()}

    g64, g32 = layer_grads(torch.float64), layer_grads(torch.float32)
    for k, p in gcn.edge_encoder.named_parameters():
        assert rel_err(p.grad.cpu().numpy(), p_ref[k].grad.numpy()) <= 1e-5, k
        ok, e = stack_ref.within(p.grad, g32[k], g64[k])
        assert ok, (k, e)


def test_config1_shape_reduced_batch(cuda_device):
    """configs[1] (B=16, C=512, 32x32, 2 layers) at B=4: the 32x32 geometry (plane split forward,
    two-wave backward) through the whole stack."""
    check_config(cuda_device, B=4, N=8, C=512, H=32, layers=2)


@pytest.mark.parametrize("combine", ["residual", "initial_mix"])
def test_residual_and_mix_stacks_full_size(cuda_device, combine):
    """The epilogue combinations at the configs[4] shape (3 layers, k-NN(4), C=1024, 16x16)."""
    check_config(cuda_device, B=4, N=16, C=1024, H=16, layers=3, knn=4, combine=combine)


# ------------------------------------------------------------------ reduced size vs the CPU oracle
def oracle_stack(net, g, x, layers, combine, alpha=0.25):
    src, dst = (t.numpy() for t in g.edges())
    h0 = h = x
    for i in range(1, layers + 1):
        gcn = getattr(net, f"gcn{i}")
        params = {k: v for k, v in gcn.edge_encoder.named_parameters()}
        a = oracle.film_aggregate(h, oracle.edge_encoder_forward(params, g.edata["pose"]), src, dst)
        if combine == "cat_compress":
            h = getattr(net, f"conv{i}")(torch.cat((h, a), 1))
        elif combine == "residual":
            h = h + a
        else:
            h = (1.0 - alpha) * a + alpha * h0
    return h


@pytest.mark.parametrize("combine", ["cat_compress", "residual", "initial_mix"])
@pytest.mark.parametrize("knn", [None, 4])
def test_three_layer_stack_vs_oracle(cuda_device, combine, knn):
    N = 12 if knn else 6
    g = frames(3, N, 16, 4, 4, seed=5, knn=knn)
    net = model(16, 3, combine, seed=3)
    x = g.ndata["image"].clone().requires_grad_(True)
    ref = oracle_stack(net, g, x, 3, combine)
    G = torch.randn_like(ref)
    ref.backward(G)
    ref_grads = {k: p.grad.clone() for k, p in net.named_parameters()}
    netd = model(16, 3, combine, seed=3).to(cuda_device)
    gd = g.to(cuda_device)
    xd = gd.ndata["image"].detach().clone().requires_grad_(True)
    out = netd(gd, xd)
    out.backward(G.to(cuda_device))
    assert rel_err(out.detach().cpu().numpy(), ref.detach().numpy()) <= 1e-5
    assert rel_err(xd.grad.cpu().numpy(), x.grad.numpy()) <= 1e-5
    for k, p in netd.named_parameters():
        assert rel_err(p.grad.cpu().numpy(), ref_grads[k].numpy()) <= 1e-5, k


def test_residual_forward_bit_exact_vs_oracle(cuda_device):
    """out = x + aggregate: the kernel's fl(a + x[v]) is torch's ``g_h + h`` (dgl_models.py:37)."""
    for knn, N in ((None, 8), (4, 16), (None, 5)):
        g = frames(3, N, 16, 8, 8, seed=N, knn=knn)
        x = g.ndata["image"]
        torch.manual_seed(2)
        gb = torch.rand(g.num_edges(), 16, 2)
        src, dst = (t.numpy() for t in g.edges())
        ref = oracle.film_aggregate(x, gb, src, dst) + x
        out = m.film_mean_residual(x.to(cuda_device), gb.to(cuda_device), g.csr(cuda_device)).cpu()
        assert torch.equal(out, ref)
        csr = g.csr(cuda_device, allow_complete=False, allow_regular=False)  # general CSR kernel too
        assert torch.equal(m.film_mean_residual(x.to(cuda_device), gb.to(cuda_device), csr).cpu(), ref)


def test_mix_forward_and_grads(cuda_device):
    g = frames(2, 8, 12, 6, 6, seed=3)
    x = g.ndata["image"]
    torch.manual_seed(4)
    x0 = torch.randn_like(x)
    gb = torch.rand(g.num_edges(), 12, 2)
    src, dst = (t.numpy() for t in g.edges())
    alpha = 0.3
    xr, x0r, gbr = (t.clone().requires_grad_(True) for t in (x, x0, gb))
    ref = (1 - alpha) * oracle.film_aggregate(xr, gbr, src, dst) + alpha * x0r
    G = torch.randn_like(ref)
    ref.backward(G)
    xd, x0d, gbd = (t.to(cuda_device).requires_grad_(True) for t in (x, x0, gb))
    out = m.film_mean_mix(xd, gbd, g.csr(cuda_device), x0d, alpha)
    out.backward(G.to(cuda_device))
    # same operations; torch may round the Python-float scales differently from the fp32 epilogue's
    assert rel_err(out.detach().cpu().numpy(), ref.detach().numpy()) <= 1e-6
    for a, b in ((xd, xr), (x0d, x0r), (gbd, gbr)):
        assert rel_err(a.grad.cpu().numpy(), b.grad.numpy()) <= 1e-5


@pytest.mark.parametrize("dtype", [torch.float64, torch.bfloat16])
def test_backward_with_non_fp32_gamma_beta(cuda_device, dtype):
    """gb in another dtype is converted to fp32 for the backward exactly as for the forward."""
    g = frames(2, 8, 8, 4, 4, seed=9)
    x = g.ndata["image"].to(cuda_device)
    gb = torch.rand(g.num_edges(), 8, 2, device=cuda_device).to(dtype)
    G = torch.randn_like(x)
    res = []
    for t in (gb, gb.float()):
        xd = x.clone().requires_grad_(True)
        gd = t.clone().requires_grad_(True)
        m.film_mean(xd, gd, g.csr(cuda_device)).backward(G)
        assert gd.grad.dtype == t.dtype
        res.append((xd.grad, gd.grad.float()))
    assert torch.equal(res[0][0], res[1][0])
    assert rel_err(res[0][1].cpu().numpy(), res[1][1].cpu().numpy()) <= (1e-2 if dtype == torch.bfloat16 else 0)
