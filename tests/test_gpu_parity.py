"""GPU parity of the HIP path (through the C ABI) against the reference's golden vectors and the
CPU oracle.  Tolerance: the north-star contract, max|got-ref| / max|ref| <= 1e-5 (fp32).  Where the
reference's own CPU reduction is a sequential fp32 sum (every complete/k-NN graph whose per-node
C*H*W block is a multiple of 64 floats, edges listed in ascending source order, no multi-edges)
the forward is additionally required to be bit-identical.
"""
import numpy as np
import pytest
import torch

import mrp_gnn_amd as m
import stack_ref
import oracle
from conftest import golden_cases, load_golden, rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-5
PARAM_KEYS = ["layers.0.weight", "layers.0.bias", "layers.2.weight", "layers.2.bias"]


def graph_from(src, dst, bnn):
    bnn = [int(v) for v in bnn]
    goff = np.concatenate([[0], np.cumsum(bnn)])
    dst = np.asarray(dst, np.int64)
    bne = [int(((dst >= goff[i]) & (dst < goff[i + 1])).sum()) for i in range(len(bnn))]
    order = np.argsort(np.searchsorted(goff, dst, side="right"), kind="stable")
    assert np.array_equal(order, np.arange(len(dst))), "fixture edges must be grouped by graph"
    return m.RobotGraph(src, dst, num_nodes=int(goff[-1]), batch_num_nodes=bnn, batch_num_edges=bne)


def exact_expected(src, dst, c_times_p):
    if c_times_p % 64:
        return False
    pairs = list(zip(np.asarray(src).tolist(), np.asarray(dst).tolist()))
    if len(set(pairs)) != len(pairs):
        return False
    for v in set(np.asarray(dst).tolist()):
        s = [u for u, w in pairs if w == v]
        if s != sorted(s):
            return False
    return True


@pytest.mark.parametrize("name", golden_cases())
def test_golden_forward(cuda_device, name):
    z = load_golden(name)
    g = graph_from(z["src"], z["dst"], z["batch_num_nodes"])
    x = torch.from_numpy(z["x"]).to(cuda_device)
    gb = torch.from_numpy(z["gb"]).to(cuda_device)
    out = m.film_mean(x, gb, g.csr(cuda_device), str(z["mode"])).cpu().numpy()
    assert rel_err(out, z["out"]) <= TOL
    C, H, W = z["x"].shape[1:]
    if exact_expected(z["src"], z["dst"], C * H * W):
        assert np.array_equal(out, z["out"]), f"max abs diff {np.abs(out - z['out']).max()}"


@pytest.mark.parametrize("name", golden_cases())
def test_golden_backward(cuda_device, name):
    z = load_golden(name)
    g = graph_from(z["src"], z["dst"], z["batch_num_nodes"])
    x = torch.from_numpy(z["x"]).to(cuda_device).requires_grad_(True)
    gb = torch.from_numpy(z["gb"]).to(cuda_device).requires_grad_(True)
    out = m.film_mean(x, gb, g.csr(cuda_device), str(z["mode"]))
    out.backward(torch.from_numpy(z["grad_out"]).to(cuda_device))
    assert rel_err(x.grad.cpu().numpy(), z["dx"]) <= TOL
    if str(z["mode"]) == "copy_mean":
        assert gb.grad is None or float(gb.grad.abs().max()) == 0.0
    else:
        assert rel_err(gb.grad.cpu().numpy(), z["dgb"]) <= TOL


@pytest.mark.parametrize("name", golden_cases())
def test_golden_gcn_module(cuda_device, name):
    """The drop-in GCN module (edge encoder on the GPU + HIP aggregation) with the reference's
    parameters: forward output and the edge-encoder parameter gradients."""
    import types
    z = load_golden(name)
    C = z["x"].shape[1]
    g = graph_from(z["src"], z["dst"], z["batch_num_nodes"])
    g.ndata["image"] = torch.from_numpy(z["x"])
    g.edata["pose"] = torch.from_numpy(z["pose"])
    g = g.to(cuda_device)
    gcn = m.GCN(types.SimpleNamespace(feature_dim=C, gcn_mode=str(z["mode"])))
    gcn.load_state_dict({"edge_encoder." + k: torch.from_numpy(z["param." + k]) for k in PARAM_KEYS})
    gcn = gcn.to(cuda_device)
    out = gcn(g)
    assert rel_err(out.detach().cpu().numpy(), z["out"]) <= TOL
    if str(z["mode"]) != "copy_mean":  # copy_u has no trainable input here
        out.backward(torch.from_numpy(z["grad_out"]).to(cuda_device))
        # the encoder's parameter gradients contain GEMMs over E edges: judged against the same
        # gradients in float64, as accurate as the reference's own fp32 run (the fixture)
        g64 = _encoder_grads_f64(z)
        for k, p in gcn.edge_encoder.named_parameters():
            ok, errs = stack_ref.within(p.grad, torch.from_numpy(z["grad." + k]), g64[k])
            assert ok, (k, errs)


def _encoder_grads_f64(z):
    """Edge-encoder parameter gradients of a golden case's GCN forward in float64 (stack_ref's
    restatement of models.py:146-154 and update_all's mean)."""
    params = {"enc." + k: torch.from_numpy(z["param." + k]).double().requires_grad_(True) for k in PARAM_KEYS}
    x = torch.from_numpy(z["x"]).double()
    src = torch.from_numpy(z["src"]).long()
    dst = torch.from_numpy(z["dst"]).long()
    out = stack_ref.aggregate(x, stack_ref.edge_gb(params, "enc.", torch.from_numpy(z["pose"])), src, dst)
    out.backward(torch.from_numpy(z["grad_out"]).double())
    return {k: params["enc." + k].grad for k in PARAM_KEYS}


def random_case(n_per_graph, C, H, W, seed, knn=None, bnn=None):
    rng = np.random.RandomState(seed)
    graphs = []
    for n in (bnn or [n_per_graph]):
        poses = np.concatenate([rng.uniform(-10, 10, (n, 3)), rng.standard_normal((n, 4))], 1)
        graphs.append(m.frame_graph(poses.astype(np.float32), knn=knn if (knn is not None and knn < n) else None))
    g = m.batch(graphs)
    torch.manual_seed(seed)
    x = torch.randn(g.num_nodes(), C, H, W)
    gb = torch.rand(g.num_edges(), C, 2)
    return g, x, gb


@pytest.mark.parametrize("n", list(range(1, 17)))
@pytest.mark.parametrize("mode", ["film_mean", "film_sum", "copy_mean"])
def test_every_graph_size_vs_oracle(cuda_device, n, mode):
    g, x, gb = random_case(n, 24, 8, 8, seed=n, bnn=[n, n, n])
    src, dst = (t.numpy() for t in g.edges())
    ref = oracle.film_aggregate(x, gb, src, dst, mode).numpy()
    out = m.film_mean(x.to(cuda_device), gb.to(cuda_device), g.csr(cuda_device), mode).cpu().numpy()
    assert rel_err(out, ref) <= TOL
    assert np.array_equal(out, ref)  # complete graphs, C*P = 1536: sequential fp32 reduction


@pytest.mark.parametrize("n", [2, 5, 8, 9, 16])
@pytest.mark.parametrize("hw", [(4, 4), (3, 5), (7, 7), (32, 32), (1, 1)])
def test_backward_vs_oracle(cuda_device, n, hw):
    H, W = hw
    g, x, gb = random_case(n, 20, H, W, seed=100 + n, bnn=[n, max(1, n - 1)])
    src, dst = (t.numpy() for t in g.edges())
    G = torch.randn_like(x)
    dx_ref, dgb_ref = oracle.film_aggregate_grads(x, gb, src, dst, G)
    xd = x.to(cuda_device).requires_grad_(True)
    gbd = gb.to(cuda_device).requires_grad_(True)
    m.film_mean(xd, gbd, g.csr(cuda_device)).backward(G.to(cuda_device))
    assert rel_err(xd.grad.cpu().numpy(), dx_ref.numpy()) <= TOL
    assert rel_err(gbd.grad.cpu().numpy(), dgb_ref.numpy()) <= TOL


@pytest.mark.parametrize("n,bnn", [(3, [3, 3]), (8, [8, 8]), (8, [8, 5, 1]), (12, [12, 12])])
@pytest.mark.parametrize("hw", [(33, 33), (48, 48), (20, 20), (64, 64), (16, 16)])
def test_plane_split_geometries(cuda_device, n, bnn, hw):
    """Large and odd planes: the forward splits each plane over ceil(PV/lanes) workgroups (segments
    that do not divide the plane, 1-float slices at 33x33), the fused backward spans a plane over
    two waves (128 lanes) and adds their Gram partials."""
    H, W = hw
    g, x, gb = random_case(n, 6, H, W, seed=7 * n + H, bnn=bnn)
    src, dst = (t.numpy() for t in g.edges())
    ref = oracle.film_aggregate(x, gb, src, dst).numpy()
    out = m.film_mean(x.to(cuda_device), gb.to(cuda_device), g.csr(cuda_device)).cpu().numpy()
    assert rel_err(out, ref) <= TOL
    if exact_expected(src, dst, 6 * H * W):
        assert np.array_equal(out, ref)
    G = torch.randn_like(x)
    dx_ref, dgb_ref = oracle.film_aggregate_grads(x, gb, src, dst, G)
    xd = x.to(cuda_device).requires_grad_(True)
    gbd = gb.to(cuda_device).requires_grad_(True)
    m.film_mean(xd, gbd, g.csr(cuda_device)).backward(G.to(cuda_device))
    assert rel_err(xd.grad.cpu().numpy(), dx_ref.numpy()) <= TOL
    assert rel_err(gbd.grad.cpu().numpy(), dgb_ref.numpy()) <= TOL


@pytest.mark.parametrize("knn", [1, 4, 7])
def test_knn_graphs(cuda_device, knn):
    g, x, gb = random_case(16, 16, 16, 16, seed=knn, knn=knn, bnn=[16, 16, 12])
    src, dst = (t.numpy() for t in g.edges())
    ref = oracle.film_aggregate(x, gb, src, dst).numpy()
    out = m.film_mean(x.to(cuda_device), gb.to(cuda_device), g.csr(cuda_device)).cpu().numpy()
    assert np.array_equal(out, ref)
    G = torch.randn_like(x)
    dx_ref, dgb_ref = oracle.film_aggregate_grads(x, gb, src, dst, G)
    xd = x.to(cuda_device).requires_grad_(True)
    gbd = gb.to(cuda_device).requires_grad_(True)
    m.film_mean(xd, gbd, g.csr(cuda_device)).backward(G.to(cuda_device))
    assert rel_err(xd.grad.cpu().numpy(), dx_ref.numpy()) <= TOL
    assert rel_err(gbd.grad.cpu().numpy(), dgb_ref.numpy()) <= TOL


def test_ragged_batch_with_empty_and_edgeless_graphs(cuda_device):
    graphs = [m.complete_graph(5), m.RobotGraph([], [], num_nodes=0), m.RobotGraph([], [], num_nodes=3),
              m.graph(([0, 2, 2], [1, 1, 0]), num_nodes=4), m.complete_graph(1)]
    g = m.batch(graphs)
    torch.manual_seed(0)
    x = torch.randn(g.num_nodes(), 12, 5, 5)
    gb = torch.rand(g.num_edges(), 12, 2)
    src, dst = (t.numpy() for t in g.edges())
    ref = oracle.film_aggregate(x, gb, src, dst).numpy()
    out = m.film_mean(x.to(cuda_device), gb.to(cuda_device), g.csr(cuda_device)).cpu().numpy()
    assert rel_err(out, ref) <= TOL
    assert np.all(out[5:8] == 0) and np.all(out[10:] == 0) and np.all(out[11] == 0)


def test_zero_edges_whole_batch(cuda_device):
    g = m.batch([m.RobotGraph([], [], num_nodes=4), m.RobotGraph([], [], num_nodes=2)])
    x = torch.randn(6, 8, 4, 4, device=cuda_device, requires_grad=True)
    gb = torch.rand(0, 8, 2, device=cuda_device, requires_grad=True)
    out = m.film_mean(x, gb, g.csr(cuda_device))
    assert float(out.abs().max()) == 0.0
    out.sum().backward()
    assert float(x.grad.abs().max()) == 0.0


def test_non_neighbour_nonfinite_does_not_leak(cuda_device):
    # node 3 feeds nobody: its inf/nan must not reach any output (DGL never gathers it)
    g = m.graph(([0, 1, 2, 0], [1, 2, 0, 2]), num_nodes=4)
    x = torch.randn(4, 8, 4, 4)
    x[3] = float("inf")
    x[3, 0] = float("nan")
    gb = torch.rand(4, 8, 2)
    out = m.film_mean(x.to(cuda_device), gb.to(cuda_device), g.csr(cuda_device)).cpu()
    assert torch.isfinite(out).all()
    ref = oracle.film_aggregate(x, gb, *[t.numpy() for t in g.edges()])
    assert torch.equal(out, ref)


def test_multiedge_and_selfloop(cuda_device):
    g = m.graph(([0, 0, 1, 1, 2, 2, 2], [1, 1, 1, 0, 2, 0, 0]), num_nodes=3)
    torch.manual_seed(3)
    x = torch.randn(3, 8, 6, 6)
    gb = torch.rand(7, 8, 2)
    src, dst = (t.numpy() for t in g.edges())
    ref = oracle.film_aggregate(x, gb, src, dst).numpy()
    out = m.film_mean(x.to(cuda_device), gb.to(cuda_device), g.csr(cuda_device)).cpu().numpy()
    assert rel_err(out, ref) <= TOL
    G = torch.randn_like(x)
    dx_ref, dgb_ref = oracle.film_aggregate_grads(x, gb, src, dst, G)
    xd = x.to(cuda_device).requires_grad_(True)
    gbd = gb.to(cuda_device).requires_grad_(True)
    m.film_mean(xd, gbd, g.csr(cuda_device)).backward(G.to(cuda_device))
    assert rel_err(xd.grad.cpu().numpy(), dx_ref.numpy()) <= TOL
    assert rel_err(gbd.grad.cpu().numpy(), dgb_ref.numpy()) <= TOL


def test_strided_input_and_cat_buffer_output(cuda_device):
    g, x, gb = random_case(8, 32, 8, 8, seed=7, bnn=[8, 8])
    src, dst = (t.numpy() for t in g.edges())
    ref = oracle.film_aggregate(x, gb, src, dst)
    big = torch.randn(x.shape[0], 64, 8, 8, device=cuda_device)
    big[:, 16:48] = x.to(cuda_device)
    xin = big[:, 16:48]  # node stride 64*P, no copy needed
    cat = torch.zeros(x.shape[0], 64, 8, 8, device=cuda_device)
    cat[:, :32] = xin
    m.film_mean_forward_into(xin, gb.to(cuda_device), g.csr(cuda_device), 0, cat[:, 32:])
    assert torch.equal(cat[:, 32:].cpu(), ref)
    assert torch.equal(cat[:, :32].cpu(), x)


def test_gcn_block_stack_backward(cuda_device):
    """gcn1 -> cat -> conv1 -> gcn2 -> cat -> conv2 (models.py:180-189): gradients flow through
    strided cat-slice grad_outs into the kernels; checked against the oracle-built stack."""
    import types
    C = 16
    o = types.SimpleNamespace(feature_dim=C, compress_gcn=True, multi_gcn=True)
    torch.manual_seed(0)
    block = m.GCNBlock(o)
    g, x, _ = random_case(5, C, 8, 8, seed=11, bnn=[5, 5, 5])
    gd = g.to(cuda_device)
    blk = block.to(cuda_device)
    xd = x.to(cuda_device).requires_grad_(True)
    out = blk(gd, xd)
    out.square().sum().backward()
    # oracle stack on CPU with the same parameters
    src, dst = (t.numpy() for t in g.edges())
    ref_block = m.GCNBlock(o)
    ref_block.load_state_dict({k: v.cpu() for k, v in blk.state_dict().items()})
    xr = x.clone().requires_grad_(True)

    def ref_gcn(gcn, h):
        params = dict(gcn.edge_encoder.named_parameters())
        return oracle.film_aggregate(h, oracle.edge_encoder_forward(params, g.edata["pose"]), src, dst)

    h = torch.cat((xr, ref_gcn(ref_block.gcn1, xr)), 1)
    h = ref_block.conv1(h)
    h = ref_block.conv2(torch.cat((h, ref_gcn(ref_block.gcn2, h)), 1))
    h.square().sum().backward()
    # the same stack in float64 (tests/stack_ref.py): the yardstick for the GEMM-containing parts,
    # whose fp32 summation order differs between any two implementations
    params = {k: v.detach().cpu() for k, v in blk.named_parameters()}
    gsrc, gdst = torch.as_tensor(src).long(), torch.as_tensor(dst).long()
    out64, dx64, dp64 = stack_ref.run(params, x, g.edata["pose"], gsrc, gdst, None, torch.float64, layers=2,
                                      loss="square_sum")
    for name, ours, f32, f64 in (("out", out, h, out64), ("dx", xd.grad, xr.grad, dx64)):
        ok, errs = stack_ref.within(ours.cpu(), f32, f64)
        assert ok, (name, errs)
    for (k, p), (_, q) in zip(blk.named_parameters(), ref_block.named_parameters()):
        ok, errs = stack_ref.within(p.grad.cpu(), q.grad, dp64[k])
        assert ok, (k, errs)


def test_deterministic(cuda_device):
    g, x, gb = random_case(8, 64, 16, 16, seed=5, bnn=[8] * 4)
    xd = x.to(cuda_device).requires_grad_(True)
    gbd = gb.to(cuda_device).requires_grad_(True)
    G = torch.randn_like(xd)
    res = []
    for _ in range(2):
        xd.grad = None
        gbd.grad = None
        out = m.film_mean(xd, gbd, g.csr(cuda_device))
        out.backward(G)
        res.append((out.detach().clone(), xd.grad.clone(), gbd.grad.clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def torch_reference_gpu(x, gb, src, dst, num_nodes):
    """fp32 torch restatement on the GPU (gather -> FiLM message -> scatter-mean), for sizes the
    CPU oracle is too slow for."""
    src = torch.as_tensor(src, device=x.device)
    dst = torch.as_tensor(dst, device=x.device)
    msg = gb[:, :, 0, None, None] * x.index_select(0, src) + gb[:, :, 1, None, None]
    acc = torch.zeros_like(x).index_add_(0, dst, msg)
    deg = torch.bincount(dst, minlength=num_nodes).clamp_min(1).to(x.dtype)
    return acc / deg[:, None, None, None]


def test_north_star_size_vs_torch_reference(cuda_device):
    """B=32, N=8, C=512, 32x32 (the benchmark workload): forward and backward vs a torch fp32
    restatement of the UDF path on the GPU, plus a size-independent property (linearity in x
    with beta = 0)."""
    B, N, C, H, W = 32, 8, 512, 32, 32
    g, _, _ = random_case(N, 1, 1, 1, seed=0, bnn=[N] * B)
    torch.manual_seed(0)
    x = torch.randn(B * N, C, H, W, device=cuda_device, requires_grad=True)
    gb = torch.rand(g.num_edges(), C, 2, device=cuda_device, requires_grad=True)
    csr = g.csr(cuda_device)
    src, dst = (t.numpy() for t in g.edges())
    out = m.film_mean(x, gb, csr)
    G = torch.randn_like(out)
    out.backward(G)
    with torch.no_grad():
        ref = torch_reference_gpu(x, gb, src, dst, B * N)
        assert float((out - ref).abs().max() / ref.abs().max()) <= TOL
    xr = x.detach().clone().requires_grad_(True)
    gbr = gb.detach().clone().requires_grad_(True)
    torch_reference_gpu(xr, gbr, src, dst, B * N).backward(G)
    assert float((x.grad - xr.grad).abs().max() / xr.grad.abs().max()) <= TOL
    assert float((gb.grad - gbr.grad).abs().max() / gbr.grad.abs().max()) <= TOL
    del xr, gbr, ref
    with torch.no_grad():
        gb0 = gb.detach().clone()
        gb0[..., 1] = 0
        a = m.film_mean(x.detach(), gb0, csr)
        b = m.film_mean(2.0 * x.detach(), gb0, csr)
        assert torch.equal(2.0 * a, b)  # scaling by 2 is exact in fp32


@pytest.mark.parametrize("n", [2, 3, 5, 8, 11, 16])
@pytest.mark.parametrize("hw", [(8, 8), (3, 5)])
def test_complete_fast_path_equals_csr_path(cuda_device, n, hw):
    """The COMPLETE kernels (arithmetic edge ids) and the general CSR kernels agree exactly on
    the forward and to rounding on the backward."""
    g, x, gb = random_case(n, 12, hw[0], hw[1], seed=200 + n, bnn=[n] * 3)
    assert g.is_complete()
    fast, slow = g.csr(cuda_device), g.csr(cuda_device, allow_complete=False, allow_regular=False)
    assert fast.graph_kind == 1 and slow.graph_kind == 0
    G = torch.randn_like(x).to(cuda_device)
    res = []
    for csr in (fast, slow):
        xd = x.to(cuda_device).requires_grad_(True)
        gbd = gb.to(cuda_device).requires_grad_(True)
        out = m.film_mean(xd, gbd, csr)
        out.backward(G)
        res.append((out.detach().cpu(), xd.grad.cpu(), gbd.grad.cpu()))
    assert torch.equal(res[0][0], res[1][0])
    assert rel_err(res[0][1].numpy(), res[1][1].numpy()) <= 1e-6
    assert rel_err(res[0][2].numpy(), res[1][2].numpy()) <= 1e-6


def regular_graph(n, k, rng, multi=False):
    """Every node has exactly k in-edges from random sources (repeats allowed when ``multi``)."""
    src, dst = [], []
    for v in range(n):
        us = rng.randint(0, n, k) if multi else rng.permutation(n)[:k]
        src += [int(u) for u in us]
        dst += [v] * k
    return m.graph((src, dst), num_nodes=n)


@pytest.mark.parametrize("n,k", [(9, 1), (10, 3), (12, 4), (16, 4), (16, 5), (13, 8), (16, 8)])
@pytest.mark.parametrize("hw", [(8, 8), (3, 5)])
@pytest.mark.parametrize("multi", [False, True])
def test_regular_backward_equals_csr_path(cuda_device, n, k, hw, multi):
    """The per-edge-slot kernels of regular graphs (film_fwd_regular, film_bwd_regular) against the
    oracle and the general CSR kernels, for mixed graph sizes, unsorted in-edges, multi-edges /
    self-loops and both slice widths.  The per-slot forward sums each mailbox in edge-id order, as
    DGL does, so it is bit-identical to the oracle wherever the oracle's sum is sequential; the dense
    CSR kernel sums by ascending source (and merges multi-edges), so it agrees to rounding."""
    rng = np.random.RandomState(n * 31 + k)
    small = max(k, n - 3)
    g = m.batch([regular_graph(n, k, rng, multi), regular_graph(small, k, rng, multi), regular_graph(n, k, rng, multi)])
    assert g.in_degree_k() == k
    fast, slow = g.csr(cuda_device), g.csr(cuda_device, allow_regular=False)
    assert fast.graph_kind == m.graph_regular(k) and slow.graph_kind == 0
    torch.manual_seed(n + k)
    x = torch.randn(g.num_nodes(), 12, *hw)
    z = torch.randn(g.num_edges(), 12, 2)
    G = torch.randn_like(x)
    src, dst = (t.numpy() for t in g.edges())
    dx_ref, dgb_ref = oracle.film_aggregate_grads(x, torch.sigmoid(z), src, dst, G)
    res = []
    for csr in (fast, slow):
        xd = x.to(cuda_device).requires_grad_(True)
        zd = z.to(cuda_device).requires_grad_(True)
        out = m.film_mean_cat(xd, zd, csr, logits=True)
        out.backward(torch.cat((G, G), 1).to(cuda_device))
        res.append((out.detach().cpu(), xd.grad.cpu(), zd.grad.cpu()))
    out_ref = oracle.film_aggregate(x, torch.sigmoid(z), src, dst)
    assert torch.equal(res[0][0][:, :12], x) and torch.equal(res[1][0][:, :12], x)
    if 12 * hw[0] * hw[1] % 64 == 0:  # the oracle's (CPU torch) mailbox mean is a sequential sum
        # gamma/beta given post-sigmoid (the device sigmoid's expf rounds differently from torch's)
        exact = m.film_mean(x.to(cuda_device), torch.sigmoid(z).to(cuda_device), fast).cpu()
        assert torch.equal(exact, out_ref)
    assert rel_err(res[0][0][:, 12:].numpy(), out_ref.numpy()) <= TOL
    assert rel_err(res[1][0][:, 12:].numpy(), out_ref.numpy()) <= TOL
    assert rel_err(res[0][1].numpy(), (dx_ref + G).numpy()) <= TOL
    dz_ref = dgb_ref * torch.sigmoid(z) * (1 - torch.sigmoid(z))
    assert rel_err(res[0][2].numpy(), dz_ref.numpy()) <= TOL
    assert rel_err(res[0][1].numpy(), res[1][1].numpy()) <= 1e-6
    assert rel_err(res[0][2].numpy(), res[1][2].numpy()) <= 1e-6


@pytest.mark.parametrize("complete", [True, False])
@pytest.mark.parametrize("bnn,hw,knn", [([8, 8, 8], (8, 8), None), ([8, 5, 3, 1], (3, 5), None),
                                        ([12, 16, 9], (4, 4), 3), ([16, 7], (1, 1), None)])
def test_cat_fused_forward_backward(cuda_device, complete, bnn, hw, knn):
    """film_mean_cat == torch.cat((x, film_mean(x)), 1), forward exactly (the kernel writes both
    halves: mrp_film_mean_cat_fwd), backward (incl. the grad_x_base accumulation of the
    concatenation's first half) to rounding; ragged, k-NN, odd and 1x1 planes."""
    g, x, gb = random_case(max(bnn), 16, hw[0], hw[1], seed=31, bnn=bnn, knn=knn)
    csr = g.csr(cuda_device, allow_complete=complete)
    x1 = x.to(cuda_device).requires_grad_(True)
    x2 = x.to(cuda_device).requires_grad_(True)
    z1 = gb.to(cuda_device).requires_grad_(True)
    z2 = gb.to(cuda_device).requires_grad_(True)
    a = m.film_mean_cat(x1, z1, csr, logits=True)
    b = torch.cat((x2, m.film_mean(x2, z2, csr, logits=True)), 1)
    assert torch.equal(a, b)
    G = torch.randn_like(a)
    a.backward(G)
    b.backward(G)
    assert rel_err(x1.grad.cpu().numpy(), x2.grad.cpu().numpy()) <= 1e-6
    assert rel_err(z1.grad.cpu().numpy(), z2.grad.cpu().numpy()) <= 1e-6


def test_cat_forward_strided_source(cuda_device):
    """x read through a node stride (a channel slice of a wider buffer), cat buffer written whole."""
    g, x, gb = random_case(6, 8, 4, 4, seed=5, bnn=[6, 6])
    wide = torch.randn(x.shape[0], 24, 4, 4)
    wide[:, 4:12] = x
    xd = wide.to(cuda_device)[:, 4:12]
    assert not xd.is_contiguous()
    buf = torch.full((x.shape[0], 16, 4, 4), float("nan"), device=cuda_device)
    m.film_mean_cat_forward_into(xd, gb.to(cuda_device), g.csr(cuda_device), 0, buf)
    ref = torch.cat((x, oracle.film_aggregate(x, gb, *[t.numpy() for t in g.edges()])), 1)
    assert torch.equal(buf.cpu(), ref)


@pytest.mark.parametrize("n,C,hw,knn", [(8, 23, (8, 8), None), (5, 16, (16, 16), None), (12, 9, (8, 8), None),
                                         (16, 13, (8, 8), 4), (11, 6, (16, 16), 6)])
@pytest.mark.parametrize("combine", ["cat", "residual"])
def test_mfma_backward_matches_valu_kernels(cuda_device, n, C, hw, knn, combine):
    """film_bwd_mfma (Gram and grad_x on the matrix cores; the default for k-NN and complete graphs of
    9..16 nodes; graphs of <= 8 nodes run the VALU kernel either way) against the VALU kernels (film_bwd_fused / film_bwd_regular) and the
    oracle: odd channel counts (a channel pair with one channel past C), graphs of 5..16 nodes, the
    cat backward's grad_x base and the residual epilogue's self term."""
    lib = m.load_library()
    g, x, gb = random_case(n, C, hw[0], hw[1], seed=n * 7 + C, knn=knn, bnn=[n, n, n])
    csr = g.csr(cuda_device)
    op = m.film_mean_cat if combine == "cat" else m.film_mean_residual
    G = torch.randn(op(x.to(cuda_device), gb.to(cuda_device), csr, logits=True).shape)
    res = []
    try:
        for on in (0, 1):
            assert lib.mrp_tuning_set(b"bwd_regular_mfma", on) == 0
            assert lib.mrp_tuning_set(b"bwd_complete_mfma", on) == 0
            xd = x.to(cuda_device).requires_grad_(True)
            zd = gb.to(cuda_device).requires_grad_(True)
            op(xd, zd, csr, logits=True).backward(G.to(cuda_device))
            res.append((xd.grad.cpu(), zd.grad.cpu()))
    finally:
        lib.mrp_tuning_set(b"reset", 0)
    assert rel_err(res[1][0].numpy(), res[0][0].numpy()) <= 1e-6
    assert rel_err(res[1][1].numpy(), res[0][1].numpy()) <= 1e-6
    src, dst = (t.numpy() for t in g.edges())
    dx_ref, dgb_ref = oracle.film_aggregate_grads(x, torch.sigmoid(gb), src, dst, G[:, C:] if combine == "cat" else G)
    dx_ref = dx_ref + (G[:, :C] if combine == "cat" else G)
    dz_ref = dgb_ref * torch.sigmoid(gb) * (1 - torch.sigmoid(gb))
    assert rel_err(res[1][0].numpy(), dx_ref.numpy()) <= TOL
    assert rel_err(res[1][1].numpy(), dz_ref.numpy()) <= TOL


@pytest.mark.parametrize("n,k,C,hw", [(5, 1, 1, (4, 4)), (16, 3, 1, (2, 2)), (9, 8, 1, (4, 4)), (16, 8, 2, (1, 4)),
                                      (7, 5, 1, (8, 8)), (12, 2, 3, (2, 6))])
def test_knn_narrow_workgroups(cuda_device, n, k, C, hw):
    """k-NN graphs whose workgroups have fewer threads than the graph has destinations (one or two
    channels of a plane of a few slices: 4-8 threads): every destination's packed slot sources must
    still be written (found by tests/test_gpu_properties.py: n = 5, k = 1, C = 1, 4 x 4)."""
    H, W = hw
    g, x, gb = random_case(n, C, H, W, seed=31 * n + k, knn=k, bnn=[n, n])
    assert g.in_degree_k() == k
    src, dst = (t.numpy() for t in g.edges())
    ref = oracle.film_aggregate(x, gb, src, dst).numpy()
    out = m.film_mean(x.to(cuda_device), gb.to(cuda_device), g.csr(cuda_device)).cpu().numpy()
    assert rel_err(out, ref) <= TOL
    G = torch.randn_like(x)
    dx_ref, dgb_ref = oracle.film_aggregate_grads(x, gb, src, dst, G)
    xd = x.to(cuda_device).requires_grad_(True)
    gbd = gb.to(cuda_device).requires_grad_(True)
    m.film_mean(xd, gbd, g.csr(cuda_device)).backward(G.to(cuda_device))
    assert rel_err(xd.grad.cpu().numpy(), dx_ref.numpy()) <= TOL
    assert rel_err(gbd.grad.cpu().numpy(), dgb_ref.numpy()) <= TOL
