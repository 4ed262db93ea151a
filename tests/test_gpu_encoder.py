"""GPU: the edge encoder path (HIP hidden layer + matrix-core logits GEMM + sigmoid fused into the
aggregation) against the reference's torch layers and the golden fixtures."""
import ctypes

import numpy as np
import pytest
import torch

import mrp_gnn_amd as m
from conftest import golden_cases, load_golden, rel_err
import stack_ref

pytestmark = pytest.mark.gpu
PARAM_KEYS = ["layers.0.weight", "layers.0.bias", "layers.2.weight", "layers.2.bias"]


@pytest.mark.parametrize("name", [n for n in golden_cases() if "copyu" not in n])
def test_encoder_matches_reference_fixture(cuda_device, name):
    z = load_golden(name)
    C = z["x"].shape[1]
    enc = m.edge_encoder([C, C])
    enc.load_state_dict({k: torch.from_numpy(z["param." + k]) for k in PARAM_KEYS})
    enc = enc.to(cuda_device)
    gb = enc.film_params(torch.from_numpy(z["pose"]).to(cuda_device))
    assert rel_err(gb.detach().cpu().numpy(), z["gb"]) <= 1e-5


@pytest.mark.parametrize("E,C", [(1, 1), (7, 3), (96, 64), (1792, 512), (100, 130), (33, 1281)])
def test_hidden_kernel_vs_torch(cuda_device, E, C):
    torch.manual_seed(E + C)
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 5).to(cuda_device)
    l1 = enc.layers[0]
    h = m.encoder.hidden_forward(pose, l1.weight, l1.bias)
    ref = torch.relu(l1(pose))
    assert float((h - ref).detach().abs().max()) <= 1e-5 * max(1.0, float(ref.detach().abs().max()))
    # the full logits path and its backward vs torch autograd through the reference layers
    g = torch.randn(E, 2 * C, device=cuda_device)
    pr = pose.clone().requires_grad_(True)
    pf = pose.clone().requires_grad_(True)
    enc.zero_grad()
    (enc.layers[2](torch.relu(enc.layers[0](pr))) * g).sum().backward()
    ref_grads = [p.grad.clone() for p in enc.parameters()] + [pr.grad.clone()]
    enc.zero_grad()
    zl = enc.logits(pf).reshape(E, 2 * C)
    assert rel_err(zl.detach().cpu().numpy(), enc.layers[2](torch.relu(enc.layers[0](pose))).detach().cpu().numpy()) <= 1e-5
    (zl * g).sum().backward()
    got_grads = [p.grad.clone() for p in enc.parameters()] + [pf.grad.clone()]
    # the same backward in float64: the yardstick (both fp32 paths sum E or C terms in GEMMs whose
    # order differs; each must be as accurate as torch's fp32 autograd of the reference layers)
    e64 = [p.detach().double().requires_grad_(True) for p in enc.parameters()]
    p64 = pose.double().requires_grad_(True)
    z64 = torch.nn.functional.linear(torch.relu(torch.nn.functional.linear(p64, e64[0], e64[1])), e64[2], e64[3])
    (z64 * g.double()).sum().backward()
    f64_grads = [t.grad for t in e64] + [p64.grad]
    for a, b, c in zip(got_grads, ref_grads, f64_grads):
        ok, errs = stack_ref.within(a, b, c)
        assert ok, errs


@pytest.mark.parametrize("complete", [True, False])
@pytest.mark.parametrize("n", [3, 8, 12])
def test_logits_fusion_equals_explicit_sigmoid(cuda_device, complete, n):
    """film_mean(x, z, logits=True) == film_mean(x, sigmoid(z)) and its gradient w.r.t. z equals
    the chain rule through torch.sigmoid."""
    rng = np.random.RandomState(n)
    graphs = [m.frame_graph(np.concatenate([rng.uniform(-5, 5, (n, 3)), rng.randn(n, 4)], 1)) for _ in range(3)]
    g = m.batch(graphs)
    csr = g.csr(cuda_device, allow_complete=complete)
    torch.manual_seed(n)
    x = torch.randn(g.num_nodes(), 16, 8, 8, device=cuda_device)
    zl = (torch.randn(g.num_edges(), 16, 2) * 3).to(cuda_device)
    G = torch.randn_like(x)
    z1 = zl.clone().requires_grad_(True)
    z2 = zl.clone().requires_grad_(True)
    a = m.film_mean(x, z1, csr, logits=True)
    b = m.film_mean(x, torch.sigmoid(z2), csr)
    assert rel_err(a.detach().cpu().numpy(), b.detach().cpu().numpy()) <= 1e-6
    a.backward(G)
    b.backward(G)
    assert rel_err(z1.grad.cpu().numpy(), z2.grad.cpu().numpy()) <= 1e-5


@pytest.mark.parametrize("E,C", [(1, 32), (63, 64), (65, 96), (1792, 512), (300, 1024), (129, 1280)])
def test_logits_kernel_vs_float64(cuda_device, E, C):
    """mrp_edge_logits_fwd (fp32 MFMA) against torch fp32 and the float64 yardstick: ragged edge counts
    (partial 64-row tiles), C % 32 == 0 from one k-stage to 40."""
    torch.manual_seed(E * 7 + C)
    h = torch.relu(torch.randn(E, C, device=cuda_device))
    w2 = torch.randn(2 * C, C, device=cuda_device) / C ** 0.5
    b2 = torch.randn(2 * C, device=cuda_device)
    z = m.encoder.logits_forward(h, w2, b2)
    ref = torch.addmm(b2, h, w2.t())
    z64 = torch.addmm(b2.double(), h.double(), w2.double().t())
    ok, errs = stack_ref.within(z, ref, z64)
    assert ok, errs


def test_logits_kernel_declines_unsupported_shapes(cuda_device):
    """C % 32 != 0: the ABI says NotSupported (and logits_forward, on the comparison paths only, takes
    the library GEMM instead; the product path pads, tests/test_gpu_encoder_train.py)."""
    h = torch.randn(10, 48, device=cuda_device)
    w2 = torch.randn(96, 48, device=cuda_device)
    b2 = torch.randn(96, device=cuda_device)
    z = torch.empty(10, 96, device=cuda_device)
    lib = m.load_library()
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    code = lib.mrp_edge_logits_fwd(p(h), 10, 48, p(w2), p(b2), p(z), ctypes.c_void_p(0))
    assert code == m._lib.HIP_ERROR_NOT_SUPPORTED
    assert torch.allclose(m.encoder.logits_forward(h, w2, b2), torch.addmm(b2, h, w2.t()), rtol=1e-5, atol=1e-5)


def _f64_logits(enc, pose):
    with torch.no_grad():
        t32 = enc.layers[2](torch.relu(enc.layers[0](pose)))
        p64 = [t.detach().double() for t in enc.parameters()]
        z64 = torch.nn.functional.linear(torch.relu(torch.nn.functional.linear(pose.double(), p64[0], p64[1])),
                                         p64[2], p64[3])
    return t32, z64


def test_edge_logits_takes_fused_kernel_only_without_grad(cuda_device):
    """edge_logits: inference -> the one-launch split-bf16 kernel; with gradients wanted -> the split
    training path (E % 32 == 0 and C % 32 == 0) or its zero-padded form (else); C = 48 runs both on
    padded weights.  All within the float64 yardstick of the reference layers."""
    torch.manual_seed(0)
    for C, E, path in ((64, 96, "split_train"), (64, 100, "split_padded"), (48, 100, "split_padded")):
        enc = m.edge_encoder([C, C]).to(cuda_device)
        pose = torch.randn(E, 9, device=cuda_device)
        n_split, n_train = m.encoder.PATH_COUNTS["split"], m.encoder.PATH_COUNTS[path]
        with torch.no_grad():
            z0 = m.encoder.edge_logits(enc.layers, pose)
        z1 = m.encoder.edge_logits(enc.layers, pose)
        assert m.encoder.PATH_COUNTS["split"] == n_split + 1 and m.encoder.PATH_COUNTS[path] == n_train + 1
        assert z1.requires_grad and not z0.requires_grad
        t32, z64 = _f64_logits(enc, pose)
        for z in (z0, z1.detach()):
            ok, errs = stack_ref.within(z, t32, z64)
            assert ok, errs


@pytest.mark.parametrize("E,C", [(1, 32), (31, 32), (33, 64), (127, 96), (129, 128), (1792, 512), (448, 2048),
                                 (300, 1024)])
@pytest.mark.parametrize("v", [1, 3, -1])
def test_split_encoder_vs_float64(cuda_device, E, C, v):
    """mrp_edge_encoder_fwd_split (three-way bf16 split, six partial products) in every form the
    library builds — the hidden layer computed once per workgroup of 4 (v 1) or 8 (v 3) waves; -1: the
    per-shape default — is as accurate as an fp32 evaluation of the reference layers (float64
    yardstick), for ragged edge counts (partial 32-edge blocks and workgroups), C from one hidden block
    to 64, column groups past 2C, poses of robot-scale magnitudes."""
    torch.manual_seed(E * 3 + C)
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 8).to(cuda_device)
    lib = m.load_library()
    assert lib.mrp_tuning_set(b"edge_split_v", v) == 0
    try:
        with torch.no_grad():
            z = m.encoder.encoder_forward_split(pose, enc.layers[0], enc.layers[2])
    finally:
        lib.mrp_tuning_set(b"reset", 0)
    assert z is not None and z.shape == (E, 2 * C)
    t32, z64 = _f64_logits(enc, pose)
    ok, errs = stack_ref.within(z, t32, z64)
    assert ok, errs


def test_split_encoder_repacks_after_weight_update(cuda_device):
    """The packed weight image follows optimizer updates (in-place, version-bumping) and is rebuilt
    after clear_packed_weights() for writes through .data; a NULL bias b2 is accepted."""
    torch.manual_seed(5)
    C, E = 64, 200
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 4).to(cuda_device)
    l1, l2 = enc.layers[0], enc.layers[2]
    with torch.no_grad():
        z_a = m.encoder.encoder_forward_split(pose, l1, l2)
        for p in enc.parameters():
            p.mul_(1.5)  # what an optimizer step does: version bump
        z_b = m.encoder.encoder_forward_split(pose, l1, l2)
    t32, z64 = _f64_logits(enc, pose)
    assert not torch.equal(z_a, z_b)
    ok, errs = stack_ref.within(z_b, t32, z64)
    assert ok, errs
    l2.weight.data.mul_(-1.0)  # no version bump: needs the explicit clear
    m.encoder.clear_packed_weights()
    with torch.no_grad():
        z_c = m.encoder.encoder_forward_split(pose, l1, l2)
    t32, z64 = _f64_logits(enc, pose)
    ok, errs = stack_ref.within(z_c, t32, z64)
    assert ok, errs
    img = m.encoder.packed_weights(l1, l2)
    zn = torch.empty(E, 2 * C, device=cuda_device)
    lib = m.load_library()
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    assert lib.mrp_edge_encoder_fwd_split(p(pose), p(img), None, E, C, p(zn), ctypes.c_void_p(0)) == 0
    torch.cuda.synchronize()
    assert rel_err((zn + l2.bias).detach().cpu().numpy(), z_c.cpu().numpy()) <= 1e-6
    assert lib.mrp_edge_encoder_pack_bytes(48) == 0
