"""The one-launch no-grad GCN layer (``mrp_gcn_fwd_fused``, ``csrc/gcn_fused.hip``): the encoder's
logits produced by the first workgroups of the aggregation's own grid and handed off per graph.

Parity bar: bit-identical to the two-launch path (``mrp_edge_encoder_fwd_split`` + ``film_fwd``) —
the same products in the same order — for the logits and the aggregate, at every complete-graph size
it serves (2..8 nodes), several planes and channel counts, the headline workload, repeated launches
(the hand-off's race guard), every producer count including none (every item then produced by the
aggregation workgroups' fallback path); plus the headline against the reference's op sequence in
float64 (``stack_ref``, the fp32 yardstick) and the reference's own fixture at 1e-5.
Reference: ``dgl/model/models.py:142-155,207-226``."""
import types

import numpy as np
import pytest
import torch

import mrp_gnn_amd as m
import stack_ref
from conftest import load_golden, rel_err
from test_gpu_parity import PARAM_KEYS, graph_from

pytestmark = pytest.mark.gpu


def complete_batch(B, N, C, H, W, seed, device):
    rng = np.random.RandomState(seed)
    gs = []
    for _ in range(B):
        t = rng.uniform(-10, 10, size=(N, 3))
        q = rng.standard_normal((N, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        gs.append(m.frame_graph(np.concatenate([t, q], 1).astype(np.float32)))
    g = m.batch(gs)
    gen = torch.Generator().manual_seed(seed)
    g.ndata["image"] = torch.randn(B * N, C, H, W, generator=gen)
    return g.to(device)


def layer(C, seed, device):
    torch.manual_seed(seed)
    return m.GCN(types.SimpleNamespace(feature_dim=C)).to(device)


def two_launch(gcn, g, x):
    m.fused.set_fused_forward(False)
    try:
        with torch.no_grad():
            z = m.encoder.edge_logits(gcn.edge_encoder.layers, g.edata["pose"])
            out = gcn(g, x)
    finally:
        m.fused.set_fused_forward(True)
    return z, out


def fused(gcn, g, x):
    E, C = g.num_edges(), x.shape[1]
    z = torch.empty((E, 2 * C), device=x.device)
    enc = gcn.edge_encoder.layers
    before = m.encoder.PATH_COUNTS["fused"]
    with torch.no_grad():
        out = m.fused.gcn_forward_fused(x, g.edata["pose"], g.csr(x.device), enc[0], enc[2], z_out=z)
    assert out is not None, "the fused launch declined a shape it serves"
    assert m.encoder.PATH_COUNTS["fused"] == before + 1
    assert m.fused.error_word(x.device) == 0
    return z, out


@pytest.mark.parametrize("N", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("C,H", [(32, 8), (64, 8), (96, 16), (128, 32), (192, 16)])
def test_fused_bit_identical_to_two_launches(cuda_device, N, C, H):
    g = complete_batch(5, N, C, H, H, seed=N * 100 + C + H, device=cuda_device)
    gcn = layer(C, seed=N + C, device=cuda_device)
    x = g.ndata["image"]
    z2, out2 = two_launch(gcn, g, x)
    z1, out1 = fused(gcn, g, x)
    assert torch.equal(z1, z2)
    assert torch.equal(out1, out2)


def test_gcn_forward_takes_the_fused_launch(cuda_device):
    """GCN.forward under no_grad runs the one launch (the benchmarked step) and matches it bit for
    bit; with a gradient wanted it runs the training path."""
    g = complete_batch(4, 8, 128, 8, 8, seed=3, device=cuda_device)
    gcn = layer(128, seed=1, device=cuda_device)
    x = g.ndata["image"]
    before = m.encoder.PATH_COUNTS["fused"]
    with torch.no_grad():
        out = gcn(g, x)
    assert m.encoder.PATH_COUNTS["fused"] == before + 1
    _, ref = two_launch(gcn, g, x)
    assert torch.equal(out, ref)
    out_t = gcn(g, x.clone().requires_grad_(True))
    assert m.encoder.PATH_COUNTS["fused"] == before + 1  # training: not the fused launch
    assert torch.equal(out_t.detach(), ref)


def test_fused_headline_repeated_and_vs_float64(cuda_device):
    """The headline workload (B = 32, N = 8, C = 512, 32 x 32): 20 launches back to back, each
    bit-identical to the two-launch path (a hand-off read too early would differ), and the result
    against the reference's op sequence in float64 with the fp32 yardstick."""
    C = 512
    g = complete_batch(32, 8, C, 32, 32, seed=11, device=cuda_device)
    gcn = layer(C, seed=0, device=cuda_device)
    x = g.ndata["image"]
    z2, out2 = two_launch(gcn, g, x)
    for _ in range(20):
        z1, out1 = fused(gcn, g, x)
        assert torch.equal(z1, z2)
        assert torch.equal(out1, out2)
    params = {"enc." + k: v.detach() for k, v in gcn.edge_encoder.named_parameters()}
    src, dst = (t.to(cuda_device).long() for t in g.edges())
    pose = g.edata["pose"]
    with torch.no_grad():
        f32 = stack_ref.aggregate(x, stack_ref.edge_gb(params, "enc.", pose), src, dst)
        p64 = {k: v.double() for k, v in params.items()}
        f64 = stack_ref.aggregate(x.double(), stack_ref.edge_gb(p64, "enc.", pose.double()), src, dst)
    ok, errs = stack_ref.within(out1, f32, f64)
    assert ok, errs


@pytest.mark.parametrize("nprod", [0, 1, 7, 64, 512, 4096])
def test_fused_any_producer_count(cuda_device, nprod):
    """Every producer count gives the same bits; 0 producers = every item produced by the aggregation
    workgroups themselves (claim after a bounded wait: the path that keeps the grid live under any
    dispatch order)."""
    lib = m.load_library()
    g = complete_batch(6, 8, 128, 16, 16, seed=21, device=cuda_device)
    gcn = layer(128, seed=2, device=cuda_device)
    x = g.ndata["image"]
    z2, out2 = two_launch(gcn, g, x)
    try:
        assert lib.mrp_tuning_set(b"fused_producers", nprod) == 0
        for _ in range(3):
            z1, out1 = fused(gcn, g, x)
            assert torch.equal(z1, z2)
            assert torch.equal(out1, out2)
    finally:
        lib.mrp_tuning_set(b"fused_producers", 128)


def test_fused_reference_fixture(cuda_device):
    """The reference's own GCN on the 8x8 fixture whose C (16) the fused launch declines (C % 32): the
    two launches serve it; a C = 64 layer with the fixture's graph runs fused, against the oracle."""
    z = load_golden("complete_n8_c16_8x8_b2")
    g = graph_from(z["src"], z["dst"], z["batch_num_nodes"])
    g.ndata["image"] = torch.from_numpy(z["x"])
    g.edata["pose"] = torch.from_numpy(z["pose"])
    g = g.to(cuda_device)
    C = z["x"].shape[1]
    gcn = m.GCN(types.SimpleNamespace(feature_dim=C, gcn_mode=str(z["mode"])))
    gcn.load_state_dict({"edge_encoder." + k: torch.from_numpy(z["param." + k]) for k in PARAM_KEYS})
    gcn = gcn.to(cuda_device)
    with torch.no_grad():
        out = gcn(g)
    assert rel_err(out.cpu().numpy(), z["out"]) <= 1e-5
    # C = 64 on the same graph (the fused launch): against the oracle op sequence on the host
    import oracle
    torch.manual_seed(5)
    x = torch.randn(g.num_nodes(), 64, 8, 8)
    gcn64 = m.GCN(types.SimpleNamespace(feature_dim=64))
    params = {k: v.detach().clone() for k, v in gcn64.edge_encoder.named_parameters()}
    src, dst = (t.cpu().numpy() for t in g.edges())
    ref = oracle.gcn_forward(params, x, g.edata["pose"].cpu(), src, dst)
    gcn64 = gcn64.to(cuda_device)
    before = m.encoder.PATH_COUNTS["fused"]
    with torch.no_grad():
        out = gcn64(g, x.to(cuda_device))
    assert m.encoder.PATH_COUNTS["fused"] == before + 1
    assert rel_err(out.cpu().numpy(), ref.numpy()) <= 1e-5


def test_fused_declines(cuda_device):
    """Shapes outside the fused launch come back as None (the caller's two launches serve them)."""
    lib = m.load_library()
    assert lib.mrp_gcn_fwd_fused_workspace_bytes(4, 9, 64, 64) == 0   # 9 nodes
    assert lib.mrp_gcn_fwd_fused_workspace_bytes(4, 8, 80, 64) == 0   # C % 32
    assert lib.mrp_gcn_fwd_fused_workspace_bytes(4, 8, 64, 6) == 0    # P % 4
    assert lib.mrp_gcn_fwd_fused_workspace_bytes(4, 1, 64, 64) == 0   # 1 node: no edges
    assert lib.mrp_gcn_fwd_fused_workspace_bytes(4, 8, 64, 16) == 0   # 4x4 planes: 64-thread workgroups
    g = complete_batch(2, 8, 64, 4, 4, seed=1, device=cuda_device)  # 4 x 4 planes: 64-thread workgroups
    gcn = layer(64, seed=1, device=cuda_device)
    enc = gcn.edge_encoder.layers
    x = g.ndata["image"]
    assert m.fused.gcn_forward_fused(x, g.edata["pose"], g.csr(cuda_device), enc[0], enc[2]) is None
    with torch.no_grad():
        out = gcn(g, x)  # two launches
    _, ref = two_launch(gcn, g, x)
    assert torch.equal(out, ref)
