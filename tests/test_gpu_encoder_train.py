"""The edge encoder's training path on the split-bf16 matrix cores (encoder.EdgeEncoderSplitFunction:
mrp_edge_encoder_fwd_split_train, _bwd_prep, _bwd_split, _bwd_t) — the reference's Linear / ReLU /
Linear (``dgl/model/models.py:146-149``) under ``loss.backward()`` (``dgl/training.py:208-210``).
Every parameter gradient, the logits and the pose gradient are judged against a float64 evaluation
of the reference layers with the fp32 yardstick (``stack_ref.within``), at the BASELINE shapes
(E, C) = (1792, 512), (448, 2048), (512, 1024) and small ones; the path taken is asserted."""
import os

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import mrp_gnn_amd as m
import stack_ref

pytestmark = pytest.mark.gpu


def _reference(enc, pose, gz, dtype):
    ps = [p.detach().to(dtype).requires_grad_(True) for p in enc.parameters()]
    pz = pose.detach().to(dtype).requires_grad_(True)
    z = torch.nn.functional.linear(torch.relu(torch.nn.functional.linear(pz, ps[0], ps[1])), ps[2], ps[3])
    z.backward(gz.to(dtype))
    return z.detach(), [p.grad for p in ps], pz.grad


@pytest.mark.parametrize("form", ["fused", "two_stream", "pose_grad"])
@pytest.mark.parametrize("E,C", [(1792, 512), (448, 2048), (512, 1024), (96, 64), (32, 32), (224, 160)])
def test_split_training_encoder_vs_float64(cuda_device, E, C, form):
    """form: "fused" — parameters only, the three-launch single-stream backward
    (``mrp_edge_encoder_bwd_fused``); "two_stream" — the same with the fused form switched off
    (``_bwd_prep`` / ``_bwd_split`` on two streams / ``_bwd_t``); "pose_grad" — the pose needs a gradient
    too, which only the two-stream form provides."""
    m.encoder.set_fused_backward(form != "two_stream")
    try:
        _check_training_encoder(cuda_device, E, C, pose_grad=form == "pose_grad")
    finally:
        m.encoder.set_fused_backward(True)


@pytest.mark.parametrize("form", ["fused", "two_stream", "pose_grad"])
@pytest.mark.parametrize("E,C", [(1, 1), (7, 3), (100, 130), (33, 1281), (1000, 48), (56, 1000), (1792, 500),
                                 (64, 96 + 1), (31, 32), (1793, 512)])
def test_padded_training_encoder_vs_float64(cuda_device, E, C, form):
    """E or C not a multiple of 32 (these trained on hipBLASLt GEMMs): the split-bf16
    kernels on zero-padded operands (``EdgeEncoderPaddedFunction``), every form, every gradient
    against float64 — e.g. ``feature_dim`` 1000 or 500, ragged edge counts, one channel."""
    m.encoder.set_fused_backward(form != "two_stream")
    try:
        _check_training_encoder(cuda_device, E, C, pose_grad=form == "pose_grad", path="split_padded")
    finally:
        m.encoder.set_fused_backward(True)


@pytest.mark.parametrize("E,C", [(1, 1), (100, 130), (33, 1281), (1000, 48), (1792, 500)])
def test_padded_inference_encoder_vs_float64(cuda_device, E, C):
    """No gradient wanted, C % 32 != 0: one ``mrp_edge_encoder_fwd_split`` launch on the padded weight
    image, z its 2C leading columns; repacked after an in-place weight update."""
    torch.manual_seed(E + 3 * C)
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 8).to(cuda_device)
    for step in range(2):
        before = m.encoder.PATH_COUNTS["split"]
        with torch.no_grad():
            z = m.encoder.edge_logits(enc.layers, pose)
        assert m.encoder.PATH_COUNTS["split"] == before + 1
        assert z.shape == (E, 2 * C) and z.is_contiguous()
        z32, _, _ = _reference(enc, pose, torch.zeros(E, 2 * C, device=cuda_device), torch.float32)
        z64, _, _ = _reference(enc, pose, torch.zeros(E, 2 * C, device=cuda_device), torch.float64)
        ok, errs = stack_ref.within(z, z32, z64)
        assert ok, (step, errs)
        with torch.no_grad():
            for p in enc.parameters():
                p.mul_(-1.25)  # an optimizer-like in-place update: the padded image is rebuilt


@pytest.mark.parametrize("E,C", [(1, 32), (63, 64), (1792, 512), (100, 2048), (20000, 64), (4097, 1312)])
def test_pose_gradient_kernel(cuda_device, E, C):
    """``mrp_edge_encoder_bwd_pose`` (dpose = (dh^T (.) [h^T > 0])^T W1) against float64: one k slice
    (many edges) and many (few edges, wide C), ragged 64-edge blocks."""
    torch.manual_seed(E + C)
    hT = torch.randn(C, E, device=cuda_device)
    dhT = torch.randn(C, E, device=cuda_device)
    w1 = torch.randn(C, 9, device=cuda_device)
    got = m.encoder.pose_grad(dhT, hT, w1)
    d = dhT * (hT > 0)
    f32 = d.t().mm(w1)
    f64 = d.double().t().mm(w1.double())
    ok, errs = stack_ref.within(got, f32, f64)
    assert ok, errs
    again = m.encoder.pose_grad(dhT, hT, w1)
    assert torch.equal(got, again)  # fixed summation order


def _check_training_encoder(cuda_device, E, C, pose_grad, path="split_train"):
    torch.manual_seed(E + 7 * C)
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 8).to(cuda_device).requires_grad_(pose_grad)
    gz = torch.randn(E, 2 * C, device=cuda_device)
    before = m.encoder.PATH_COUNTS[path]
    z = m.encoder.edge_logits(enc.layers, pose)
    assert m.encoder.PATH_COUNTS[path] == before + 1
    z.backward(gz)
    z32, g32, p32 = _reference(enc, pose, gz, torch.float32)
    z64, g64, p64 = _reference(enc, pose, gz, torch.float64)
    ok, errs = stack_ref.within(z.detach(), z32, z64)
    assert ok, ("z", errs)
    for name, p, a32, a64 in zip(("w1", "b1", "w2", "b2"), enc.parameters(), g32, g64):
        ok, errs = stack_ref.within(p.grad, a32, a64)
        assert ok, (name, errs)
    if pose_grad:
        ok, errs = stack_ref.within(pose.grad, p32, p64)
        assert ok, ("pose", errs)


def test_fused_and_two_stream_backward_agree(cuda_device):
    """The fused backward and the two-stream one compute the same products in the same order per
    output except for their split-K counts: dW1/db1/dW2/db2 agree to fp32 rounding."""
    torch.manual_seed(5)
    E, C = 1792, 512
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 8).to(cuda_device)
    gz = torch.randn(E, 2 * C, device=cuda_device)
    grads = []
    for fused in (True, False):
        m.encoder.set_fused_backward(fused)
        enc.zero_grad(set_to_none=True)
        m.encoder.edge_logits(enc.layers, pose).backward(gz)
        grads.append([p.grad.clone() for p in enc.parameters()])
    m.encoder.set_fused_backward(True)
    for a, b in zip(*grads):
        assert float((a - b).abs().max() / b.abs().max()) < 1e-5


def test_split_training_encoder_deterministic_and_repacks(cuda_device):
    """Two backward passes give bit-identical gradients (fixed-order sums, no atomics); after an
    optimizer-style in-place update the packed image and W2^T follow the new weights."""
    torch.manual_seed(3)
    E, C = 448, 256
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 8).to(cuda_device)
    gz = torch.randn(E, 2 * C, device=cuda_device)
    grads = []
    for _ in range(2):
        enc.zero_grad(set_to_none=True)
        m.encoder.edge_logits(enc.layers, pose).backward(gz)
        grads.append([p.grad.clone() for p in enc.parameters()])
    for a, b in zip(*grads):
        assert torch.equal(a, b)
    with torch.no_grad():
        for p in enc.parameters():
            p.mul_(-0.5)
    enc.zero_grad(set_to_none=True)
    z = m.encoder.edge_logits(enc.layers, pose)
    z.backward(gz)
    z32, g32, _ = _reference(enc, pose, gz, torch.float32)
    z64, g64, _ = _reference(enc, pose, gz, torch.float64)
    assert stack_ref.within(z.detach(), z32, z64)[0]
    for p, a32, a64 in zip(enc.parameters(), g32, g64):
        assert stack_ref.within(p.grad, a32, a64)[0]


def _prop_settings():
    return settings(max_examples=int(os.environ.get("MRP_PROPERTY_EXAMPLES", "12")), deadline=None,
                    derandomize=not os.environ.get("MRP_PROPERTY_HUNT"), database=None,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


@_prop_settings()
@given(st.integers(1, 64), st.integers(1, 24), st.sampled_from(["fused", "two_stream", "pose_grad"]))
def test_split_training_encoder_property(cuda_device, e32, c32, form):
    """Property form of the test above (hypothesis, bounded and derandomized; ``MRP_PROPERTY_EXAMPLES``
    / ``MRP_PROPERTY_HUNT`` as in tests/test_gpu_properties.py): any E and C the split training path
    takes (multiples of 32, E up to 2048, C up to 768) on every backward form."""
    m.encoder.set_fused_backward(form != "two_stream")
    try:
        _check_training_encoder(cuda_device, 32 * e32, 32 * c32, pose_grad=form == "pose_grad")
    finally:
        m.encoder.set_fused_backward(True)


@_prop_settings()
@given(st.integers(1, 1500), st.integers(1, 700), st.sampled_from(["fused", "two_stream", "pose_grad"]))
def test_padded_training_encoder_property(cuda_device, E, C, form):
    """Property form of the padded path: any E and C (``EdgeEncoderPaddedFunction`` where either is not
    a multiple of 32, the split path where both are), every backward form, against float64."""
    path = "split_train" if E % 32 == 0 and C % 32 == 0 else "split_padded"
    m.encoder.set_fused_backward(form != "two_stream")
    try:
        _check_training_encoder(cuda_device, E, C, pose_grad=form == "pose_grad", path=path)
    finally:
        m.encoder.set_fused_backward(True)


@pytest.mark.parametrize("E,C", [(1792, 512), (448, 2048), (96, 64)])
def test_fused_backward_w2t_image_bit_identical(cuda_device, E, C):
    """The fused backward with both products' A operands pre-split (knob enc_bwd_psa 2, the default:
    W2^T's packed image, dz^T written as one by dzT_pack), with W2^T's only (1) and with both split in
    the kernel (0) form the same products in the same order: dW1, db1 and dW2 bit-identical; db2 (summed
    per 64-edge block under 2, per split otherwise) to fp32 rounding."""
    torch.manual_seed(E + C)
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 8).to(cuda_device)
    gz = torch.randn(E, 2 * C, device=cuda_device)
    lib = m.load_library()
    grads = []
    try:
        for v in (2, 1, 0):
            assert lib.mrp_tuning_set(b"enc_bwd_psa", v) == 0
            enc.zero_grad(set_to_none=True)
            m.encoder.edge_logits(enc.layers, pose).backward(gz)
            grads.append([p.grad.clone() for p in enc.parameters()])
    finally:
        lib.mrp_tuning_set(b"reset", 0)
    for g in grads[1:]:
        for i in range(3):  # w1, b1, w2
            assert torch.equal(grads[0][i], g[i]), i
        assert float((grads[0][3] - g[3]).abs().max()) <= 1e-6 * float(g[3].abs().max()) + 1e-7
    assert torch.equal(grads[1][3], grads[2][3])


@pytest.mark.parametrize("E,C", [(1792, 512), (896, 512), (448, 2048), (224, 160)])
def test_train_forward_writes_hidden(cuda_device, E, C):
    """``mrp_edge_encoder_fwd_split_train`` directly: h^T (C, E) against relu(pose W1^T + b1) evaluated in
    float64 with the fp32 yardstick, and the logits bit-identical to the inference kernel's — at the
    headline shape (8 waves, every hidden block before z, h^T stored after the z loop) and at shapes
    that take the round-by-round form (4 waves, or more hidden blocks than the LDS slots hold)."""
    import ctypes

    from mrp_gnn_amd.aggregate import _ptr
    torch.manual_seed(E + C)
    enc = m.edge_encoder([C, C]).to(cuda_device)
    l1, l2 = enc.layers[0], enc.layers[2]
    pose = (torch.randn(E, 9) * 8).to(cuda_device)
    img = m.encoder.packed_weights(l1, l2)
    z = torch.empty(E, 2 * C, device=cuda_device)
    hT = torch.full((C, E), float("nan"), device=cuda_device)
    lib = m.load_library()
    m._lib.check(lib.mrp_edge_encoder_fwd_split_train(
        _ptr(pose), _ptr(img), _ptr(l2.bias.detach().contiguous()), E, C, _ptr(z), _ptr(hT), E,
        ctypes.c_void_p(torch.cuda.current_stream(cuda_device).cuda_stream)), "mrp_edge_encoder_fwd_split_train")
    with torch.no_grad():
        z_inf = m.encoder.encoder_forward_split(pose, l1, l2)
        h32 = torch.relu(torch.nn.functional.linear(pose, l1.weight, l1.bias)).t()
        h64 = torch.relu(torch.nn.functional.linear(pose.double(), l1.weight.double(), l1.bias.double())).t()
    torch.cuda.synchronize()
    assert torch.equal(z, z_inf)
    assert not torch.isnan(hT).any()
    ok, errs = stack_ref.within(hT, h32, h64)
    assert ok, errs
