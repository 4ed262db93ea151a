"""The zero-padding of shapes the matrix-core kernels do not tile (round 6; ``compress._fwd`` /
``_bwd_data`` / ``_bwd_weight``, ``encoder.EdgeEncoderPaddedFunction``), checked on the CPU as algebra:
the padded operands, multiplied in float64 exactly as the kernels multiply them, give the unpadded
products in their leading blocks.  The kernels themselves run these paths in the GPU suite
(``test_compress_function_declined_shapes``, ``test_padded_training_encoder_vs_float64``)."""
import pytest
import torch

import mrp_gnn_amd as m


@pytest.mark.parametrize("n,C,H,W", [(3, 48, 7, 7), (2, 1, 1, 1), (4, 100, 6, 6), (1, 33, 3, 5)])
def test_compress_padding_algebra(n, C, H, W):
    cp = m.compress
    torch.manual_seed(C + H)
    w = torch.randn(C, 2 * C, 1, 1, dtype=torch.float64)
    b = torch.randn(C, dtype=torch.float64)
    x, a, gy = (torch.randn(n, C, H, W, dtype=torch.float64) for _ in range(3))
    Cp, Pf, Pw = cp._round(C, 32), cp._round(H * W, 4), cp._round(H * W, 32)
    wp, bp = cp._padded_params(w.float(), b.float())
    wp, bp = wp.double(), bp.double()
    assert wp.shape == (Cp, 2 * Cp, 1, 1) and bp.shape == (Cp,)

    def pad(t, P):
        return cp._pad_planes(t.float(), Cp, P).double()

    def unpad(t):
        return cp._unpad_planes(t.float(), C, H, W).double()

    W2 = w.reshape(C, 2 * C)
    Wp = wp.reshape(Cp, 2 * Cp)
    # forward: y = W [x; a] + b
    xp, ap = pad(x, Pf), pad(a, Pf)
    y_ref = torch.einsum("oc,nchw->nohw", W2, torch.cat((x, a), 1)) + b[None, :, None, None]
    yp = torch.einsum("oc,nchw->nohw", Wp, torch.cat((xp, ap), 1)) + bp[None, :, None, None]
    assert torch.allclose(unpad(yp), y_ref.float().double(), rtol=1e-6, atol=1e-5)
    # data gradient: [dx; da] = W^T dy
    gp = pad(gy, Pf)
    d_ref = torch.einsum("oc,nohw->nchw", W2, gy)
    dp = torch.einsum("oc,nohw->nchw", Wp, gp)
    assert torch.allclose(unpad(dp[:, :Cp].contiguous()), d_ref[:, :C].float().double(), rtol=1e-6, atol=1e-5)
    assert torch.allclose(unpad(dp[:, Cp:].contiguous()), d_ref[:, C:].float().double(), rtol=1e-6, atol=1e-5)
    # weight gradient: dW = sum dy [x; a]^T, padded planes of 32 pixels, then the two leading blocks
    gw, xw, aw = pad(gy, Pw), pad(x, Pw), pad(a, Pw)
    dw_ref = torch.einsum("nohw,nchw->oc", gy, torch.cat((x, a), 1))
    dwp = torch.einsum("nohw,nchw->oc", gw, torch.cat((xw, aw), 1))
    dw = torch.cat((dwp[:C, :C], dwp[:C, Cp:Cp + C]), 1)
    assert torch.allclose(dw, dw_ref.float().double(), rtol=1e-5, atol=1e-4)
    assert torch.equal(dwp[C:], torch.zeros_like(dwp[C:]))  # padded output rows: exact zeros


def test_compress_padded_params_cached_per_version():
    cp = m.compress
    w = torch.randn(40, 80, 1, 1)
    b = torch.randn(40)
    p1 = cp._padded_params(w, b)
    assert cp._padded_params(w, b)[0] is p1[0]  # same version: cached
    with torch.no_grad():
        w.mul_(2.0)  # an optimizer-like in-place update bumps the version
    p2 = cp._padded_params(w, b)
    assert p2[0] is not p1[0] and torch.equal(p2[0][:40, :40, 0, 0], w[:, :40, 0, 0])
    cp.clear_packed_weights()


@pytest.mark.parametrize("E,C", [(1, 1), (100, 130), (33, 48), (64, 97)])
def test_encoder_padding_algebra(E, C):
    """z = relu(pose W1^T + b1) W2^T + b2 on W1 / b1 / W2 / b2 zero-padded to C32 (W2 in the top-left
    corner) and E32 zero pose rows: z's 2C columns of its E rows; every parameter gradient the
    leading block of the padded one, the padded rows / columns of dW exact zeros."""
    torch.manual_seed(E + C)
    Cp, Ep = (C + 31) // 32 * 32, (E + 31) // 32 * 32
    w1, b1 = torch.randn(C, 9, dtype=torch.float64), torch.randn(C, dtype=torch.float64)
    w2, b2 = torch.randn(2 * C, C, dtype=torch.float64), torch.randn(2 * C, dtype=torch.float64)
    pose, dz = torch.randn(E, 9, dtype=torch.float64), torch.randn(E, 2 * C, dtype=torch.float64)
    w1p = torch.zeros(Cp, 9, dtype=torch.float64)
    w1p[:C] = w1
    b1p = torch.zeros(Cp, dtype=torch.float64)
    b1p[:C] = b1
    w2p = torch.zeros(2 * Cp, Cp, dtype=torch.float64)
    w2p[: 2 * C, :C] = w2
    b2p = torch.zeros(2 * Cp, dtype=torch.float64)
    b2p[: 2 * C] = b2
    pp = torch.zeros(Ep, 9, dtype=torch.float64)
    pp[:E] = pose
    dzp = torch.zeros(Ep, 2 * Cp, dtype=torch.float64)
    dzp[:E, : 2 * C] = dz

    def run(p, a1, c1, a2, c2, g):
        ps = [t.clone().requires_grad_(True) for t in (p, a1, c1, a2, c2)]
        z = torch.nn.functional.linear(torch.relu(torch.nn.functional.linear(ps[0], ps[1], ps[2])), ps[3], ps[4])
        z.backward(g)
        return z.detach(), [t.grad for t in ps]

    z, g = run(pose, w1, b1, w2, b2, dz)
    zp, gp = run(pp, w1p, b1p, w2p, b2p, dzp)
    assert torch.allclose(zp[:E, : 2 * C], z, rtol=1e-12, atol=1e-12)
    assert torch.allclose(gp[0][:E], g[0])  # dpose
    assert torch.allclose(gp[1][:C], g[1]) and torch.allclose(gp[2][:C], g[2])  # dW1, db1
    assert torch.allclose(gp[3][: 2 * C, :C], g[3]) and torch.allclose(gp[4][: 2 * C], g[4])  # dW2, db2
    assert torch.equal(gp[3][2 * C:], torch.zeros_like(gp[3][2 * C:]))
    assert torch.equal(gp[3][:, C:], torch.zeros_like(gp[3][:, C:]))
