"""Property-based accuracy (hypothesis) of the split-bf16 compress GEMMs — the 1x1 ``Conv2d(2C, C)``
after the aggregation (``dgl/model/models.py:182-189``) and both its gradients — on arbitrary layer
shapes: node counts 1..24, C any multiple of 32 up to 512, planes of any height and width that the
kernels take (H W % 4 == 0; the split weight gradient C % 64 == 0 and H W % 32 == 0, else the fp32
MFMA one, which may decline the plane), with the forward / data-gradient form drawn among the
default (per shape), the 16x16x32 form forced on every shape (ragged M tiles) and the 128-row form.
Each result against float64 with the fp32 yardstick (``tests/stack_ref.py``); repeated launches
bit-identical.  Example counts bounded and derandomized (``MRP_PROPERTY_EXAMPLES`` /
``MRP_PROPERTY_HUNT`` as in tests/test_gpu_properties.py)."""
import os

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import mrp_gnn_amd as m
import stack_ref

pytestmark = pytest.mark.gpu

SETTINGS = settings(max_examples=int(os.environ.get("MRP_PROPERTY_EXAMPLES", "20")), deadline=None,
                    derandomize=not os.environ.get("MRP_PROPERTY_HUNT"), database=None,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


@SETTINGS
@given(st.integers(1, 24), st.integers(1, 16), st.integers(1, 8), st.sampled_from([4, 8, 12, 16, 32]),
       st.sampled_from([-1, 7, 2]), st.integers(0, 2 ** 31 - 1))
def test_compress_gemms_vs_float64(cuda_device, n, c32, H, W, form, seed):
    C = 32 * c32
    gen = torch.Generator().manual_seed(seed)
    w = (torch.randn(C, 2 * C, 1, 1, generator=gen) / (2 * C) ** 0.5).to(cuda_device)
    b = torch.randn(C, generator=gen).to(cuda_device)
    x, a, gy = (torch.randn(n, C, H, W, generator=gen).to(cuda_device) for _ in range(3))
    lib = m.load_library()
    prev = m.compress.compress_path()
    m.compress.set_compress_path("split")
    assert lib.mrp_tuning_set(b"gemm_split", form) == 0
    try:
        y = m.compress.compress_forward(w, b, x, a)
        gx, ga = m.compress.compress_backward_data(w, gy)
        wg = m.compress.compress_backward_weight(gy, x, a)
        assert torch.equal(y, m.compress.compress_forward(w, b, x, a))
        d2 = m.compress.compress_backward_data(w, gy)
        assert torch.equal(d2[0], gx) and torch.equal(d2[1], ga)
    finally:
        lib.mrp_tuning_set(b"gemm_split", -1)
        m.compress.set_compress_path(prev)
    cat = torch.cat((x, a), 1)
    w2 = w.reshape(C, 2 * C)
    ok, errs = stack_ref.within(y, torch.einsum("oc,nchw->nohw", w2, cat) + b.view(1, C, 1, 1),
                                torch.einsum("oc,nchw->nohw", w2.double(), cat.double()) + b.double().view(1, C, 1, 1))
    assert ok, ("y", errs)
    ok, errs = stack_ref.within(torch.cat((gx, ga), 1), torch.einsum("oc,nohw->nchw", w2, gy),
                                torch.einsum("oc,nohw->nchw", w2.double(), gy.double()))
    assert ok, ("grad", errs)
    if wg is None:  # the weight-gradient kernels decline this plane; the caller falls back to torch
        assert (H * W) % 32 != 0
        return
    gw, gb = wg
    ok, errs = stack_ref.within(gw, torch.einsum("nohw,nchw->oc", gy, cat).reshape(C, 2 * C, 1, 1),
                                torch.einsum("nohw,nchw->oc", gy.double(), cat.double()).reshape(C, 2 * C, 1, 1))
    assert ok, ("gw", errs)
    ok, errs = stack_ref.within(gb, gy.sum((0, 2, 3)), gy.double().sum((0, 2, 3)))
    assert ok, ("gb", errs)
