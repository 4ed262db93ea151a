"""The 1x1 compress conv as batched GEMMs (compress.py) against torch's own Conv2d on the GPU
(the reference op, dgl/model/models.py:165,183), forward and all three gradients.  fp32 both
ways; only the summation order differs, so the bound is the north-star 1e-5 relative."""
import pytest
import torch

import mrp_gnn_amd as m
from conftest import rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,C,hw", [(10, 16, (8, 8)), (24, 64, (4, 4)), (3, 8, (3, 5)), (5, 32, (1, 1))])
@pytest.mark.parametrize("bias", [True, False])
def test_compress_matches_conv2d(cuda_device, n, C, hw, bias):
    torch.manual_seed(n + C)
    conv = torch.nn.Conv2d(2 * C, C, kernel_size=1, bias=bias).to(cuda_device)
    h = torch.randn(n, 2 * C, *hw, device=cuda_device)
    G = torch.randn(n, C, *hw, device=cuda_device)
    h1 = h.clone().requires_grad_(True)
    h2 = h.clone().requires_grad_(True)
    a = m.compress.compress_1x1(conv, h1)
    a.backward(G)
    grads_a = [p.grad.clone() for p in conv.parameters()]
    conv.zero_grad(set_to_none=True)
    b = conv(h2)
    b.backward(G)
    grads_b = [p.grad.clone() for p in conv.parameters()]
    assert rel_err(a.detach().cpu().numpy(), b.detach().cpu().numpy()) <= 1e-5
    assert rel_err(h1.grad.cpu().numpy(), h2.grad.cpu().numpy()) <= 1e-5
    for ga, gb in zip(grads_a, grads_b):
        assert rel_err(ga.cpu().numpy(), gb.cpu().numpy()) <= 1e-5


def test_compress_noncontiguous_input(cuda_device):
    conv = torch.nn.Conv2d(16, 8, 1).to(cuda_device)
    wide = torch.randn(4, 24, 5, 5, device=cuda_device)
    h = wide[:, 4:20]
    assert not h.is_contiguous()
    with torch.no_grad():
        assert rel_err(m.compress.compress_1x1(conv, h).cpu().numpy(), conv(h).cpu().numpy()) <= 1e-5
