"""GPU: the fused edge encoder (mrp_edge_encoder_fwd) against the reference's torch layers and the
golden fixtures; its autograd backward against torch autograd."""
import numpy as np
import pytest
import torch

import mrp_gnn_amd as m
from conftest import golden_cases, load_golden, rel_err

pytestmark = pytest.mark.gpu
PARAM_KEYS = ["layers.0.weight", "layers.0.bias", "layers.2.weight", "layers.2.bias"]


@pytest.mark.parametrize("name", [n for n in golden_cases() if "copyu" not in n])
def test_fused_encoder_matches_reference_fixture(cuda_device, name):
    z = load_golden(name)
    C = z["x"].shape[1]
    enc = m.edge_encoder([C, C])
    enc.load_state_dict({k: torch.from_numpy(z["param." + k]) for k in PARAM_KEYS})
    enc = enc.to(cuda_device)
    gb = enc.film_params(torch.from_numpy(z["pose"]).to(cuda_device))
    assert rel_err(gb.detach().cpu().numpy(), z["gb"]) <= 1e-5


@pytest.mark.parametrize("E,C", [(1, 1), (7, 3), (96, 64), (1792, 512), (100, 130), (33, 1280), (448, 2048)])
def test_fused_encoder_vs_torch_layers(cuda_device, E, C):
    torch.manual_seed(E + C)
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 5).to(cuda_device)
    fused = enc.film_params(pose)
    ref = enc.layers(pose).view(E, C, 2)
    assert fused.shape == ref.shape
    assert float((fused - ref).abs().max()) <= 2e-6  # sigmoid outputs in (0, 1)
    # backward: custom Function vs torch autograd through the same layers
    g = torch.randn_like(ref)
    pr = pose.clone().requires_grad_(True)
    pf = pose.clone().requires_grad_(True)
    enc.zero_grad()
    (enc.layers(pr).view(E, C, 2) * g).sum().backward()
    ref_grads = [p.grad.clone() for p in enc.parameters()] + [pr.grad.clone()]
    enc.zero_grad()
    (enc.film_params(pf) * g).sum().backward()
    got_grads = [p.grad.clone() for p in enc.parameters()] + [pf.grad.clone()]
    for a, b in zip(got_grads, ref_grads):
        assert rel_err(a.cpu().numpy(), b.cpu().numpy()) <= 1e-4


def test_fused_encoder_empty(cuda_device):
    enc = m.edge_encoder([8, 8]).to(cuda_device)
    out = enc.film_params(torch.zeros(0, 9, device=cuda_device))
    assert out.shape == (0, 8, 2)
