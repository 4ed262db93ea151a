"""CPU: the drop-in model classes keep the reference's API and state_dict keys."""
import types

import pytest
import torch

import mrp_gnn_amd as m
from conftest import golden_cases, load_golden


def opt(**kw):
    d = dict(feature_dim=8, compress_gcn=False, multi_gcn=False, camera_num=4, image_size=64)
    d.update(kw)
    return types.SimpleNamespace(**d)


def test_gcn_state_dict_keys_match_reference():
    z = load_golden(golden_cases()[0])
    ref_keys = sorted("edge_encoder." + k[len("param."):] for k in z if k.startswith("param."))
    gcn = m.GCN(opt())
    assert sorted(gcn.state_dict().keys()) == ref_keys
    # and the reference's tensors load into it unchanged
    sd = {"edge_encoder." + k[len("param."):]: torch.from_numpy(v) for k, v in z.items() if k.startswith("param.")}
    m.GCN(opt(feature_dim=sd["edge_encoder.layers.0.weight"].shape[0])).load_state_dict(sd)


def test_edge_encoder_reference_return_values():
    enc = m.edge_encoder([8, 8])
    pose = torch.randn(5, 9)
    g, b = enc(pose)
    assert g.shape == (5, 8, 1, 1) and b.shape == (5, 8, 1, 1)
    gb = enc.film_params(pose)
    assert torch.equal(gb[:, :, 0], g[:, :, 0, 0]) and torch.equal(gb[:, :, 1], b[:, :, 0, 0])


def test_stack_keys_follow_multi_view_dgl_model():
    o = opt(compress_gcn=True, multi_gcn=True)
    keys = set(m.multi_view_dgl_model(o).state_dict())
    prefixes = {k.split(".")[0] for k in keys}
    assert prefixes == {"gcn1", "conv1", "gcn2", "conv2"}
    assert keys == set(m.GCNBlock(o).state_dict())
    assert m.multi_view_dgl_model(o).conv1.weight.shape == (8, 16, 1, 1)


def test_multi_gcn_requires_compress():
    with pytest.raises(AssertionError):
        m.GCNBlock(opt(multi_gcn=True))


def test_gcn_return_input_mode_is_reference_faithful():
    g = m.complete_graph(4)
    x = torch.randn(4, 8, 3, 3)
    g.ndata["image"] = x
    g.edata["pose"] = torch.randn(12, 9)
    gcn = m.GCN(opt(gcn_return="input"))
    assert gcn(g) is x  # models.py:226 returns g.ndata['image']
    assert gcn(g, x) is x


def test_aggregate_mode_on_cpu_fails_loudly():
    g = m.complete_graph(4)
    g.ndata["image"] = torch.randn(4, 8, 3, 3)
    g.edata["pose"] = torch.randn(12, 9)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m.GCN(opt())(g)
