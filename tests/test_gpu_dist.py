"""The gradient all-reducer with the HIP backward kernels writing into its bucket slots.

One rank (gloo, world 1, in this process): what matters here is where the kernels write, not the
collective.  A parameter of odd size registered after the GCN comes first in backward order — the
layout of ``multi_view_dgl_model``, whose decoder (``dgl/training.py:282``: ``num_classes + 1``
output channels) follows the GCN — so without aligned slots the encoder's 16-byte-aligned gradient
pointers would land misaligned and the kernels would refuse them.
"""
import socket
import types

import pytest
import torch
import torch.distributed as dist

import mrp_gnn_amd as m
from mrp_gnn_amd.dist import GradAllReducer

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def world1():
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    try:
        yield
    finally:
        dist.destroy_process_group()


class _WithDecoder(torch.nn.Module):
    def __init__(self, C):
        super().__init__()
        torch.manual_seed(0)
        self.gcn = m.GCNStack(types.SimpleNamespace(feature_dim=C, compress_gcn=True, multi_gcn=False,
                                                    gcn_layers=2, gcn_combine="cat_compress"))
        self.decoder = torch.nn.Module()  # registered after the GCN: first in backward order
        self.decoder.head = torch.nn.Parameter(torch.randn(7))  # odd numel

    def forward(self, g, x):
        return self.gcn(g, x) * self.decoder.head.sum()


def _frames(B, N, C, H, dev):
    import numpy as np
    rng = np.random.RandomState(3)
    gs = []
    for _ in range(B):
        poses = np.concatenate([rng.uniform(-10, 10, (N, 3)), rng.standard_normal((N, 4))], 1).astype(np.float32)
        gs.append(m.frame_graph(poses))
    g = m.batch(gs)
    torch.manual_seed(1)
    g.ndata["image"] = torch.randn(g.num_nodes(), C, H, H)
    return g.to(dev)


def test_reducer_slots_with_odd_parameter_first(cuda_device, world1):
    C = 64
    g = _frames(4, 8, C, 8, cuda_device)
    x = g.ndata["image"]
    gy = torch.randn_like(x)
    ref = _WithDecoder(C).to(cuda_device)
    ref(g, x).backward(gy)
    net = _WithDecoder(C).to(cuda_device)
    red = GradAllReducer(net.parameters())
    assert red.buckets[0][0] is net.decoder.head
    for step in range(2):
        for p in net.parameters():
            p.grad = None
        before = red.copies
        red.arm()
        net(g, x).backward(gy)
        red.synchronize()
        # the head's gradient comes from torch (one copy); every GCN gradient was written in its slot
        # by a HIP kernel — encoder W1/b1/W2/b2 and the compress weight/bias of both layers
        assert red.copies - before == 1, (step, red.copies - before)
        for (k, p), (_, q) in zip(net.named_parameters(), ref.named_parameters()):
            flat = red._flat[red._bucket_of[id(p)]]
            assert flat.data_ptr() <= p.grad.data_ptr() < flat.data_ptr() + flat.numel() * 4, k
            assert p.grad.data_ptr() % 16 == 0, k
            assert torch.equal(p.grad, q.grad), k  # same kernels, same order: bit-identical
    red.remove()
