"""CPU: the DGL-free graph container and its kernel-facing CSR."""
import numpy as np
import pytest
import torch

import mrp_gnn_amd as m
from mrp_gnn_amd.graph import build_csr


def test_complete_edges_reference_order():
    # dgl/dataloader.py:88-95: i-major, i != j
    src, dst = m.complete_edges(3)
    assert src == [0, 0, 1, 1, 2, 2]
    assert dst == [1, 2, 0, 2, 0, 1]


def test_csr_is_by_destination_in_edge_id_order():
    g = m.complete_graph(4)
    indptr, src, eid, goff, max_nodes = g.host_csr()
    s, d = (t.numpy() for t in g.edges())
    assert indptr.tolist() == [0, 3, 6, 9, 12]
    assert max_nodes == 4 and goff.tolist() == [0, 4]
    for v in range(4):
        seg = eid[indptr[v]:indptr[v + 1]]
        assert list(seg) == sorted(seg)
        assert all(d[e] == v for e in seg)
        assert list(src[indptr[v]:indptr[v + 1]]) == [s[e] for e in seg]
        # complete graph: mailbox order is ascending source (the kernel's summation order)
        assert list(src[indptr[v]:indptr[v + 1]]) == sorted(src[indptr[v]:indptr[v + 1]])


def test_batch_offsets_and_features():
    g1 = m.frame_graph(np.random.RandomState(0).randn(3, 7))
    g2 = m.frame_graph(np.random.RandomState(1).randn(5, 7))
    g1.ndata["image"] = torch.zeros(3, 2, 4, 4)
    g2.ndata["image"] = torch.ones(5, 2, 4, 4)
    b = m.batch([g1, g2])
    assert b.num_nodes() == 8 and b.num_edges() == 6 + 20 and b.batch_size == 2
    assert b.batch_num_nodes().tolist() == [3, 5]
    s, d = b.edges()
    assert int(s[6:].min()) == 3 and int(d[6:].min()) == 3
    assert b.ndata["image"].shape == (8, 2, 4, 4)
    assert torch.equal(b.edata["pose"][6:], g2.edata["pose"])
    csr = b.csr("cpu")
    assert csr.graph_off.tolist() == [0, 3, 8] and csr.max_nodes == 5 and csr.num_graphs == 2


def test_crossing_edge_rejected():
    g = m.RobotGraph([0, 2], [2, 1], num_nodes=4, batch_num_nodes=[2, 2], batch_num_edges=[1, 1])
    with pytest.raises(ValueError, match="crosses"):
        g.host_csr()


def test_too_many_nodes_rejected():
    with pytest.raises(ValueError, match="up to 16"):
        m.complete_graph(17).host_csr()


def test_local_scope_discards_writes():
    g = m.complete_graph(3)
    x = torch.randn(3, 2, 2, 2)
    g.ndata["image"] = x
    with g.local_scope():
        g.ndata["image"] = torch.zeros(3, 2, 2, 2)
        g.ndata["extra"] = torch.zeros(3)
        g.edata["w"] = torch.zeros(6)
    assert g.ndata["image"] is x and "extra" not in g.ndata and "w" not in g.edata


def test_feature_leading_dim_checked():
    g = m.complete_graph(3)
    with pytest.raises(ValueError):
        g.ndata["image"] = torch.zeros(4, 2)
    with pytest.raises(ValueError):
        g.edata["pose"] = torch.zeros(5, 9)


def test_to_shares_structure_and_csr_cache():
    g = m.complete_graph(3)
    g.ndata["image"] = torch.randn(3, 1, 2, 2)
    h = g.to("cpu")
    assert h.num_edges() == 6 and h.ndata["image"].shape == (3, 1, 2, 2)
    c1 = g.csr("cpu")
    assert h.csr("cpu") is c1


def test_knn_edges():
    pos = np.array([[0, 0, 0], [1, 0, 0], [3, 0, 0], [7, 0, 0]], float)
    src, dst = m.knn_edges(pos, 2)
    by_dst = {v: [u for u, w in zip(src, dst) if w == v] for v in range(4)}
    assert by_dst == {0: [1, 2], 1: [0, 2], 2: [0, 1], 3: [1, 2]}
    assert all(len(v) == 2 for v in by_dst.values())


def test_empty_and_zero_degree():
    g = m.RobotGraph([], [], num_nodes=3)
    indptr, src, eid, goff, mx = g.host_csr()
    assert indptr.tolist() == [0, 0, 0, 0] and src.size == 0 and mx == 3
    g2 = m.RobotGraph([0], [1], num_nodes=3)
    assert g2.in_degrees().tolist() == [0, 1, 0]


def test_build_csr_multiedge_and_selfloop():
    indptr, src, eid, goff, mx = build_csr(np.array([0, 0, 2, 1]), np.array([1, 1, 2, 1]), 3, [3])
    assert indptr.tolist() == [0, 0, 3, 4]
    assert eid.tolist() == [0, 1, 3, 2] and src.tolist() == [0, 0, 1, 2]


def test_is_complete_detection():
    rng = np.random.RandomState(0)
    frames = [m.frame_graph(rng.randn(5, 7)) for _ in range(3)]
    assert m.batch(frames).is_complete()
    assert m.batch(frames).csr("cpu").graph_kind == 1
    assert m.batch(frames).csr("cpu", allow_complete=False, allow_regular=False).graph_kind == 0
    # without the complete fast path a complete graph is still regular: in-degree n-1
    assert m.batch(frames).csr("cpu", allow_complete=False).graph_kind == m.graph_regular(4)
    assert not m.batch([m.complete_graph(5), m.complete_graph(4)]).is_complete()  # ragged
    assert not m.frame_graph(rng.randn(6, 7), knn=3).is_complete()
    assert m.batch([m.complete_graph(1), m.complete_graph(1)]).is_complete()
    # same edge set, different edge order -> not the arithmetic numbering
    s, d = m.complete_edges(4)
    assert not m.graph((s[::-1], d[::-1]), num_nodes=4).is_complete()


def test_regular_degree_detection():
    rng = np.random.RandomState(1)
    knn = m.batch([m.frame_graph(rng.randn(12, 7), knn=4), m.frame_graph(rng.randn(9, 7), knn=4)])
    assert knn.in_degree_k() == 4 and knn.csr("cpu").graph_kind == m.graph_regular(4) == (4 << 8) | 2
    assert m.batch([m.frame_graph(rng.randn(12, 7), knn=4), m.frame_graph(rng.randn(9, 7), knn=3)]).in_degree_k() == 0
    wide = m.frame_graph(rng.randn(14, 7), knn=9)  # in-degree above the per-edge-slot limit
    assert wide.in_degree_k() == 9 and wide.csr("cpu").graph_kind == 0
    assert m.graph(([0, 1], [1, 1]), num_nodes=2).in_degree_k() == 0  # node 0 has no in-edge
