"""The DGL binary graph-file reader (``dgl_format.py``; the reference's cache ``dgl_graph_<N>.bin``,
``dgl/dataloader.py:165-175``).  PARITY UNPINNED: DGL is absent and the reference holds no file DGL
wrote, so these tests check the reader against files laid out as the module restates DGL's format
(``tests/dgl_bin_writer.py``) — round trips of the reference's own graph shape (complete N-camera
graphs with image/depth/seg node data and pose edge data), edge-id order, label tensors, selection,
dtypes, and that every malformed or unsupported file fails with a clear error."""
import importlib

import numpy as np
import pytest
import torch

import dgl_bin_writer as W
import mrp_gnn_amd as m
from mrp_gnn_amd import dgl_format

G = importlib.import_module(m.__name__ + ".graph")  # (m.graph is the DGL-style constructor)


def _complete(n):
    src = [i for i in range(n) for j in range(n) if i != j]
    dst = [j for i in range(n) for j in range(n) if i != j]
    return np.array(src), np.array(dst)


def _reference_like(n, seed):
    """One frame as dgl/dataloader.py:96-122 builds it: dgl.graph(edge_list) of the complete
    directed graph, ndata image/depth (float) and seg (long), edata pose (float)."""
    rng = np.random.default_rng(seed)
    src, dst = _complete(n)
    nd = [("image", rng.standard_normal((n, 3, 8, 12)).astype(np.float32)),
          ("depth", rng.standard_normal((n, 1, 8, 12)).astype(np.float32)),
          ("seg", rng.integers(0, 5, (n, 8, 12)).astype(np.int64))]
    ed = [("pose", rng.standard_normal((len(src), 9)).astype(np.float32))]
    return src, dst, nd, ed


def _check(g, src, dst, nd, ed):
    s, d = g.edges()
    assert torch.equal(s, torch.as_tensor(src)) and torch.equal(d, torch.as_tensor(dst))
    for k, v in nd:
        assert torch.equal(g.ndata[k], torch.from_numpy(v)), k
    for k, v in ed:
        assert torch.equal(g.edata[k], torch.from_numpy(v)), k


def test_reference_cache_round_trip(tmp_path):
    frames = [_reference_like(5, s) for s in range(3)]
    path = tmp_path / "dgl_graph_5.bin"
    W.write(path, [W.graph_record(s, d, 5, nd, ed) for s, d, nd, ed in frames])
    assert dgl_format.is_dgl_graph_file(str(path))
    graphs, labels = dgl_format.read_dgl_graphs(str(path))
    assert labels == {} and len(graphs) == 3
    for g, (s, d, nd, ed) in zip(graphs, frames):
        assert g.num_nodes() == 5 and g.num_edges() == 20
        _check(g, s, d, nd, ed)
    # through the package's load_graphs (the dataset's load(), dataloader.py:171-175), with the
    # parity-unpinned warning, and batched into the GCN's graph container
    with pytest.warns(UserWarning, match="parity unpinned"):
        G._WARNED_DGL = False
        g2, _ = G.load_graphs(str(path), [2, 0])
    _check(g2[0], *frames[2])
    _check(g2[1], *frames[0])
    b = G.batch(g2)
    assert b.num_nodes() == 10 and b.num_edges() == 40


def test_edge_ids_order_and_labels(tmp_path):
    src, dst, nd, ed = _reference_like(4, 7)
    eids = np.random.default_rng(0).permutation(len(src))
    labels = [("y", np.arange(6, dtype=np.int64)), ("w", np.linspace(0, 1, 6).astype(np.float32))]
    path = tmp_path / "g.bin"
    W.write(path, [W.graph_record(src, dst, 4, nd, ed, eids=eids)], labels=labels)
    (g,), lab = dgl_format.read_dgl_graphs(str(path))
    _check(g, src, dst, nd, ed)
    assert torch.equal(lab["y"], torch.arange(6)) and torch.equal(lab["w"], torch.linspace(0, 1, 6))


def test_graph_without_tensors_and_dtypes(tmp_path):
    src, dst = _complete(3)
    path = tmp_path / "g.bin"
    nd = [("mask", np.array([True, False, True])), ("h", np.arange(3, dtype=np.float16)),
          ("b", (np.arange(3, dtype=np.int16), (4, 16)))]
    W.write(path, [W.graph_record(src, dst, 3, [], []), W.graph_record(src, dst, 3, nd, [])])
    (g0, g1), _ = dgl_format.read_dgl_graphs(str(path))
    assert g0.num_edges() == 6 and not g0.ndata and not g0.edata
    assert g1.ndata["mask"].dtype == torch.bool and g1.ndata["h"].dtype == torch.float16
    assert g1.ndata["b"].dtype == torch.bfloat16
    s, d = g1.edges()
    assert torch.equal(s, torch.as_tensor(src)) and torch.equal(d, torch.as_tensor(dst))


def test_isolated_nodes_and_empty_file(tmp_path):
    path = tmp_path / "g.bin"
    src, dst = np.array([0, 2]), np.array([2, 0])
    W.write(path, [W.graph_record(src, dst, 6, [("x", np.zeros((6, 2), np.float32))], [])])
    (g,), _ = dgl_format.read_dgl_graphs(str(path))
    assert g.num_nodes() == 6 and g.num_edges() == 2
    W.write(path, [])
    assert dgl_format.read_dgl_graphs(str(path)) == ([], {})


def test_node_data_ending_like_a_tensor_block_header(tmp_path):
    """int64 node data whose last two values are 1, 0 also parse, from 16 bytes before the edge
    tensors, as a block with one node type and no node tensors: the earliest parsing offset wins
    (found with random seg maps in a 100-frame file)."""
    src, dst, nd, ed = _reference_like(4, 3)
    seg = nd[2][1].copy()
    seg.reshape(-1)[-2:] = (1, 0)
    nd = nd[:2] + [("seg", seg)]
    path = tmp_path / "g.bin"
    W.write(path, [W.graph_record(src, dst, 4, nd, ed)] * 2)
    for g in dgl_format.read_dgl_graphs(str(path))[0]:
        _check(g, src, dst, nd, ed)


def test_csr_only_record_rejected_when_its_arrays_look_like_coo(tmp_path):
    """A CSR-only record whose index arrays happen to fit a COO (E <= N): the indptr before them
    marks it, and it is rejected rather than misread."""
    path = tmp_path / "g.bin"
    src, dst = np.array([0, 1, 3]), np.array([1, 2, 0])
    W.write(path, [W.graph_record(src, dst, 5, [], [("w", np.ones(3, np.float32))], csr_only=True)])
    with pytest.raises(ValueError, match="COO"):
        dgl_format.read_dgl_graphs(str(path))


@pytest.mark.parametrize("case", ["magic", "version1", "truncated", "hetero", "csr_only", "index", "counts"])
def test_rejects_malformed_or_unsupported(tmp_path, case):
    src, dst, nd, ed = _reference_like(3, 1)
    path = tmp_path / "g.bin"
    kw = {}
    rec = dict(src=src, dst=dst, n=3, ndata=nd, edata=ed)
    if case == "hetero":
        rec.update(ntypes=("cam", "robot"), node_counts=[3, 2])
    if case == "csr_only":
        rec.update(csr_only=True)
    if case == "counts":
        rec.update(node_counts=[4])  # node tensors have 3 rows
    if case == "magic":
        kw = dict(magic=W.FILE_MAGIC ^ 1)
    if case == "version1":
        kw = dict(version=1)
    W.write(path, [W.graph_record(**rec)], **kw)
    if case == "truncated":
        data = path.read_bytes()
        path.write_bytes(data[:-40])
    err = IndexError if case == "index" else ValueError
    with pytest.raises(err):
        dgl_format.read_dgl_graphs(str(path), [5] if case == "index" else None)
