"""Drop-in compatibility with the reference harness: a checkpoint pickled by the
reference (``torch.save({'model': GCN ...})``, class path ``model.models.GCN``; the fixture
``tests/golden/ref_gcn_checkpoint.pt`` was written by ``tests/golden/make_golden.py`` from the
reference's own classes) unpickles into the MI355X classes through ``compat.reference_class_path``;
``from dgl import batch`` / ``from model import models`` resolve; the reference's training-loop
plumbing runs on the HIP path.  The fixture is our own file, so ``weights_only=False`` is allowed."""
import os
import subprocess
import sys
import types

import warnings

import numpy as np
import pytest
import torch

import mrp_gnn_amd as m
from conftest import GOLDEN_DIR, ROOT, load_golden, rel_err

CKPT = os.path.join(GOLDEN_DIR, "ref_gcn_checkpoint.pt")


def load_reference_checkpoint(**kw):
    import warnings
    with m.compat.reference_class_path(**kw), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return torch.load(CKPT, weights_only=False)


def test_reference_checkpoint_unpickles_into_native_classes():
    saved = {k: sys.modules.get(k) for k in ("model", "model.models")}
    ck = load_reference_checkpoint()
    assert {k: sys.modules.get(k) for k in ("model", "model.models")} == saved  # aliases removed again
    gcn = ck["model"]
    assert type(gcn) is m.GCN and type(gcn.edge_encoder) is m.edge_encoder
    assert ck["n_iter"] == 3
    io = load_golden("ref_gcn_checkpoint_io")
    sd = gcn.state_dict()
    assert sorted(sd) == sorted(k[len("gcn1."):] for k in io if k.startswith("gcn1."))
    for k, v in sd.items():
        assert np.array_equal(v.numpy(), io["gcn1." + k])
    stack = ck["stack"]
    assert type(stack.gcn2) is m.GCN and stack.gcn1 is gcn
    assert gcn.opt.feature_dim == 8 and gcn.opt.compress_gcn  # the reference's argparse opt travels along
    # the reference opt has no gcn_return: the unpickled layers keep the reference's return-the-input
    assert not hasattr(gcn.opt, "gcn_return") and gcn.gcn_return_default == "input"
    assert load_reference_checkpoint(gcn_return="aggregate")["model"].gcn_return_default == "aggregate"


def test_unpickled_reference_gcn_warns_and_returns_input():
    with m.compat.reference_class_path():
        with pytest.warns(UserWarning, match="models.py:226"):
            ck = torch.load(CKPT, weights_only=False)
    io = load_golden("ref_gcn_checkpoint_io")
    g = m.RobotGraph(io["src"], io["dst"], num_nodes=io["x"].shape[0], batch_num_nodes=[4, 4],
                     batch_num_edges=[12, 12])
    x = torch.from_numpy(io["x"])
    g.ndata["image"] = x
    assert ck["model"](g) is x  # what the reference forward returns; no kernel runs (works on the CPU)


def _native_stack(C=32):
    opt = types.SimpleNamespace(feature_dim=C, compress_gcn=True, multi_gcn=True)
    torch.manual_seed(1)
    return m.GCNStack(opt)


def _round_trips(obj, tmp_path):
    import copy
    import io
    import warnings
    buf = io.BytesIO()
    torch.save({"model": obj}, buf)  # the reference's whole-module checkpoint (training.py:345-355)
    buf.seek(0)
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # no "returning the input" warning for a native model
        return [copy.deepcopy(obj), torch.load(buf, weights_only=False)["model"]]  # our own file


def test_native_gcn_survives_deepcopy_and_checkpoint(tmp_path):
    """A GCN built here (opt without gcn_return) keeps computing the aggregate after deepcopy and a
    whole-module torch.save / torch.load; only a reference-pickled GCN falls back to 'input'."""
    stack = _native_stack()
    assert stack.gcn1._return_mode() == "aggregate"
    for copy_ in _round_trips(stack, tmp_path):
        assert copy_.gcn1._return_mode() == "aggregate" and copy_.gcn2._return_mode() == "aggregate"
        assert sorted(copy_.state_dict()) == sorted(stack.state_dict())


@pytest.mark.gpu
def test_native_gcn_round_trip_outputs_identical(cuda_device, tmp_path):
    stack = _native_stack().to(cuda_device)
    rng = np.random.RandomState(4)
    g = m.batch([m.frame_graph(np.concatenate([rng.uniform(-5, 5, (4, 3)), rng.standard_normal((4, 4))], 1)
                               .astype(np.float32)) for _ in range(3)])
    g.ndata["image"] = torch.randn(12, 32, 8, 8)
    g = g.to(cuda_device)
    with torch.no_grad():
        ref = stack(g, g.ndata["image"])
        assert not torch.equal(ref, g.ndata["image"][:, :32])
        for copy_ in _round_trips(stack, tmp_path):
            assert torch.equal(copy_.to(cuda_device)(g, g.ndata["image"]), ref)


def test_models_alias_resolves_reference_only_names_through_fallback():
    with m.compat.reference_class_path():
        from model import models
        assert models.GCN is m.GCN and models.multi_view_dgl_model is m.multi_view_dgl_model
        with pytest.raises(AttributeError, match="fallback"):
            models.decoder  # noqa: B018  (torchvision/dense-conv code, outside the hot path)
    fb = types.SimpleNamespace(decoder="ref-decoder", GCN="not-used")
    with m.compat.reference_class_path(fallback=fb):
        from model import models
        assert models.decoder == "ref-decoder" and models.GCN is m.GCN


def test_dgl_alias_when_dgl_is_absent():
    code = ("import sys; sys.path.insert(0, %r); import mrp_gnn_amd as m; m.compat.install();"
            "from dgl import batch; import dgl;"
            "g = batch([m.complete_graph(3), m.complete_graph(3)]);"
            "assert batch is m.batch and dgl.DGLGraph is m.RobotGraph and g.num_nodes() == 6;"
            "from model import models; assert models.GCN is m.GCN; print('ok')") % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().endswith("ok")


def test_collate_matches_dgl_batch_semantics():
    rng = np.random.RandomState(0)
    frames = []
    for _ in range(3):
        g = m.frame_graph(rng.rand(4, 7).astype(np.float32))
        g.ndata["image"] = torch.randn(4, 2, 3, 3)
        g.ndata["depth"] = torch.randn(4, 1, 8, 8)
        frames.append(g)
    b = m.compat.collate(frames)
    assert b.batch_size == 3 and b.num_nodes() == 12 and b.num_edges() == 36
    assert torch.equal(b.ndata["depth"][4:8], frames[1].ndata["depth"])
    assert b.is_complete()


@pytest.mark.gpu
def test_reference_checkpoint_runs_on_the_hip_path(cuda_device):
    ck = load_reference_checkpoint()
    io = load_golden("ref_gcn_checkpoint_io")
    g = m.RobotGraph(io["src"], io["dst"], num_nodes=io["x"].shape[0], batch_num_nodes=[4, 4],
                     batch_num_edges=[12, 12])
    g.ndata["image"] = torch.from_numpy(io["x"])
    g.edata["pose"] = torch.from_numpy(io["pose"])
    gd = g.to(cuda_device)
    stack = ck["stack"].to(cuda_device)
    with torch.no_grad():
        assert stack.gcn1(gd) is gd.ndata["image"]  # the reference as shipped returns its input
    stack = load_reference_checkpoint(gcn_return="aggregate")["stack"].to(cuda_device)
    with torch.no_grad():
        assert rel_err(stack.gcn1(gd).cpu(), io["out_gcn1"]) <= 1e-5
        assert rel_err(stack.gcn2(gd).cpu(), io["out_gcn2"]) <= 1e-5


@pytest.mark.gpu
def test_reference_training_loop_plumbing(cuda_device):
    """``train_dgl`` (dgl/training.py:176-218) driven unchanged over the aliases: DataLoader with
    the dgl.batch collate, ``data.to('cuda:0')``, ``model(data)``, backward, Adam step."""
    opt = types.SimpleNamespace(feature_dim=16, compress_gcn=True, multi_gcn=True, camera_num=4, image_size=8,
                                skip_level=False, task="depth")
    with m.compat.reference_class_path():
        from dgl import batch as dgl_batch  # noqa: F401  (what training.py imports, if DGL is absent)
        from model import models
        torch.manual_seed(0)
        model = models.multi_view_dgl_model(opt).to(cuda_device)
    rng = np.random.RandomState(1)
    frames = []
    for _ in range(6):
        g = m.frame_graph(np.concatenate([rng.uniform(-5, 5, (4, 3)), rng.standard_normal((4, 4))], 1)
                          .astype(np.float32))
        g.ndata["image"] = torch.randn(4, 16, 8, 8)  # feature maps (the encoder is outside the hot path)
        g.ndata["depth"] = torch.rand(4, 1, 8, 8)
        frames.append(g)
    loader = torch.utils.data.DataLoader(frames, batch_size=2, shuffle=False, collate_fn=m.compat.collate)
    optimizer = torch.optim.Adam(model.parameters(), 0.005)
    before = {k: v.detach().clone() for k, v in model.state_dict().items()}
    for data in loader:
        optimizer.zero_grad()
        data = data.to("cuda:0")
        pred = model(data)
        assert pred.shape == (8, 16, 8, 8)
        loss = torch.nn.functional.smooth_l1_loss(pred[:, :1], data.ndata["depth"])
        loss.backward()
        optimizer.step()
    after = model.state_dict()
    for k in before:
        assert torch.isfinite(after[k]).all()
        assert not torch.equal(before[k], after[k]), f"{k} did not train"


def test_graph_cache_round_trip(tmp_path):
    rng = np.random.RandomState(2)
    graphs = []
    for n in (3, 5, 4):
        g = m.frame_graph(rng.rand(n, 7).astype(np.float32), knn=2 if n == 5 else None)
        g.ndata["image"] = torch.randn(n, 3, 4, 4)
        g.ndata["seg"] = torch.randint(0, 7, (n, 1, 4, 4))
        graphs.append(g)
    path = str(tmp_path / "dgl_graph_5.bin")  # the reference's file name (dataloader.py:168)
    m.save_graphs(path, graphs, {"glabel": torch.arange(3)})
    back, labels = m.load_graphs(path)
    assert torch.equal(labels["glabel"], torch.arange(3))
    assert len(back) == 3
    for a, b in zip(graphs, back):
        assert a.num_nodes() == b.num_nodes() and a.num_edges() == b.num_edges()
        for t, u in zip(a.edges(), b.edges()):
            assert torch.equal(t, u)
        for k in a.ndata:
            assert torch.equal(a.ndata[k], b.ndata[k]) and a.ndata[k].dtype == b.ndata[k].dtype
        assert torch.equal(a.edata["pose"], b.edata["pose"])
    sel, _ = m.load_graphs(path, [2, 0])
    assert [g.num_nodes() for g in sel] == [4, 3]
    assert m.unbatch(m.batch(back))[1].num_edges() == graphs[1].num_edges()
    # a file with DGL's magic goes to the DGL-format reader (tests/test_dgl_format.py), which
    # rejects this one (version 0) with a clear error; anything else that is not ours is refused
    foreign = tmp_path / "dgl_written.bin"
    foreign.write_bytes(b"\x3f\xa1\xb4\x46\xf0\x4f\x2e\xdd" + bytes(64))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        with pytest.raises(ValueError, match="DGL graph file version 0"):
            m.load_graphs(str(foreign))
    foreign.write_bytes(b"not a cache at all")
    with pytest.raises(ValueError, match="not an mrp_gnn graph cache"):
        m.load_graphs(str(foreign))


def test_dataset_lifecycle_like_the_reference(tmp_path):
    """A subclass shaped like MultiViewDGLDataset (dgl/dataloader.py:15-202): processes and saves on
    the first construction, loads the cache on the second; a foreign cache is rebuilt."""
    with m.compat.reference_class_path():
        from dgl import load_graphs, save_graphs
        from dgl.data import DGLDataset
    calls = []

    class Frames(DGLDataset):
        def __init__(self, save_dir):
            super().__init__(name="FlightmareDGL", raw_dir=str(tmp_path / "raw"), save_dir=save_dir)

        def process(self):
            calls.append("process")
            self.graphs = [m.complete_graph(4) for _ in range(3)]
            for g in self.graphs:
                g.ndata["image"] = torch.ones(4, 2)

        def path(self):
            return os.path.join(self.save_dir, "dgl_graph_4.bin")

        def save(self):
            calls.append("save")
            save_graphs(self.path(), self.graphs)

        def load(self):
            calls.append("load")
            self.graphs, _ = load_graphs(self.path())

        def has_cache(self):
            return os.path.exists(self.path())

        def __getitem__(self, i):
            return self.graphs[i]

        def __len__(self):
            return len(self.graphs)

    d1 = Frames(str(tmp_path / "proc"))
    d2 = Frames(str(tmp_path / "proc"))
    assert calls == ["process", "save", "load"]
    assert len(d2) == 3 and d2[1].num_edges() == 12 and torch.equal(d2[2].ndata["image"], torch.ones(4, 2))
    assert d1.save_dir == str(tmp_path / "proc") and d1.name == "FlightmareDGL"
    (tmp_path / "proc" / "dgl_graph_4.bin").write_bytes(b"not ours")
    calls.clear()
    Frames(str(tmp_path / "proc"))
    assert calls == ["load", "process", "save"]
