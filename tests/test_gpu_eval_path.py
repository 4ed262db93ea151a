"""The inference path end to end: what the reference's eval loop runs (``torch.no_grad()`` around
``model(data)``, ``dgl/eval.py:184-198``, ``dgl/training.py:225-240``) and what ``bench.py`` times —
``GCN.forward`` with no gradient wanted, i.e. the one-launch split-bf16 edge encoder
(``mrp_edge_encoder_fwd_split``) -> logits -> sigmoid inside the aggregation kernel -> ``film_fwd``.

* against the reference's own golden fixture (its ``GCN``/``edge_encoder`` modules, stub-imported by
  ``tests/golden/make_golden.py``) at 1e-5, the north-star tolerance;
* at the headline workload (B = 32 complete 8-robot graphs, C = 512, 32 x 32) against a float64
  restatement of the reference's op sequence (``stack_ref``), with the fp32-restatement yardstick;
* the encoder's column sums at C = 2048 (the accumulation of 128 16-k steps per output): the check
  that exposed a biased single-accumulator sum in the compress GEMMs;
* the train (autograd: hidden kernel + fp32-MFMA logits) and eval (split-bf16) encoders on the same
  weights: both within the yardstick, and their mutual difference stated.
Every test asserts the split kernel actually ran (``encoder.PATH_COUNTS``)."""
import types

import numpy as np
import pytest
import torch

import mrp_gnn_amd as m
import stack_ref
from conftest import load_golden, rel_err
from test_gpu_parity import PARAM_KEYS, graph_from

pytestmark = pytest.mark.gpu


def _split_calls():
    return m.encoder.PATH_COUNTS["split"]


def test_eval_gcn_matches_reference_fixture(cuda_device):
    """No-grad GCN.forward on the C = 32 fixture (complete 5-robot graphs, 8 x 8, batch 3) with the
    reference's parameters reproduces the reference GCN's aggregate at 1e-5 — through the split
    encoder (C % 32 == 0), not the training path."""
    z = load_golden("complete_n5_c32_8x8_b3")
    C = z["x"].shape[1]
    assert C % 32 == 0
    g = graph_from(z["src"], z["dst"], z["batch_num_nodes"])
    g.ndata["image"] = torch.from_numpy(z["x"])
    g.edata["pose"] = torch.from_numpy(z["pose"])
    g = g.to(cuda_device)
    gcn = m.GCN(types.SimpleNamespace(feature_dim=C, gcn_mode=str(z["mode"])))
    gcn.load_state_dict({"edge_encoder." + k: torch.from_numpy(z["param." + k]) for k in PARAM_KEYS})
    gcn = gcn.to(cuda_device)
    before = _split_calls()
    with torch.no_grad():
        out = gcn(g)
    torch.cuda.synchronize()
    assert _split_calls() == before + 1, "the no-grad forward did not take the split-bf16 encoder"
    assert rel_err(out.cpu().numpy(), z["out"]) <= 1e-5


def _headline_graph(device, B=32, N=8, C=512, H=32, seed=11):
    rng = np.random.RandomState(seed)
    graphs = []
    for _ in range(B):
        t = rng.uniform(-10, 10, size=(N, 3))
        q = rng.standard_normal((N, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        graphs.append(m.frame_graph(np.concatenate([t, q], 1).astype(np.float32)))
    g = m.batch(graphs)
    gen = torch.Generator().manual_seed(seed)
    g.ndata["image"] = torch.randn(B * N, C, H, H, generator=gen)
    return g.to(device)


def test_eval_headline_vs_float64(cuda_device):
    """The benchmarked step itself (bench.py: no-grad GCN.forward, B = 32, N = 8, C = 512, 32 x 32)
    against the reference's op sequence in float64: as accurate as the same sequence run in fp32."""
    C = 512
    g = _headline_graph(cuda_device, C=C)
    torch.manual_seed(0)
    gcn = m.GCN(types.SimpleNamespace(feature_dim=C)).to(cuda_device)
    x = g.ndata["image"]
    before = _split_calls()
    with torch.no_grad():
        out = gcn(g, x)
    torch.cuda.synchronize()
    assert _split_calls() == before + 1
    params = {"enc." + k: v.detach() for k, v in gcn.edge_encoder.named_parameters()}
    src, dst = (t.to(cuda_device).long() for t in g.edges())
    pose = g.edata["pose"]
    with torch.no_grad():
        f32 = stack_ref.aggregate(x, stack_ref.edge_gb(params, "enc.", pose), src, dst)
        p64 = {k: v.double() for k, v in params.items()}
        f64 = stack_ref.aggregate(x.double(), stack_ref.edge_gb(p64, "enc.", pose.double()), src, dst)
    ok, errs = stack_ref.within(out, f32, f64)
    assert ok, errs
    del f32, f64
    torch.cuda.empty_cache()


def _col_sum_err(z, z64):
    s, s64 = z.double().sum(0), z64.sum(0)
    return float((s - s64).abs().max() / s64.abs().max())


@pytest.mark.parametrize("E,C", [(448, 2048), (1792, 512), (512, 1024)])
def test_split_encoder_column_sums(cuda_device, E, C):
    """Column sums of z over the edges (what db2 and every per-channel sum downstream see) from the
    split encoder are as accurate as fp32's: a single accumulator for all six partial products biased
    such sums in the compress GEMMs (6x the fp32 error); the encoder keeps a0 b0 apart likewise."""
    torch.manual_seed(C + E)
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 8).to(cuda_device)
    before = _split_calls()
    with torch.no_grad():
        z = m.encoder.edge_logits(enc.layers, pose)
        p64 = [t.detach().double() for t in enc.parameters()]
        z64 = torch.nn.functional.linear(torch.relu(torch.nn.functional.linear(pose.double(), p64[0], p64[1])),
                                         p64[2], p64[3])
        h32 = torch.relu(torch.nn.functional.linear(pose, enc.layers[0].weight, enc.layers[0].bias))
        z32 = torch.nn.functional.linear(h32, enc.layers[2].weight, enc.layers[2].bias)
    assert _split_calls() == before + 1
    e_split, e_f32 = _col_sum_err(z, z64), _col_sum_err(z32, z64)
    assert e_split <= max(1e-6, 4.0 * e_f32), (e_split, e_f32)
    ok, errs = stack_ref.within(z, z32, z64)
    assert ok, errs


@pytest.mark.parametrize("E,C", [(1792, 512), (448, 2048), (100, 64)])
def test_train_and_eval_encoders_agree(cuda_device, E, C):
    """Train and eval logits of the same weights.  Where E % 32 == 0 (every reference configuration)
    training runs the same split-bf16 kernel (EdgeEncoderSplitFunction), so the two are bit-identical;
    otherwise training runs that kernel on zero-padded edges (EdgeEncoderPaddedFunction, possibly in
    another workgroup form than the unpadded eval launch), and then each is within the float64
    yardstick, so they differ by at most the sum of two fp32-level errors — stated here."""
    torch.manual_seed(3 * C + E)
    enc = m.edge_encoder([C, C]).to(cuda_device)
    pose = (torch.randn(E, 9) * 8).to(cuda_device)
    before = dict(m.encoder.PATH_COUNTS)
    with torch.no_grad():
        z_eval = m.encoder.edge_logits(enc.layers, pose)
    z_train = m.encoder.edge_logits(enc.layers, pose)
    assert z_train.requires_grad
    assert m.encoder.PATH_COUNTS["split"] == before.get("split", 0) + 1
    split_train = E % 32 == 0
    key = "split_train" if split_train else "split_padded"
    assert m.encoder.PATH_COUNTS[key] == before.get(key, 0) + 1
    if split_train:
        assert torch.equal(z_eval, z_train.detach())
    with torch.no_grad():
        p64 = [t.detach().double() for t in enc.parameters()]
        z64 = torch.nn.functional.linear(torch.relu(torch.nn.functional.linear(pose.double(), p64[0], p64[1])),
                                         p64[2], p64[3])
        z32 = enc.layers[2](torch.relu(enc.layers[0](pose)))
    e_f32 = stack_ref.err(z32, z64)
    for z in (z_eval, z_train.detach()):
        ok, errs = stack_ref.within(z, z32, z64)
        assert ok, errs
    diff = stack_ref.err(z_eval, z_train.detach()) * float(z_train.abs().max()) / float(z64.abs().max())
    assert diff <= 2 * max(1e-5, 4.0 * e_f32), (diff, e_f32)


def _forward(gcn, g, x, own_stream):
    m.encoder.set_encoder_stream(own_stream)
    try:
        with torch.no_grad():
            return gcn(g, x).clone()
    finally:
        m.encoder.set_encoder_stream(True)


def test_encoder_stream_ordered_after_input_writes(cuda_device):
    """The inference encoder runs on its own stream (``encoder.set_encoder_stream``, the default), ordered
    after the producers of what it reads, not after everything queued before it.  Its results are the
    caller's-stream results bit for bit; in-place writes to the poses and to the weights (an optimizer
    step), queued behind long kernels on the caller's stream, are seen by the next forward; and under
    stream capture the layer records on one stream and replays to the same bits."""
    C = 64
    g = _headline_graph(cuda_device, B=6, C=C, H=16)
    torch.manual_seed(2)
    gcn = m.GCN(types.SimpleNamespace(feature_dim=C)).to(cuda_device)
    x = g.ndata["image"]
    a, b = _forward(gcn, g, x, True), _forward(gcn, g, x, False)
    assert torch.equal(a, b)
    busy = torch.randn(64 << 20, device=cuda_device)  # 256 MB: keeps the caller's stream busy

    def stall():
        for _ in range(4):
            busy.mul_(1.0)

    # poses written in place (a version bump) behind the stall
    pose = g.edata["pose"]
    with torch.no_grad():
        stall()
        pose.mul_(1.25)
    c = _forward(gcn, g, x, True)
    assert torch.equal(c, _forward(gcn, g, x, False)) and not torch.equal(c, a)
    # every weight updated in place behind the stall, as an optimizer step would
    with torch.no_grad():
        stall()
        for p in gcn.parameters():
            p.mul_(0.75)
    d = _forward(gcn, g, x, True)
    assert torch.equal(d, _forward(gcn, g, x, False)) and not torch.equal(d, c)
    # only b2 changed: it is not in the packed image's key, its own readiness event orders it
    with torch.no_grad():
        stall()
        gcn.edge_encoder.layers[2].bias.add_(0.5)
    e = _forward(gcn, g, x, True)
    assert torch.equal(e, _forward(gcn, g, x, False)) and not torch.equal(e, d)
    # the features written in place behind the stall
    with torch.no_grad():
        stall()
        x.mul_(1.5)
    f = _forward(gcn, g, x, True)
    assert torch.equal(f, _forward(gcn, g, x, False)) and not torch.equal(f, e)
    # back-to-back calls (each encoder running ahead beside the previous aggregation), each as on the
    # caller's stream
    with torch.no_grad():
        runs = [gcn(g, x * (1.0 + 0.1 * i)) for i in range(4)]
        refs = []
        m.encoder.set_encoder_stream(False)
        try:
            refs = [gcn(g, x * (1.0 + 0.1 * i)) for i in range(4)]
        finally:
            m.encoder.set_encoder_stream(True)
    assert all(torch.equal(a_, b_) for a_, b_ in zip(runs, refs))
    e = f
    # stream capture: one stream, replayed
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.stream(side):
        gcn(g, x)  # warm the allocator and the packed image outside the capture
        torch.cuda.current_stream().synchronize()
        with torch.cuda.graph(graph, stream=side):
            out = gcn(g, x)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, e)
