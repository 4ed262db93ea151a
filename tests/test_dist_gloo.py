"""CPU, world_size 2 over gloo: graph sharding and the bucketed gradient all-reduce give the
single-process full-batch gradients (the multi-GPU path minus RCCL)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mrp_gnn_amd.dist import GradAllReducer, shard, shard_range


def test_shard_range_partitions():
    for n in range(0, 40):
        for w in range(1, 9):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1
    assert shard(list(range(10)), 1, 3) == [4, 5, 6]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(9, 16), torch.nn.ReLU(), torch.nn.Linear(16, 32),
                               torch.nn.Sigmoid(), torch.nn.Linear(32, 3))


def _worker(rank, world, port, bucket_bytes):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(123)
        data = torch.randn(8, 9)
        target = torch.randn(8, 3)
        # single-process reference on the full batch
        ref = _model()
        torch.nn.functional.mse_loss(ref(data), target).backward()
        # data-parallel: each rank its contiguous shard, grads averaged by the reducer
        model = _model()
        red = GradAllReducer(model.parameters(), bucket_bytes=bucket_bytes)
        lo, hi = shard_range(8, rank, world)
        for _ in range(2):  # twice: the reducer must re-arm after synchronize()
            model.zero_grad(set_to_none=True)
            torch.nn.functional.mse_loss(model(data[lo:hi]), target[lo:hi]).backward()
            red.synchronize()
            for p, q in zip(model.parameters(), ref.parameters()):
                assert torch.allclose(p.grad, q.grad, rtol=1e-5, atol=1e-6), (rank, p.shape)
        assert len(red.buckets) >= (2 if bucket_bytes < 1024 else 1)
        red.remove()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket_bytes", [256, 32 << 20])
def test_grad_allreduce_world2_matches_full_batch(bucket_bytes):
    mp.spawn(_worker, args=(2, _free_port(), bucket_bytes), nprocs=2, join=True)


def _gcn_params(C):
    torch.manual_seed(5)
    import mrp_gnn_amd as m
    opt = type("opt", (), {"feature_dim": C, "compress_gcn": True, "multi_gcn": False})()
    blk = m.GCNBlock(opt)
    return {k: v.detach().clone() for k, v in blk.named_parameters()}


def _block_loss(params, g):
    """mean((conv1(cat(x, gcn1(x))))^2) with the CPU oracle for the GCN layer
    (dgl/model/models.py:180-184): the edge encoder and conv1 parameters are the leaves."""
    import oracle
    enc = {k[len("gcn1.edge_encoder."):]: v for k, v in params.items() if k.startswith("gcn1.edge_encoder.")}
    x = g.ndata["image"]
    src, dst = (t.numpy() for t in g.edges())
    agg = oracle.film_aggregate(x, oracle.edge_encoder_forward(enc, g.edata["pose"]), src, dst)
    h = torch.nn.functional.conv2d(torch.cat((x, agg), 1), params["conv1.weight"], params["conv1.bias"])
    return h.square().mean()


def _frames(B, N, C, seed):
    import numpy as np

    import mrp_gnn_amd as m
    rng = np.random.RandomState(seed)
    frames = []
    for _ in range(B):
        poses = np.concatenate([rng.uniform(-5, 5, (N, 3)), rng.standard_normal((N, 4))], 1).astype(np.float32)
        f = m.frame_graph(poses)
        f.ndata["image"] = torch.from_numpy(rng.standard_normal((N, C, 4, 4)).astype(np.float32))
        frames.append(f)
    return m.batch(frames)


def _gcn_worker(rank, world, port, B):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mrp_gnn_amd.dist import shard_graph
        C = 8
        g = _frames(B, 4, C, seed=11)
        # full batch on one process: the reference gradient
        ref = {k: v.clone().requires_grad_(True) for k, v in _gcn_params(C).items()}
        _block_loss(ref, g).backward()
        # this rank's graphs only, gradients reduced (weighted by graph count: uneven shards)
        params = {k: torch.nn.Parameter(v.clone()) for k, v in _gcn_params(C).items()}
        red = GradAllReducer(params.values(), bucket_bytes=4096)
        sub, (lo, hi) = shard_graph(g, rank, world)
        assert sub.batch_size == hi - lo and sub.num_nodes() == 4 * (hi - lo)
        assert torch.equal(sub.ndata["image"], g.ndata["image"][4 * lo:4 * hi])
        for _ in range(2):
            for p in params.values():
                p.grad = None
            red.set_local_count(hi - lo)
            _block_loss(params, sub).backward()
            red.synchronize()
            for k in params:
                assert torch.allclose(params[k].grad, ref[k].grad, rtol=1e-5, atol=1e-7), (rank, k)
        red.remove()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [4, 5])
def test_gcn_layer_grads_world2_sharded_batch(B):
    """The GCN layer's parameters (edge encoder + 1x1 compress) trained data-parallel over a
    sharded RobotGraph batch: the reduced gradients equal the full-batch ones, including an
    uneven split (B=5 over 2 ranks: 3 + 2 graphs)."""
    mp.spawn(_gcn_worker, args=(2, _free_port(), B), nprocs=2, join=True)


def _accum_worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _model()
        red = GradAllReducer(model.parameters())
        data = torch.randn(4, 9)
        model(data).sum().backward()
        with pytest.raises(RuntimeError, match="synchronize"):
            model(data).sum().backward()  # a second backward before synchronize()
    finally:
        dist.destroy_process_group()


def test_second_backward_before_synchronize_raises():
    mp.spawn(_accum_worker, args=(2, _free_port()), nprocs=2, join=True)


def _stack_params(C, layers):
    torch.manual_seed(9)
    import mrp_gnn_amd as m
    opt = type("opt", (), {"feature_dim": C, "compress_gcn": True, "multi_gcn": False, "gcn_layers": layers,
                           "gcn_combine": "cat_compress"})()
    return {k: v.detach().clone() for k, v in m.GCNStack(opt).named_parameters()}


def _stack_loss(params, g, layers):
    """mean(stack(x)^2) for a k-layer cat_compress stack with the CPU oracle per layer
    (dgl/model/models.py:180-189 generalised): gcn_i's edge encoder and conv_i are the leaves."""
    import oracle
    h = g.ndata["image"]
    src, dst = (t.numpy() for t in g.edges())
    for i in range(1, layers + 1):
        pre = f"gcn{i}.edge_encoder."
        enc = {k[len(pre):]: v for k, v in params.items() if k.startswith(pre)}
        agg = oracle.film_aggregate(h, oracle.edge_encoder_forward(enc, g.edata["pose"]), src, dst)
        h = torch.nn.functional.conv2d(torch.cat((h, agg), 1), params[f"conv{i}.weight"], params[f"conv{i}.bias"])
    return h.square().mean()


def _knn_frames(B, N, C, k, seed):
    import numpy as np

    import mrp_gnn_amd as m
    rng = np.random.RandomState(seed)
    frames = []
    for _ in range(B):
        poses = np.concatenate([rng.uniform(-5, 5, (N, 3)), rng.standard_normal((N, 4))], 1).astype(np.float32)
        f = m.frame_graph(poses, knn=k)
        f.ndata["image"] = torch.from_numpy(rng.standard_normal((N, C, 4, 4)).astype(np.float32))
        frames.append(f)
    return m.batch(frames)


def _overlap_worker(rank, world, port):
    """configs[4]'s stack at reduced size (3 layers, k-NN(4) graphs of 16 robots, C=8): the reduced
    gradients equal the full batch's, and backward launches a bucket's all-reduce before the last
    parameter's gradient lands (the all-reduce overlaps the rest of backward)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mrp_gnn_amd.dist import shard_graph
        C, L = 8, 3
        g = _knn_frames(5, 16, C, 4, seed=21)
        ref = {k: v.clone().requires_grad_(True) for k, v in _stack_params(C, L).items()}
        _stack_loss(ref, g, L).backward()
        params = {k: torch.nn.Parameter(v.clone()) for k, v in _stack_params(C, L).items()}
        # registration order = the stack's parameter order; buckets of ~one layer's gradients
        red = GradAllReducer(params.values(), bucket_bytes=4 * (2 * C * C + 12 * C + 2 * C * C + C))
        assert len(red.buckets) >= 3
        sub, (lo, hi) = shard_graph(g, rank, world)
        red.set_local_count(hi - lo)
        _stack_loss(params, sub, L).backward()
        red.synchronize()
        ev = red.last_events
        last_grad = max(i for i, (e, _) in enumerate(ev) if e == "grad")
        first_launch = min(i for i, (e, _) in enumerate(ev) if e == "launch")
        assert first_launch < last_grad, ev  # a bucket went out while backward was still producing grads
        assert sum(1 for e, _ in ev if e == "launch") == len(red.buckets)
        for k in params:
            assert torch.allclose(params[k].grad, ref[k].grad, rtol=1e-5, atol=1e-7), (rank, k)
        red.remove()
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_overlaps_backward_three_layer_stack():
    mp.spawn(_overlap_worker, args=(2, _free_port()), nprocs=2, join=True)


def _empty_shard_worker(rank, world, port):
    """More ranks than graphs (a DataLoader's short last batch): the empty rank's NaN mean loss must
    not poison the reduced gradient."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mrp_gnn_amd.dist import shard_graph
        C = 8
        g = _frames(1, 4, C, seed=3)
        ref = {k: v.clone().requires_grad_(True) for k, v in _gcn_params(C).items()}
        _block_loss(ref, g).backward()
        params = {k: torch.nn.Parameter(v.clone()) for k, v in _gcn_params(C).items()}
        red = GradAllReducer(params.values())
        sub, (lo, hi) = shard_graph(g, rank, world)
        assert (hi - lo) == (1 if rank == 0 else 0)
        red.set_local_count(hi - lo)
        loss = _block_loss(params, sub)
        if rank == 1:
            assert torch.isnan(loss)  # mean over zero graphs
        loss.backward()
        red.synchronize()
        for k in params:
            assert torch.isfinite(params[k].grad).all(), (rank, k)
            assert torch.allclose(params[k].grad, ref[k].grad, rtol=1e-5, atol=1e-7), (rank, k)
        red.remove()
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_world2_batch1_empty_shard():
    mp.spawn(_empty_shard_worker, args=(2, _free_port()), nprocs=2, join=True)


class _MatW(torch.autograd.Function):
    """y = x W^T whose weight gradient is written where ``dist.grad_out_like`` says (as the HIP
    backward kernels do): into the reducer's bucket slot."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x.mm(w.t())

    @staticmethod
    def backward(ctx, gy):
        from mrp_gnn_amd.dist import grad_out_like
        x, w = ctx.saved_tensors
        dw = grad_out_like(w)
        if dw is None:
            dw = torch.empty_like(w)
        torch.mm(gy.t(), x, out=dw)
        return gy.mm(w), dw


def _views_worker(rank, world, port):
    """Gradients live in the reducer's flat buckets (p.grad are views of them): no per-step
    concatenation or copy back; a gradient written through grad_out_like is adopted with no copy at
    all; one autograd allocated is copied into its slot once; zero_grad(set_to_none=False)
    accumulates straight into the views (no copy).  Results equal the full-batch gradients."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(7)
        data, target = torch.randn(8, 9), torch.randn(8, 5)
        w_ref = torch.randn(5, 9)
        lin_ref = torch.nn.Linear(9, 9)
        ref_w = w_ref.clone().requires_grad_(True)
        lin_r = torch.nn.Linear(9, 9)
        lin_r.load_state_dict(lin_ref.state_dict())
        torch.nn.functional.mse_loss(_MatW.apply(lin_r(data), ref_w), target).backward()
        w = torch.nn.Parameter(w_ref.clone())
        lin = torch.nn.Linear(9, 9)
        lin.load_state_dict(lin_ref.state_dict())
        params = [w] + list(lin.parameters())
        red = GradAllReducer(params, bucket_bytes=1 << 20)
        assert len(red.buckets) == 1
        flat = red._flat[0]
        lo, hi = shard_range(8, rank, world)

        def in_bucket(t):
            base = flat.data_ptr()
            return base <= t.data_ptr() < base + flat.numel() * flat.element_size()

        for step in range(3):
            before = red.copies
            if step < 2:
                for p in params:
                    p.grad = None
            else:
                for p in params:
                    p.grad.zero_()  # zero_grad(set_to_none=False): accumulate into the views
            red.arm()  # slots are handed to the kernels only for the backward the reducer reduces
            torch.nn.functional.mse_loss(_MatW.apply(lin(data[lo:hi]), w), target[lo:hi]).backward()
            red.synchronize()
            copies = red.copies - before
            # the Linear's two gradients are allocated by autograd (copied once each) unless they
            # already are the views; w's is written in its slot by the backward itself
            assert copies == (2 if step < 2 else 0), (step, copies)
            for p in params:
                assert in_bucket(p.grad), step
            assert torch.allclose(w.grad, ref_w.grad, rtol=1e-5, atol=1e-6)
            for p, q in zip(lin.parameters(), lin_r.parameters()):
                assert torch.allclose(p.grad, q.grad, rtol=1e-5, atol=1e-6)
        red.remove()
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_bucket_views_world2():
    mp.spawn(_views_worker, args=(2, _free_port()), nprocs=2, join=True)


def _slot_rules_worker(rank, world, port):
    """every slot is SLOT_ALIGN-byte aligned whatever precedes it in the bucket; slots go
    to kernels only while armed; non-fp32 parameters never get one; a slot a kernel declined is given
    back; arming re-keys on moved storage and raises on a device / dtype change."""
    from mrp_gnn_amd.dist import grad_out_like, release_grad_out
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # odd numels first in backward order (registration order reversed): the decoder-before-encoder
        # layout of multi_view_dgl_model, whose last conv bias has num_classes + 1 elements
        enc = torch.nn.Parameter(torch.randn(64, 9))
        odd = [torch.nn.Parameter(torch.randn(n)) for n in (3, 5, 7)]
        half = torch.nn.Parameter(torch.randn(8).half())
        params = [enc] + odd
        red = GradAllReducer(params + [half], bucket_bytes=1 << 20)
        for p in params:  # relative to the bucket's base (torch's GPU allocator aligns it to >= 512 B)
            base = red._flat[red._bucket_of[id(p)]].data_ptr()
            assert (red.view(p).data_ptr() - base) % GradAllReducer.SLOT_ALIGN == 0
        assert grad_out_like(enc) is None  # not armed
        red.arm()
        assert grad_out_like(half) is None  # fp16: the HIP kernels write fp32
        v = grad_out_like(enc)
        assert v is not None and v.data_ptr() == red.view(enc).data_ptr()
        assert grad_out_like(enc) is None  # once per step
        release_grad_out(enc, v)  # the kernel declined: the slot is free again
        v2 = grad_out_like(enc)
        assert v2 is not None and v2.data_ptr() == v.data_ptr()
        loss = (enc.sum() + sum(p.sum() for p in odd) + half.float().sum()) * (rank + 1)
        loss.backward()
        red.synchronize()
        assert grad_out_like(odd[0]) is None  # disarmed by synchronize()
        for p in params:
            assert torch.allclose(p.grad, torch.full_like(p, 1.5))
        # storage moved in place (e.g. model.to() onto the same device re-allocating): re-keyed on arm
        enc.data = enc.data.clone()
        for p in params + [half]:
            p.grad = None
        red.arm()
        assert grad_out_like(enc) is not None
        red.synchronize()
        enc.data = enc.data.double()
        with pytest.raises(RuntimeError, match="re-cast"):
            red.arm()
        red.remove()
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_slot_rules_world2():
    mp.spawn(_slot_rules_worker, args=(2, _free_port()), nprocs=2, join=True)


def test_bench_self_launch_command():
    """bench.py --gpus N (no launcher around it) starts N ranks itself: torch.distributed.run on
    127.0.0.1, one process per GPU, the same arguments, WORLD_SIZE left to the launcher."""
    import importlib.util
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    os.environ["WORLD_SIZE"] = "3"
    try:
        cmd, env = bench.launcher_command(["--gpus", "4", "--steps", "5"], 4, 29555)
    finally:
        del os.environ["WORLD_SIZE"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-port=29555" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-3:] == ["--gpus", "4", "--steps", "5"][-3:] and cmd[-4] == "--gpus"
    assert os.path.basename(cmd[cmd.index("--master-port=29555") + 1]) == "bench.py"
    assert "WORLD_SIZE" not in env and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    args = bench.parse_args(["--gpus", "2", "--dist-backend", "gloo"])
    assert args.gpus == 2 and args.dist_backend == "gloo"


def _premul_worker(rank, world, port):
    """The RCCL path's scale fold, run over gloo: the backend query answers "nccl", RCCL's
    pre-multiplied-sum op is stood in for by a marker that the all-reduce wrapper applies (as the
    collective would, inside its own pass), and the reducer must hand the collective UNSCALED buckets
    with its n_r / N in the op — no pass over a bucket before its all-reduce."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    real_all_reduce, real_backend = dist.all_reduce, dist.get_backend
    seen = []

    def all_reduce(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
        if isinstance(op, tuple) and op[0] == "premul":
            seen.append((t.clone(), op[1]))
            t.mul_(op[1])  # what RCCL's pre-multiplied sum does inside the collective
            op = dist.ReduceOp.SUM
        return real_all_reduce(t, op=op, group=group, async_op=async_op)

    try:
        dist.get_backend = lambda group=None: "nccl"
        dist._make_nccl_premul_sum = lambda factor: ("premul", factor)
        dist.all_reduce = all_reduce
        torch.manual_seed(321)
        data, target = torch.randn(7, 9), torch.randn(7, 3)
        ref = _model()
        torch.nn.functional.mse_loss(ref(data), target).backward()
        lo, hi = shard_range(7, rank, world)  # 4 + 3 rows: uneven shards
        local = _model()
        torch.nn.functional.mse_loss(local(data[lo:hi]), target[lo:hi]).backward()
        model = _model()
        red = GradAllReducer(model.parameters(), bucket_bytes=512)
        scale = red.set_local_count(hi - lo)
        assert abs(scale - (hi - lo) / 7) < 1e-12
        torch.nn.functional.mse_loss(model(data[lo:hi]), target[lo:hi]).backward()
        red.synchronize()
        assert red.scaled_passes_skipped == len(red.buckets) >= 2
        # every bucket reached the collective unscaled, with this rank's scale in the op
        local_grads = {id(p): q.grad for p, q in zip(model.parameters(), local.parameters())}
        assert len(seen) == len(red.buckets)
        for (flat, factor), bucket in zip(seen, red.buckets):
            assert factor == scale
            for p in bucket:
                bi, off, n = red._slot[id(p)]
                assert torch.equal(flat[off:off + n].view_as(p), local_grads[id(p)])
        for p, q in zip(model.parameters(), ref.parameters()):
            assert torch.allclose(p.grad, q.grad, rtol=1e-5, atol=1e-6), (rank, p.shape)
        red.remove()
    finally:
        dist.all_reduce, dist.get_backend = real_all_reduce, real_backend
        dist.destroy_process_group()


def test_grad_allreduce_scale_rides_in_the_collective():
    mp.spawn(_premul_worker, args=(2, _free_port()), nprocs=2, join=True)


def _arming_worker(rank, world, port):
    """a reducer armed once and then not re-armed warns (once) when gradients take the copy
    path; ``auto_arm=True`` re-arms in every synchronize(), so the kernels keep their in-place slots."""
    import warnings

    from mrp_gnn_amd.dist import grad_out_like
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = torch.nn.Parameter(torch.randn(16, 9))
        red = GradAllReducer([w])
        red.arm()
        w.sum().backward()
        red.synchronize()
        w.grad = None
        with pytest.warns(UserWarning, match="not armed"):
            w.sum().backward()  # not re-armed: the gradient is copied into its slot
            red.synchronize()
        w.grad = None
        with warnings.catch_warnings():
            warnings.simplefilter("error")  # warned once only
            w.sum().backward()
            red.synchronize()
        red.remove()
        v = torch.nn.Parameter(torch.randn(16, 9))
        auto = GradAllReducer([v], auto_arm=True)
        auto.arm()
        for _ in range(3):
            v.grad = None
            slot = grad_out_like(v)  # what a HIP backward kernel asks for: handed out every step
            assert slot is not None and slot.data_ptr() == auto.view(v).data_ptr()
            v.grad = slot.fill_(1.0)
            (v * 0).sum().backward()
            auto.synchronize()
            assert torch.allclose(v.grad, torch.ones_like(v))
        assert auto.copies == 0
        auto.remove()
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_arming_world2():
    mp.spawn(_arming_worker, args=(2, _free_port()), nprocs=2, join=True)
