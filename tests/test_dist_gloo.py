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
