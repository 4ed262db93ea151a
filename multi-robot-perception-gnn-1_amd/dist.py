"""Multi-GPU data parallelism for the GCN path: one process per GPU, RCCL over xGMI.

Replaces ``torch.nn.DataParallel(model, device_ids=[0, 1])`` (``dgl/training.py:324-325``), the
reference's only parallelism (single process, and it cannot scatter a DGLGraph).

* The graphs of a batch are independent (``dgl.batch`` of per-frame graphs), so the forward and
  the aggregation need no communication: :func:`shard_range` gives each rank a contiguous range
  of graphs (weak scaling when every rank keeps its own batch).
* Parameters are replicated; the only collective is the gradient all-reduce.
  :class:`GradAllReducer` packs gradients into flat buckets in reverse registration order (the
  order backward produces them), launches each bucket's ``all_reduce`` asynchronously from a
  post-accumulate-grad hook as soon as its last gradient lands (overlapping the rest of
  backward), and averages on :meth:`GradAllReducer.synchronize`.  Buckets default to 32 MiB:
  large enough that each ring step over one ~153 GB/s xGMI link is bandwidth- rather than
  latency-bound, few enough that the per-layer edge-encoder (2C^2+12C) and 1x1 compress
  (2C^2+C) gradients of a GCN layer land in one or two buckets.

Averaging: each rank's loss is normally a mean over its own graphs, so with uneven shards
(``shard_range`` of B graphs over P ranks when P does not divide B) the full-batch gradient is
``sum_r (n_r / N) g_r``, not ``(1/P) sum_r g_r``.  :meth:`GradAllReducer.set_local_count` gives the
reducer ``n_r`` (one tiny all-reduce finds ``N``); every bucket is then scaled by ``n_r / N``
before its SUM all-reduce.  Without it the reducer assumes equal shards and scales by ``1/P``.
One backward per :meth:`GradAllReducer.synchronize`: a gradient that lands again after its
bucket's all-reduce was launched (gradient accumulation over several backwards) raises instead
of silently reducing a partial sum.
"""
from __future__ import annotations

import os
from typing import Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist


def env_rank_world() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (defaults 0, 1, 0)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def shard_range(num_items: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) share of ``num_items`` for ``rank`` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(num_items, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def shard(items, rank: int, world: int):
    lo, hi = shard_range(len(items), rank, world)
    return items[lo:hi]


def shard_graph(g, rank: int, world: int):
    """This rank's share of a batched graph (``dgl.batch`` of frames): the contiguous range of
    graphs ``shard_range(g.batch_size, rank, world)`` as a batched graph of its own (node and edge
    ids renumbered from 0, every node/edge feature sliced without a copy).  Returns
    ``(sub_graph, (lo, hi))``.  Replaces what ``DataParallel`` (``dgl/training.py:324-325``) could
    not do: scatter a graph batch."""
    import numpy as np

    from .graph import RobotGraph
    lo, hi = shard_range(g.batch_size, rank, world)
    bnn = [int(v) for v in g.batch_num_nodes().tolist()]
    bne = [int(v) for v in g.batch_num_edges().tolist()]
    noff = np.concatenate([[0], np.cumsum(bnn)]).astype(np.int64)
    eoff = np.concatenate([[0], np.cumsum(bne)]).astype(np.int64)
    n0, n1, e0, e1 = (int(v) for v in (noff[lo], noff[hi], eoff[lo], eoff[hi]))
    src, dst = g.edges()
    sub = RobotGraph(src[e0:e1] - n0, dst[e0:e1] - n0, num_nodes=n1 - n0, batch_num_nodes=bnn[lo:hi],
                     batch_num_edges=bne[lo:hi])
    for k, v in g.ndata.items():
        sub.ndata[k] = v[n0:n1]
    for k, v in g.edata.items():
        sub.edata[k] = v[e0:e1]
    return sub, (lo, hi)


class GradAllReducer:
    """Bucketed, backward-overlapped gradient averaging over a process group."""

    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_bytes: int = 32 << 20,
                 group: Optional[dist.ProcessGroup] = None):
        self.group = group
        self.world = dist.get_world_size(group)
        params = [p for p in params if p.requires_grad]
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in reversed(params):  # backward produces gradients roughly in reverse order
            nbytes = p.numel() * p.element_size()
            if cur and (size + nbytes > bucket_bytes or p.dtype != cur[0].dtype or p.device != cur[0].device):
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self._bucket_of[id(p)] = bi
        self._scale = 1.0 / self.world
        self._empty = False  # this rank holds no graphs this step (set_local_count(0))
        #: (event, bucket) in the order they happen during a backward: ("grad", b) when a parameter's
        #: gradient lands, ("launch", b) when a bucket's all-reduce is started; ``last_events`` is the
        #: record of the last synchronized step — the evidence that the all-reduces overlap backward
        #: (tests/test_dist_gloo.py)
        self.events: List[Tuple[str, int]] = []
        self.last_events: List[Tuple[str, int]] = []
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params]
        self.reset()

    def set_local_count(self, n_local: int) -> float:
        """This rank holds ``n_local`` of the step's graphs (its loss a mean over them): scale its
        gradients by ``n_local / N`` (N = the sum over ranks) so the reduced gradient is the
        full-batch mean even for uneven shards.  Call before backward; returns the scale."""
        t = torch.tensor([float(n_local)], dtype=torch.float64,
                         device=self._device() if dist.get_backend(self.group) == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        total = float(t.item())
        self._scale = float(n_local) / total if total > 0 else 0.0
        # an empty shard (more ranks than graphs, e.g. a DataLoader's short last batch) has a mean loss
        # of 0/0 = NaN: its contribution must be exact zeros, since 0 * NaN would poison every rank
        self._empty = n_local == 0
        return self._scale

    def _device(self):
        for b in self.buckets:
            return b[0].device
        return torch.device("cpu")

    def reset(self) -> None:
        self.events = []
        self._pending = [len(b) for b in self.buckets]
        self._work = [None] * len(self.buckets)
        self._flat = [None] * len(self.buckets)

    def _on_grad(self, p: torch.Tensor) -> None:
        bi = self._bucket_of[id(p)]
        if self._work[bi] is not None:
            raise RuntimeError("GradAllReducer: a gradient landed after its bucket's all-reduce was launched "
                               "(more than one backward before synchronize()); call synchronize() after "
                               "every backward")
        self.events.append(("grad", bi))
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def _launch(self, bi: int) -> None:
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.buckets[bi]]
        flat = torch.cat([g.reshape(-1) for g in grads])
        if self._empty:
            flat.zero_()
        else:
            flat.mul_(self._scale)  # n_r / N (or 1 / P): the SUM all-reduce then yields the average
        self.events.append(("launch", bi))
        self._flat[bi] = flat
        self._work[bi] = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def synchronize(self) -> None:
        """Wait for every bucket (launching any whose hooks did not all fire, e.g. unused
        parameters) and write the averaged gradients back."""
        for bi in range(len(self.buckets)):
            if self._work[bi] is None:
                self._launch(bi)
        for bi, b in enumerate(self.buckets):
            self._work[bi].wait()
            flat = self._flat[bi]
            off = 0
            for p in b:
                n = p.numel()
                g = flat[off:off + n].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
                off += n
        self.last_events = self.events
        self.reset()

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
