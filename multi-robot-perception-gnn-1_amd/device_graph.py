"""Per-frame robot graphs built on the GPU (``mrp_frame_graph_build``, ``csrc/frame_graph.hip``).

The reference builds every frame's graph on the host while it prepares the dataset:
the complete edge list (``dgl/dataloader.py:88-95``), one ``cal_relative_pose`` per edge
(``dgl/dataloader.py:116-122``, ``dgl/utils.py:54-77``), then ``dgl.batch`` in the collate
(``dgl/training.py:57-58``).  :func:`frame_batch` does the same for a whole batch in one kernel
launch from the robots' poses already on the device: edge features, the kernels' CSR and the
graph offsets come out in device memory, with no host loop and no host-to-device copy per batch.

The result is an ordinary :class:`~graph.RobotGraph` (``ndata``/``edata``, ``local_scope``, ``to``,
``csr``); its host edge list is only produced (one device-to-host copy) if something asks for it.
Edge poses are bit-identical to :func:`graph.frame_graph` on float32 poses, and the k-NN edges are
those of :func:`graph.knn_edges` (tested in ``tests/test_gpu_frame_graph.py``).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import _lib
from .graph import GraphCSR, RobotGraph, complete_edges


def _complete_host_edges(B: int, n: int):
    cs, cd = (np.asarray(t, dtype=np.int64) for t in complete_edges(n))
    off = (np.arange(B, dtype=np.int64) * n)[:, None]
    return (cs[None] + off).reshape(-1), (cd[None] + off).reshape(-1)


def frame_batch(poses: torch.Tensor, knn: Optional[int] = None, stream=None) -> RobotGraph:
    """A batch of per-frame graphs built on the device.

    ``poses``: (B, n, 7) float32 CUDA tensor, rows ``(tx, ty, tz, qx, qy, qz, qw)``; n <= 16.
    ``knn=None``: the reference's complete graphs (edge order of ``dgl.batch`` over
    ``dgl/dataloader.py:88-95`` frames); ``knn=k``: k-NN(k) graphs (edges destination-major,
    sources ascending, as :func:`graph.knn_edges`).  Sets ``edata['pose']`` (E, 9) on the device.
    """
    if not poses.is_cuda:
        raise RuntimeError("frame_batch builds graphs on the GPU; use graph.frame_graph + graph.batch on the host")
    if poses.dim() != 3 or poses.shape[-1] != 7:
        raise ValueError(f"poses must be (B, n, 7), got {tuple(poses.shape)}")
    B, n = int(poses.shape[0]), int(poses.shape[1])
    if n > _lib.MAX_NODES:
        raise ValueError(f"{n} robots per frame; the kernels support up to {_lib.MAX_NODES}")
    k = 0 if knn is None else int(knn)
    if knn is not None and not 1 <= k < n:
        raise ValueError(f"knn={k} needs 1 <= k < n={n}")
    poses = poses.detach().to(torch.float32).contiguous()
    dev = poses.device
    nt = B * n
    ne = nt * k if k else nt * max(n - 1, 0)
    i32 = dict(dtype=torch.int32, device=dev)
    edge_pose = torch.empty(ne, 9, dtype=torch.float32, device=dev)
    indptr = torch.empty(nt + 1, **i32)
    src = torch.empty(ne, **i32)
    eid = torch.empty(ne, **i32)
    goff = torch.empty(B + 1, **i32)
    lib = _lib.load_library()
    st = (stream if stream is not None else torch.cuda.current_stream(dev)).cuda_stream
    with torch.cuda.device(dev):
        _lib.check(lib.mrp_frame_graph_build(poses.data_ptr(), B, n, k, edge_pose.data_ptr(), indptr.data_ptr(),
                                             src.data_ptr(), eid.data_ptr(), goff.data_ptr(), st),
                   "mrp_frame_graph_build")
    if k == 0:
        kind = _lib.GRAPH_COMPLETE
        edge_fn = lambda: _complete_host_edges(B, n)  # noqa: E731  (arithmetic, no device copy)
    else:
        kind = _lib.graph_regular(k) if k <= _lib.MAX_REGULAR_K else _lib.GRAPH_CSR
        # edges are destination-major: edge e goes to node e // k; src (CSR order) is in edge order
        edge_fn = lambda: (src.cpu().numpy().astype(np.int64), np.arange(ne, dtype=np.int64) // k)  # noqa: E731
    csr = GraphCSR(indptr, src, eid, goff, B, n, nt, ne, kind)
    g = RobotGraph._from_device(edge_fn, nt, ne, [n] * B, [ne // B if B else 0] * B, csr=csr, device=dev,
                                complete=(k == 0 and n >= 1) if B else False, kdeg=(k if k else (n - 1 if n > 1 else 0)))
    # the same arrays are a valid CSR description under the other graph kinds too
    kdeg = k if k else n - 1
    g._csr_cache.setdefault((str(dev), _lib.GRAPH_CSR), csr._replace(graph_kind=_lib.GRAPH_CSR))
    if 1 <= kdeg <= _lib.MAX_REGULAR_K:
        g._csr_cache.setdefault((str(dev), _lib.graph_regular(kdeg)), csr._replace(graph_kind=_lib.graph_regular(kdeg)))
    g.edata["pose"] = edge_pose
    return g
