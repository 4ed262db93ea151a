"""ORACLE (test infrastructure only): the reference's GCN message passing on the CPU, op for op.

What the reference executes for one GCN layer (``dgl/model/models.py:219-226``)::

    gamma, beta = edge_encoder(g.edata['pose'])          # models.py:142-155, 222
    g.update_all(edge_udf, node_udf)                       # models.py:223 (DGL)
        edge_udf: m = gamma * edges.src['image'] + beta    # models.py:210-211
        node_udf: images = mailbox['m'].mean(1)            # models.py:207-208

``update_all`` is DGL's (third-party, absent here).  Restated from its UDF execution path
(DGL >= 0.5, ``dgl.core.invoke_udf_reduce``): messages for all edges at once from gathered
source features; destination nodes grouped by in-degree ("degree bucketing"); for each
non-zero degree d the mailbox is ``(n_d, d, ...)`` with each node's in-edges sorted by edge
id; the reduce UDF runs per bucket; results are scattered back; zero-in-degree nodes keep the
frame's zero initialiser.

Everything is torch on the CPU in fp32 — the reference's own arithmetic — so autograd through
it gives the reference backward too.  It is also the ``cpu_baseline`` of ``bench.py`` ("port").
"""
from __future__ import annotations

from typing import Callable, Dict

import numpy as np
import torch
import torch.nn.functional as F


class _Batch:
    """Minimal EdgeBatch / NodeBatch: the attributes the reference UDFs read."""

    def __init__(self, src=None, data=None, mailbox=None):
        self.src = src
        self.data = data
        self.mailbox = mailbox


def update_all(src: torch.Tensor, dst: torch.Tensor, num_nodes: int, ndata: Dict[str, torch.Tensor],
               edata: Dict[str, torch.Tensor], message_func: Callable, reduce_func: Callable) -> Dict[str, torch.Tensor]:
    """DGL ``update_all(message_func, reduce_func)`` with user-defined functions; returns the new
    node fields (to be merged into ndata by the caller)."""
    src = torch.as_tensor(src, dtype=torch.int64)
    dst = torch.as_tensor(dst, dtype=torch.int64)
    # 1. messages over all edges: edges.src[k] = ndata[k][src]
    ebatch = _Batch(src={k: v.index_select(0, src) for k, v in ndata.items()}, data=edata)
    msgs = message_func(ebatch)
    # 2. degree bucketing
    deg = torch.bincount(dst, minlength=num_nodes)
    eids_by_dst = [[] for _ in range(num_nodes)]
    for e, v in enumerate(dst.tolist()):
        eids_by_dst[v].append(e)  # ascending edge id
    results, nodes = [], []
    for d in sorted(set(deg.tolist())):
        if d == 0:
            continue  # reduce skipped; zero initialiser below
        bucket = [v for v in range(num_nodes) if deg[v] == d]
        eid = torch.tensor([e for v in bucket for e in eids_by_dst[v]], dtype=torch.int64)
        mailbox = {k: m.index_select(0, eid).reshape((len(bucket), d) + tuple(m.shape[1:])) for k, m in msgs.items()}
        results.append(reduce_func(_Batch(mailbox=mailbox)))
        nodes.append(torch.tensor(bucket, dtype=torch.int64))
    out = {}
    if results:
        merged_nodes = torch.cat(nodes)
        for k in results[0]:
            val = torch.cat([r[k] for r in results], 0)
            full = torch.zeros((num_nodes,) + tuple(val.shape[1:]), dtype=val.dtype)
            out[k] = full.index_copy(0, merged_nodes, val)
    return out


def edge_udf(edges):
    """``models.py:210-211``: FiLM message."""
    return {"m": edges.data["pose_gamma"] * edges.src["image"] + edges.data["pose_beta"]}


def copy_u(edges):
    """``fn.copy_u('image', 'm')`` (the commented-out variant, ``models.py:225``)."""
    return {"m": edges.src["image"]}


def node_udf(nodes):
    """``models.py:207-208``: mailbox mean."""
    return {"images": nodes.mailbox["m"].mean(1)}


def node_udf_sum(nodes):
    return {"images": nodes.mailbox["m"].sum(1)}


def edge_encoder_forward(params: Dict[str, torch.Tensor], pose: torch.Tensor) -> torch.Tensor:
    """``models.py:146-154``: Linear(9,C) -> ReLU -> Linear(C,2C) -> Sigmoid, viewed (E, C, 2).
    ``params`` uses the reference state_dict keys without the ``edge_encoder.`` prefix."""
    h = F.relu(F.linear(pose.float(), params["layers.0.weight"], params["layers.0.bias"]))
    out = torch.sigmoid(F.linear(h, params["layers.2.weight"], params["layers.2.bias"]))
    return out.view(out.shape[0], out.shape[1] // 2, 2)  # (E, C, 2); explicit C so E = 0 works


def film_aggregate(x: torch.Tensor, gb: torch.Tensor, src, dst, mode: str = "film_mean") -> torch.Tensor:
    """The aggregate ``update_all`` writes to ``ndata['images']`` for node features x (N,C,H,W)
    and interleaved gamma/beta gb (E, C, 2)."""
    n = x.shape[0]
    edata = {}
    if mode != "copy_mean":
        C = x.shape[1]
        gb = gb.reshape(-1, C, 2)
        edata = {"pose_gamma": gb[:, :, 0].unsqueeze(-1).unsqueeze(-1),
                 "pose_beta": gb[:, :, 1].unsqueeze(-1).unsqueeze(-1)}
    msg = copy_u if mode == "copy_mean" else edge_udf
    red = node_udf_sum if mode == "film_sum" else node_udf
    out = update_all(src, dst, n, {"image": x}, edata, msg, red)
    if "images" not in out:  # no edges at all
        return torch.zeros_like(x)
    return out["images"]


def film_aggregate_grads(x: torch.Tensor, gb: torch.Tensor, src, dst, grad_out: torch.Tensor,
                         mode: str = "film_mean"):
    """Reference backward by torch autograd through the UDF path: (dx, dgb (E, C, 2))."""
    x = x.detach().clone().requires_grad_(True)
    gb = gb.detach().clone().reshape(-1, x.shape[1], 2).requires_grad_(True)
    out = film_aggregate(x, gb, src, dst, mode)
    dx, dgb = torch.autograd.grad(out, (x, gb), grad_out, allow_unused=True)
    if dx is None:
        dx = torch.zeros_like(x)
    if dgb is None:
        dgb = torch.zeros_like(gb)
    return dx, dgb


def gcn_forward(params, x, pose, src, dst, mode="film_mean", gcn_return="aggregate"):
    """``GCN.forward`` (``models.py:219-226``); ``gcn_return='input'`` is the reference as
    shipped (it returns ``g.ndata['image']``)."""
    if gcn_return == "input":
        return x
    gb = edge_encoder_forward(params, pose) if mode != "copy_mean" else None
    return film_aggregate(x, gb, src, dst, mode)


def dense_film_mean(x: np.ndarray, gb: np.ndarray, src, dst) -> np.ndarray:
    """Closed form in float64 numpy (for property tests): out_v = (1/deg v) sum_e (g_e x_u + b_e)."""
    x = np.asarray(x, np.float64)
    gb = np.asarray(gb, np.float64).reshape(len(src), x.shape[1], 2)
    out = np.zeros_like(x)
    deg = np.zeros(x.shape[0])
    for e, (u, v) in enumerate(zip(src, dst)):
        out[v] += gb[e, :, 0, None, None] * x[u] + gb[e, :, 1, None, None]
        deg[v] += 1
    nz = deg > 0
    out[nz] /= deg[nz, None, None, None]
    return out
