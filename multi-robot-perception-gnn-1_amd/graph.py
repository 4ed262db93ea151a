"""DGL-free batched robot graph: the graph object the GCN hot path consumes.

Replaces the parts of ``dgl.DGLGraph`` the reference touches on this path:

* ``dgl.graph((src, dst))`` per frame            ``dgl/dataloader.py:88-99``
* ``g.ndata`` / ``g.edata`` feature dicts         ``dgl/dataloader.py:112-122``, ``dgl/model/models.py:175,180,222``
* ``g.local_scope()``                             ``dgl/model/models.py:174,220``
* ``g.to('cuda:0')``                              ``dgl/training.py:183``, ``dgl/eval.py:187``
* ``dgl.batch(list)`` collate                     ``dgl/training.py:57-58``

On top of that it exposes the kernel's view of the graph, :meth:`RobotGraph.csr`: int32 CSR by
destination (in-edges of each node in increasing edge id = DGL mailbox order), per-graph node
offsets and the host-known maximum graph size, cached per device.

The structure (``src``/``dst``) lives on the host; only the CSR arrays and the features move to
the device.  Batched graphs are disjoint unions, so every edge must stay inside its own graph;
this is checked when the CSR is built (the kernel relies on it).
"""
from __future__ import annotations

import contextlib
import warnings
from typing import Dict, Iterable, List, NamedTuple, Optional, Sequence

import numpy as np
import torch

from ._lib import GRAPH_COMPLETE, GRAPH_CSR, MAX_NODES, MAX_REGULAR_K, graph_regular
from .pose import relative_pose_batch


class GraphCSR(NamedTuple):
    """Device-side graph arguments of ``mrp_film_mean_fwd`` / ``mrp_film_mean_bwd``."""

    indptr: torch.Tensor  # (num_nodes + 1,) int32
    src: torch.Tensor  # (num_edges,) int32, global source id, CSR order
    eid: torch.Tensor  # (num_edges,) int32, edge id (row of the (E, C, 2) gamma/beta tensor)
    graph_off: torch.Tensor  # (num_graphs + 1,) int32
    num_graphs: int
    max_nodes: int
    num_nodes: int
    num_edges: int
    graph_kind: int  # GRAPH_COMPLETE (reference topology, arithmetic edge ids), graph_regular(k) or GRAPH_CSR


class _FeatureDict(dict):
    """``ndata``/``edata``: a dict whose values must have ``num`` rows (DGL raises the same)."""

    def __init__(self, num: int, kind: str):
        super().__init__()
        self._num = num
        self._kind = kind

    def __setitem__(self, key, value):
        if not torch.is_tensor(value):
            raise TypeError(f"{self._kind}[{key!r}] must be a tensor")
        if value.dim() == 0 or value.shape[0] != self._num:
            raise ValueError(
                f"{self._kind}[{key!r}] has leading dimension {tuple(value.shape)[:1]}, expected {self._num}"
            )
        super().__setitem__(key, value)


class RobotGraph:
    """A (batched) directed graph of robots/cameras with node and edge feature dicts."""

    def __init__(
        self,
        src,
        dst,
        num_nodes: Optional[int] = None,
        batch_num_nodes: Optional[Sequence[int]] = None,
        batch_num_edges: Optional[Sequence[int]] = None,
    ):
        src_t = torch.as_tensor(np.asarray(src), dtype=torch.int64).reshape(-1).cpu()
        dst_t = torch.as_tensor(np.asarray(dst), dtype=torch.int64).reshape(-1).cpu()
        if src_t.shape != dst_t.shape:
            raise ValueError("src and dst must have the same length")
        if src_t.numel() and int(min(src_t.min(), dst_t.min())) < 0:
            raise ValueError("node ids must be non-negative")
        inferred = int(max(src_t.max(), dst_t.max())) + 1 if src_t.numel() else 0
        n = inferred if num_nodes is None else int(num_nodes)
        if n < inferred:
            raise ValueError(f"num_nodes={n} but edges reference node {inferred - 1}")
        self._edge_store = (src_t, dst_t)
        self._edge_fn = None
        self._ne = int(src_t.numel())
        self._num_nodes = n
        self._bnn = [n] if batch_num_nodes is None else [int(v) for v in batch_num_nodes]
        self._bne = [src_t.numel()] if batch_num_edges is None else [int(v) for v in batch_num_edges]
        if sum(self._bnn) != n or sum(self._bne) != src_t.numel() or len(self._bnn) != len(self._bne):
            raise ValueError("batch_num_nodes / batch_num_edges do not add up")
        self.ndata: Dict[str, torch.Tensor] = _FeatureDict(n, "ndata")
        self.edata: Dict[str, torch.Tensor] = _FeatureDict(src_t.numel(), "edata")
        self._csr_cache: Dict[str, GraphCSR] = {}
        self._host_csr = None

    @classmethod
    def _from_device(cls, edge_fn, num_nodes: int, num_edges: int, bnn: Sequence[int], bne: Sequence[int],
                     csr: Optional[GraphCSR] = None, device=None, complete: Optional[bool] = None,
                     kdeg: Optional[int] = None) -> "RobotGraph":
        """A graph whose structure was built on the device (``frame_batch``): the host edge list is
        produced by ``edge_fn()`` only if something asks for it (``edges()``, ``host_csr()``)."""
        g = cls.__new__(cls)
        g._edge_store = None
        g._edge_fn = edge_fn
        g._ne = int(num_edges)
        g._num_nodes = int(num_nodes)
        g._bnn, g._bne = [int(v) for v in bnn], [int(v) for v in bne]
        g.ndata = _FeatureDict(g._num_nodes, "ndata")
        g.edata = _FeatureDict(g._ne, "edata")
        g._csr_cache = {}
        if csr is not None:
            g._csr_cache[(str(torch.device(device)), csr.graph_kind)] = csr
        g._host_csr = None
        g._complete = complete
        g._kdeg = kdeg
        return g

    @property
    def _src(self) -> torch.Tensor:
        return self._edges_host()[0]

    @property
    def _dst(self) -> torch.Tensor:
        return self._edges_host()[1]

    def _edges_host(self):
        if self._edge_store is None:
            src, dst = self._edge_fn()
            self._edge_store = (torch.as_tensor(src, dtype=torch.int64).cpu(),
                                torch.as_tensor(dst, dtype=torch.int64).cpu())
        return self._edge_store

    # ----------------------------------------------------------------- DGL-like API
    def num_nodes(self) -> int:
        return self._num_nodes

    def num_edges(self) -> int:
        return self._ne

    @property
    def batch_size(self) -> int:
        return len(self._bnn)

    def batch_num_nodes(self) -> torch.Tensor:
        return torch.tensor(self._bnn, dtype=torch.int64)

    def batch_num_edges(self) -> torch.Tensor:
        return torch.tensor(self._bne, dtype=torch.int64)

    def edges(self):
        """(src, dst) int64 host tensors in edge-id order."""
        return self._src, self._dst

    def in_degrees(self) -> torch.Tensor:
        return torch.bincount(self._dst, minlength=self._num_nodes)

    @property
    def device(self) -> torch.device:
        for t in list(self.ndata.values()) + list(self.edata.values()):
            return t.device
        return torch.device("cpu")

    @contextlib.contextmanager
    def local_scope(self):
        """Feature writes inside the scope are discarded on exit (in-place tensor edits are not),
        the semantics ``models.py:174,220`` rely on."""
        saved_n = dict(self.ndata)
        saved_e = dict(self.edata)
        try:
            yield self
        finally:
            dict.clear(self.ndata)
            dict.update(self.ndata, saved_n)
            dict.clear(self.edata)
            dict.update(self.edata, saved_e)

    def to(self, device, non_blocking: bool = False) -> "RobotGraph":
        """A graph sharing this structure with every feature moved to ``device``."""
        g = RobotGraph.__new__(RobotGraph)
        # share the structure (and its lazily built host edge list) without materialising it
        g._edge_store, g._edge_fn, g._ne, g._num_nodes = self._edge_store, self._edge_fn, self._ne, self._num_nodes
        g._bnn, g._bne = list(self._bnn), list(self._bne)
        g.ndata = _FeatureDict(self._num_nodes, "ndata")
        g.edata = _FeatureDict(self.num_edges(), "edata")
        for k, v in self.ndata.items():
            g.ndata[k] = v.to(device, non_blocking=non_blocking)
        for k, v in self.edata.items():
            g.edata[k] = v.to(device, non_blocking=non_blocking)
        g._csr_cache = self._csr_cache  # structure is shared, so is its device CSR
        g._host_csr = self._host_csr
        g._complete = getattr(self, "_complete", None)
        g._kdeg = getattr(self, "_kdeg", None)
        return g

    def cuda(self, device=None) -> "RobotGraph":
        return self.to(torch.device("cuda") if device is None else device)

    # ----------------------------------------------------------------- kernel view
    def host_csr(self):
        """int32 numpy CSR by destination, validated: (indptr, src, eid, graph_off, max_nodes)."""
        if self._host_csr is None:
            self._host_csr = build_csr(self._src.numpy(), self._dst.numpy(), self._num_nodes, self._bnn)
        return self._host_csr

    def is_complete(self) -> bool:
        """True when every graph of the batch is the reference's complete graph over the same
        number of robots with edges in ``complete_edges`` order (``dgl/dataloader.py:88-95``);
        the kernels then compute edge ids arithmetically instead of walking the CSR."""
        if getattr(self, "_complete", None) is None:
            self._complete = is_complete_batch(self._src.numpy(), self._dst.numpy(), self._bnn)
        return self._complete

    def in_degree_k(self) -> int:
        """k when every node has exactly k in-edges (k-NN frames), else 0."""
        if getattr(self, "_kdeg", None) is None:
            deg = np.diff(self.host_csr()[0])
            self._kdeg = int(deg[0]) if deg.size and deg[0] > 0 and np.all(deg == deg[0]) else 0
        return self._kdeg

    def csr(self, device, allow_complete: bool = True, allow_regular: bool = True) -> GraphCSR:
        """Device CSR for the kernels.  ``graph_kind`` is GRAPH_COMPLETE for the reference topology,
        ``graph_regular(k)`` when every node has k in-edges (k <= 8; the backward then keeps one
        Gram accumulator per edge), else GRAPH_CSR."""
        device = torch.device(device)
        if allow_complete and self.is_complete():
            kind = GRAPH_COMPLETE
        elif allow_regular and 1 <= self.in_degree_k() <= MAX_REGULAR_K:
            kind = graph_regular(self.in_degree_k())
        else:
            kind = GRAPH_CSR
        key = (str(device), kind)
        hit = self._csr_cache.get(key)
        if hit is not None:
            return hit
        indptr, src, eid, goff, max_nodes = self.host_csr()
        to = lambda a: torch.from_numpy(a).to(device)  # noqa: E731
        csr = GraphCSR(to(indptr), to(src), to(eid), to(goff), len(self._bnn), max_nodes,
                       self._num_nodes, self.num_edges(), kind)
        self._csr_cache[key] = csr
        return csr

    def __repr__(self) -> str:
        return (f"RobotGraph(num_nodes={self._num_nodes}, num_edges={self.num_edges()}, "
                f"batch_size={self.batch_size}, ndata={list(self.ndata)}, edata={list(self.edata)})")


def build_csr(src: np.ndarray, dst: np.ndarray, num_nodes: int, batch_num_nodes: Sequence[int]):
    """CSR by destination with in-edges in increasing edge id (DGL's mailbox order).

    Raises ``ValueError`` if an edge crosses graphs, a graph exceeds ``MAX_NODES`` nodes, or an id
    does not fit int32.
    """
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    E = src.shape[0]
    if num_nodes >= 2 ** 31 or E >= 2 ** 31:
        raise ValueError("graph too large for int32 CSR")
    goff = np.zeros(len(batch_num_nodes) + 1, dtype=np.int64)
    np.cumsum(np.asarray(batch_num_nodes, dtype=np.int64), out=goff[1:])
    max_nodes = int(max(batch_num_nodes)) if len(batch_num_nodes) else 0
    if max_nodes > MAX_NODES:
        raise ValueError(f"a graph has {max_nodes} nodes; the kernels support up to {MAX_NODES} per graph")
    if E:
        gs = np.searchsorted(goff, src, side="right") - 1
        gd = np.searchsorted(goff, dst, side="right") - 1
        if not np.array_equal(gs, gd):
            bad = int(np.nonzero(gs != gd)[0][0])
            raise ValueError(f"edge {bad} ({src[bad]}->{dst[bad]}) crosses graphs of the batch")
    order = np.argsort(dst, kind="stable")
    indptr = np.zeros(num_nodes + 1, dtype=np.int64)
    np.cumsum(np.bincount(dst, minlength=num_nodes), out=indptr[1:])
    return (indptr.astype(np.int32), src[order].astype(np.int32), order.astype(np.int32),
            goff.astype(np.int32), max_nodes)


def is_complete_batch(src: np.ndarray, dst: np.ndarray, batch_num_nodes: Sequence[int]) -> bool:
    """Every graph has the same n nodes and exactly the edges of ``complete_edges(n)``, in that
    order, offset graph by graph (what ``dgl.batch`` of the reference's frames produces)."""
    if not len(batch_num_nodes):
        return False
    n = int(batch_num_nodes[0])
    B = len(batch_num_nodes)
    if n < 1 or any(int(v) != n for v in batch_num_nodes) or n > MAX_NODES:
        return False
    if len(src) != B * n * (n - 1):
        return False
    if n == 1:
        return True
    cs, cd = (np.asarray(t, dtype=np.int64) for t in complete_edges(n))
    off = (np.arange(B, dtype=np.int64) * n)[:, None]
    return bool(np.array_equal(np.asarray(src).reshape(B, -1), cs[None] + off)
                and np.array_equal(np.asarray(dst).reshape(B, -1), cd[None] + off))


# --------------------------------------------------------------------- constructors
def graph(edge_list, num_nodes: Optional[int] = None) -> RobotGraph:
    """``dgl.graph((src_list, dst_list))`` equivalent (``dgl/dataloader.py:99``)."""
    src, dst = edge_list
    return RobotGraph(src, dst, num_nodes=num_nodes)


def complete_edges(n: int):
    """The reference's per-frame edge list: every ordered pair i != j, i-major
    (``dgl/dataloader.py:88-95``)."""
    src = [i for i in range(n) for j in range(n) if i != j]
    dst = [j for i in range(n) for j in range(n) if i != j]
    return src, dst


def complete_graph(n: int) -> RobotGraph:
    return RobotGraph(*complete_edges(n), num_nodes=n)


def knn_edges(positions, k: int):
    """k-nearest-neighbour in-edges: for each destination v (ascending), the k sources u != v
    with the smallest ``|t_u - t_v|`` (ties -> lower index), listed in ascending u.
    (The BASELINE's k-NN(4) configuration; the reference only builds complete graphs.)"""
    pos = np.asarray(positions, dtype=np.float64)
    n = pos.shape[0]
    if not 0 <= k < max(n, 1):
        raise ValueError(f"k={k} needs 0 <= k < n={n}")
    d = np.linalg.norm(pos[:, None, :] - pos[None, :, :], axis=-1)
    src, dst = [], []
    for v in range(n):
        cand = [u for u in range(n) if u != v]
        cand.sort(key=lambda u: (d[u, v], u))
        for u in sorted(cand[:k]):
            src.append(u)
            dst.append(v)
    return src, dst


def frame_graph(poses, knn: Optional[int] = None) -> RobotGraph:
    """One frame: nodes = robots, ``edata['pose']`` = relative pose of every edge
    (``dgl/dataloader.py:97-122``).  ``poses``: (n, 7) ``(t, q_xyzw)``; complete graph unless
    ``knn`` is given."""
    poses = np.asarray(poses)
    n = poses.shape[0]
    src, dst = complete_edges(n) if knn is None else knn_edges(poses[:, :3], knn)
    g = RobotGraph(src, dst, num_nodes=n)
    if len(src):
        rel = relative_pose_batch(poses[np.asarray(src)], poses[np.asarray(dst)])
    else:
        rel = np.zeros((0, 9))
    g.edata["pose"] = torch.from_numpy(np.ascontiguousarray(rel)).float()
    return g


def batch(graphs: Iterable[RobotGraph]) -> RobotGraph:
    """``dgl.batch`` equivalent: disjoint union, node ids offset per graph, features
    concatenated for keys present in every graph (``dgl/training.py:57-58``)."""
    graphs: List[RobotGraph] = list(graphs)
    if not graphs:
        raise ValueError("batch() needs at least one graph")
    srcs, dsts, bnn, bne = [], [], [], []
    off = 0
    for g in graphs:
        s, d = g.edges()
        srcs.append(s + off)
        dsts.append(d + off)
        bnn.extend(g._bnn)
        bne.extend(g._bne)
        off += g.num_nodes()
    out = RobotGraph(torch.cat(srcs), torch.cat(dsts), num_nodes=off, batch_num_nodes=bnn, batch_num_edges=bne)
    for key in graphs[0].ndata:
        if all(key in g.ndata for g in graphs):
            out.ndata[key] = torch.cat([g.ndata[key] for g in graphs], 0)
    for key in graphs[0].edata:
        if all(key in g.edata for g in graphs):
            out.edata[key] = torch.cat([g.edata[key] for g in graphs], 0)
    return out


def unbatch_offsets(g: RobotGraph):
    """Node offsets of the graphs in a batch (int64 numpy, length batch_size + 1)."""
    return np.concatenate([[0], np.cumsum(g._bnn)]).astype(np.int64)


def unbatch(g: RobotGraph) -> List[RobotGraph]:
    """``dgl.unbatch`` equivalent: split a batched graph into its per-frame graphs (node and edge
    ids renumbered from 0 per graph, features sliced)."""
    src, dst = (t.numpy() for t in g.edges())
    noff = np.concatenate([[0], np.cumsum(g._bnn)]).astype(np.int64)
    eoff = np.concatenate([[0], np.cumsum(g._bne)]).astype(np.int64)
    out = []
    for i in range(len(g._bnn)):
        e0, e1, n0, n1 = eoff[i], eoff[i + 1], noff[i], noff[i + 1]
        s, d = src[e0:e1] - n0, dst[e0:e1] - n0
        if s.size and (s.min() < 0 or d.min() < 0 or s.max() >= n1 - n0 or d.max() >= n1 - n0):
            raise ValueError(f"graph {i}: its edges leave its node range (not a dgl.batch result)")
        gi = RobotGraph(s, d, num_nodes=int(n1 - n0))
        for k, v in g.ndata.items():
            gi.ndata[k] = v[n0:n1]
        for k, v in g.edata.items():
            gi.edata[k] = v[e0:e1]
        out.append(gi)
    return out


# ------------------------------------------------------------------ graph cache on disk
_CACHE_MAGIC = "mrp_gnn_graph_cache_v1"


def save_graphs(filename: str, g_list, labels: Optional[Dict[str, torch.Tensor]] = None) -> None:
    """``dgl.save_graphs`` equivalent for the dataset cache (``dgl/dataloader.py:165-169``).

    Format: a NumPy ``.npz`` archive (no pickles) written to ``filename`` as given — the batched
    structure (src, dst, per-graph node/edge counts) plus every node/edge feature and label.  This is
    this package's own cache format; :func:`load_graphs` reads it and, without DGL, a cache DGL wrote
    (:mod:`.dgl_format`, parity unpinned).  Writing DGL's format is not offered: with no DGL to check
    against, a file written here could not be promised to load in DGL."""
    g_list = [g_list] if isinstance(g_list, RobotGraph) else list(g_list)
    arrays = {"magic": np.array(_CACHE_MAGIC), "num_graphs": np.array(len(g_list), np.int64)}
    if g_list:
        b = batch(g_list)
        src, dst = (t.numpy() for t in b.edges())
        arrays.update(src=src, dst=dst, bnn=np.asarray(b._bnn, np.int64), bne=np.asarray(b._bne, np.int64))
        for k, v in b.ndata.items():
            arrays["ndata/" + k] = v.detach().cpu().numpy()
        for k, v in b.edata.items():
            arrays["edata/" + k] = v.detach().cpu().numpy()
    for k, v in (labels or {}).items():
        arrays["label/" + k] = torch.as_tensor(v).detach().cpu().numpy()
    with open(filename, "wb") as f:
        np.savez(f, **arrays)


_WARNED_DGL = False


def load_graphs(filename: str, idx_list: Optional[Sequence[int]] = None):
    """``dgl.load_graphs`` equivalent: ``(list of graphs, labels dict)`` from :func:`save_graphs`'s
    format (``dgl/dataloader.py:172-175``); ``idx_list`` selects graphs by index.  A file DGL wrote
    (``dgl_graph_<N>.bin``, version 2) is read by :mod:`.dgl_format` — parity unpinned (no DGL and
    no DGL-written file to check it against), said once per process."""
    from . import dgl_format
    if dgl_format.is_dgl_graph_file(filename):
        global _WARNED_DGL
        if not _WARNED_DGL:
            _WARNED_DGL = True
            warnings.warn("mrp_gnn: reading a DGL-written graph file with a reader restated from DGL's "
                          "serializer and not checked against DGL (parity unpinned)", stacklevel=2)
        return dgl_format.read_dgl_graphs(filename, idx_list)
    try:
        z = np.load(filename, allow_pickle=False)
    except ValueError as e:
        raise ValueError(f"{filename}: not an mrp_gnn graph cache (DGL's binary format is not read; "
                         "delete the file so the dataset rebuilds it)") from e
    with z:
        if "magic" not in z.files or str(z["magic"]) != _CACHE_MAGIC:
            raise ValueError(f"{filename}: not an mrp_gnn graph cache")
        labels = {k[len("label/"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("label/")}
        if int(z["num_graphs"]) == 0:
            return [], labels
        bnn, bne = z["bnn"].tolist(), z["bne"].tolist()
        b = RobotGraph(z["src"], z["dst"], num_nodes=int(sum(bnn)), batch_num_nodes=bnn, batch_num_edges=bne)
        for k in z.files:
            if k.startswith("ndata/"):
                b.ndata[k[len("ndata/"):]] = torch.from_numpy(z[k])
            elif k.startswith("edata/"):
                b.edata[k[len("edata/"):]] = torch.from_numpy(z[k])
    graphs = unbatch(b)
    if idx_list is not None:
        graphs = [graphs[i] for i in idx_list]
    return graphs, labels
