"""Reader of DGL's binary graph file — the format ``dgl.save_graphs`` writes and the reference's
dataset cache uses (``dgl_graph_<N>.bin``, ``dgl/dataloader.py:165-175``), so a cache processed by
the reference loads here without DGL.

PARITY UNPINNED.  DGL is third-party, absent from this image and version-unpinned by the reference
(SURVEY §0, L2'), and the reference ships no ``.bin`` file: nothing here is checked against a file
DGL wrote.  The layout is restated from DGL's serializer (DGL >= 0.6, file version 2:
``src/graph/serialize/heterograph_serialize.cc`` ``SaveHeteroGraphs``, ``heterograph_data.h``
``HeteroGraphDataObject::Save``, ``src/runtime/ndarray.cc`` ``SaveDLTensor``, dmlc-core's
``Stream::Write`` for vectors and strings), and the reader leans only on the parts of it that are
plain containers:

  file    u64 magic 0xDD2E4FF046B4A13F, u64 version (2), u64 graph type, u64 num_graphs,
          vector<u64> graph offsets, vector<pair<string, NDArray>> labels, then the graph records
  graph   [graph structure: HeteroGraph::Save], node tensors vector<vector<pair<string, NDArray>>>
          (one inner vector per node type), edge tensors (same, per edge type), vector<string> node
          type names, vector<string> edge type names — the record ends at the next graph's offset
  NDArray u64 magic 0xDD5E40F096B4A13F, u64 reserved, i32 device type, i32 device id, i32 ndim,
          u8 type code, u8 bits, u16 lanes, i64 shape[ndim], i64 byte count, the bytes
  vector  u64 count, then the elements;  string: u64 length, then the bytes (little-endian)

The graph-structure part (the metagraph and the relation graph's sparse matrix, whose inner magic
numbers and field order this restatement does not rely on) is read structurally: the record's
named-tensor block is located as the earliest offset from which the whole tail parses and ends
exactly at the record's end; the per-type node counts are the vector<i64> just before it; the edge
list is the relation graph's COO matrix — the last two consecutive integer arrays of one length E
(E = the edge tensors' leading dimension when there are any) with every value below the node count,
and a third such array that is a permutation of 0..E-1 is taken as the edge ids.  DGL saves the COO
form whenever the graph has one (``dgl.graph(edge_list)``, as the reference builds them, does); a
record holding only CSR/CSC is rejected with a clear error, as are heterographs (more than one
node or edge type) and file version 1 (DGL < 0.6).  Every check failure raises ``ValueError``.

Host-side file parsing (numpy over a memory map of the file); no GPU, no torch kernels.
"""
from __future__ import annotations

import mmap
import os
import struct
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

FILE_MAGIC = 0xDD2E4FF046B4A13F
NDARRAY_MAGIC = 0xDD5E40F096B4A13F
_NDARRAY_MAGIC_BYTES = struct.pack("<Q", NDARRAY_MAGIC)

# DLDataType (code, bits) -> numpy dtype; code 0 int, 1 uint, 2 float, 4 bfloat, 6 bool
_DTYPES = {(0, 8): np.int8, (0, 16): np.int16, (0, 32): np.int32, (0, 64): np.int64,
           (1, 8): np.uint8, (1, 16): np.uint16, (1, 32): np.uint32, (1, 64): np.uint64,
           (2, 16): np.float16, (2, 32): np.float32, (2, 64): np.float64, (4, 16): np.int16,
           (6, 8): np.bool_}

_MAX_NAME = 4096
_MAX_TYPES = 1 << 16


class _Reader:
    """Little-endian cursor over the file's bytes; every read bounds-checked."""

    def __init__(self, buf: bytes, pos: int = 0, end: Optional[int] = None):
        self.buf, self.pos = buf, pos
        self.end = len(buf) if end is None else end

    def need(self, n: int):
        if n < 0 or self.pos + n > self.end:
            raise ValueError(f"truncated record at byte {self.pos} (needs {n} more)")

    def u64(self) -> int:
        self.need(8)
        v = struct.unpack_from("<Q", self.buf, self.pos)[0]
        self.pos += 8
        return v

    def i64(self) -> int:
        self.need(8)
        v = struct.unpack_from("<q", self.buf, self.pos)[0]
        self.pos += 8
        return v

    def string(self) -> str:
        n = self.u64()
        if n > _MAX_NAME:
            raise ValueError(f"string of {n} bytes at byte {self.pos - 8}")
        self.need(n)
        raw = self.buf[self.pos:self.pos + n]
        self.pos += n
        s = raw.decode("utf-8")
        if not s.isprintable():
            raise ValueError(f"non-printable name at byte {self.pos - n}")
        return s

    def ndarray(self) -> Tuple[np.ndarray, int]:
        """One NDArray record -> (array, its DL type code)."""
        start = self.pos
        if self.u64() != NDARRAY_MAGIC:
            raise ValueError(f"no NDArray at byte {start}")
        self.u64()  # reserved
        self.need(8 + 4 + 4)
        _dev_type, _dev_id, ndim = struct.unpack_from("<iii", self.buf, self.pos)
        self.pos += 12
        code, bits, lanes = struct.unpack_from("<BBH", self.buf, self.pos)
        self.pos += 4
        if not 0 <= ndim <= 32 or lanes != 1 or (code, bits) not in _DTYPES:
            raise ValueError(f"NDArray at byte {start}: ndim {ndim}, dtype ({code}, {bits}, {lanes})")
        self.need(8 * ndim)
        shape = struct.unpack_from(f"<{ndim}q", self.buf, self.pos)
        self.pos += 8 * ndim
        nbytes = self.i64()
        count = int(np.prod(shape, dtype=np.int64)) if ndim else 1
        if min(shape, default=0) < 0 or nbytes != count * bits // 8:
            raise ValueError(f"NDArray at byte {start}: shape {shape} with {nbytes} bytes")
        self.need(nbytes)
        # a writable copy of the bytes: nothing keeps a view into the file's memory map
        arr = np.frombuffer(bytearray(self.buf[self.pos:self.pos + nbytes]), dtype=_DTYPES[(code, bits)],
                            count=count).reshape(shape)
        self.pos += nbytes
        return arr, code

    def named_tensors(self) -> List[Tuple[str, np.ndarray, int]]:
        n = self.u64()
        if n > _MAX_TYPES:
            raise ValueError(f"{n} named tensors at byte {self.pos - 8}")
        out = []
        for _ in range(n):
            name = self.string()
            arr, code = self.ndarray()
            out.append((name, arr, code))
        return out

    def strings(self) -> List[str]:
        n = self.u64()
        if n > _MAX_TYPES:
            raise ValueError(f"{n} names at byte {self.pos - 8}")
        return [self.string() for _ in range(n)]


def _tensor(arr: np.ndarray, code: int) -> torch.Tensor:
    t = torch.from_numpy(arr)
    return t.view(torch.bfloat16) if code == 4 else t


def _parse_tail(buf: bytes, start: int, end: int):
    """The named-tensor block of a graph record, if it parses from ``start`` to exactly ``end``."""
    r = _Reader(buf, start, end)
    nt = r.u64()
    if not 1 <= nt <= _MAX_TYPES:
        raise ValueError("node type count")
    ntensors = [r.named_tensors() for _ in range(nt)]
    et = r.u64()
    if not 1 <= et <= _MAX_TYPES:
        raise ValueError("edge type count")
    etensors = [r.named_tensors() for _ in range(et)]
    ntypes, etypes = r.strings(), r.strings()
    if r.pos != end or len(ntypes) != nt or len(etypes) != et:
        raise ValueError("tail does not end the record")
    return ntensors, etensors, ntypes, etypes


def _locate_tail(buf: bytes, start: int, end: int):
    """Offset of the named-tensor block: tried at every candidate implied by an NDArray record whose
    name string precedes it, and (a record without named tensors) at every offset of the last 4 KiB."""
    cands = []
    p = buf.find(_NDARRAY_MAGIC_BYTES, start, end)
    while p >= 0:
        for L in range(1, min(_MAX_NAME, p - start) + 1):
            q = p - L - 8
            if q < start:
                break
            if struct.unpack_from("<Q", buf, q)[0] == L:
                # [types][count] before the first tensor of the first non-empty group; empty groups
                # before it add (count 0) or (count 0, types) words
                for extra in range(0, 6):
                    s = q - 16 - 8 * extra
                    if s >= start:
                        cands.append(s)
        p = buf.find(_NDARRAY_MAGIC_BYTES, p + 8, end)
    cands.extend(range(max(start, end - 4096), end))
    # the earliest offset that parses is the block: a later one is a suffix of it that the last node
    # tensor's trailing bytes happen to complete (e.g. int64 values 1, 0 read as one node type with
    # no tensors — seen with random int64 node data)
    found = None
    for s in sorted(set(cands)):
        try:
            found = (s, _parse_tail(buf, s, end))
            break
        except (ValueError, UnicodeDecodeError, struct.error):
            continue
    if found is None:
        raise ValueError(f"graph record at byte {start}: no node/edge tensor block ends the record")
    return found


def _structure_arrays(buf: bytes, start: int, end: int) -> List[np.ndarray]:
    """Integer NDArray records of the graph-structure part, in file order."""
    out = []
    p = buf.find(_NDARRAY_MAGIC_BYTES, start, end)
    while p >= 0:
        try:
            r = _Reader(buf, p, end)
            arr, code = r.ndarray()
        except (ValueError, struct.error):
            p = buf.find(_NDARRAY_MAGIC_BYTES, p + 1, end)
            continue
        if code in (0, 1) and arr.ndim == 1:
            out.append(arr.astype(np.int64))
        p = buf.find(_NDARRAY_MAGIC_BYTES, r.pos, end)
    return out


def _is_indptr(p: np.ndarray, n: int, m: int) -> bool:
    return p.shape[0] == n + 1 and p[0] == 0 and p[-1] == m and bool(np.all(np.diff(p) >= 0))


def _edge_list(arrays: List[np.ndarray], n: int, e: Optional[int]):
    """(src, dst) of the relation graph's COO matrix: the last two consecutive arrays of equal length
    (= e when known) with every value in [0, n); a following permutation of 0..E-1 orders the edges."""
    for i in range(len(arrays) - 2, -1, -1):
        a, b = arrays[i], arrays[i + 1]
        m = a.shape[0]
        if b.shape[0] != m or (e is not None and m != e):
            continue
        if m and (a.min() < 0 or b.min() < 0 or a.max() >= n or b.max() >= n):
            continue
        if i >= 1 and _is_indptr(arrays[i - 1], n, m):
            break  # (indptr, indices, ids): a CSR/CSC matrix, not a COO one
        if i + 2 < len(arrays) and arrays[i + 2].shape[0] == m and m > 0:
            eid = arrays[i + 2]
            if np.array_equal(np.sort(eid), np.arange(m)):
                order = np.empty(m, np.int64)
                order[eid] = np.arange(m)
                return a[order], b[order]
        return a, b
    raise ValueError("no COO edge list in the graph record (a CSR/CSC-only record is not read: its "
                     "orientation is not recoverable without DGL's format code)")


def read_dgl_graphs(filename: str, idx_list: Optional[Sequence[int]] = None):
    """``dgl.load_graphs(filename, idx_list)`` for a version-2 DGL file: ``(graphs, labels)`` —
    :class:`~mrp_gnn_amd.graph.RobotGraph` objects with their ``ndata``/``edata`` tensors, and the
    label dict.  Parity unpinned (module docstring)."""
    with open(filename, "rb") as f:
        if os.fstat(f.fileno()).st_size == 0:
            raise ValueError(f"{filename}: empty file")
        # memory-mapped: a dataset cache of image frames can be many GB; only the selected graphs'
        # bytes are touched (tensors are copied out of the map)
        with mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as buf:
            return _read(buf, filename, idx_list)


def _read(buf, filename: str, idx_list: Optional[Sequence[int]]):
    from .graph import RobotGraph
    r = _Reader(buf)
    if r.u64() != FILE_MAGIC:
        raise ValueError(f"{filename}: not a DGL graph file (magic)")
    version = r.u64()
    if version != 2:
        raise ValueError(f"{filename}: DGL graph file version {version} is not read (version 2, DGL >= 0.6)")
    r.u64()  # graph type
    num = r.u64()
    offsets = [r.u64() for _ in range(r.u64())]
    if len(offsets) != num:
        raise ValueError(f"{filename}: {len(offsets)} graph offsets for {num} graphs")
    labels = {name: _tensor(arr, code) for name, arr, code in r.named_tensors()}
    bounds = offsets + [len(buf)]
    if num and (offsets[0] != r.pos or any(b <= a for a, b in zip(bounds, bounds[1:]))):
        raise ValueError(f"{filename}: graph offsets {offsets[:4]}... do not follow the header at byte {r.pos}")
    picks = range(num) if idx_list is None else [int(i) for i in idx_list]
    graphs = []
    for i in picks:
        if not 0 <= i < num:
            raise IndexError(f"graph index {i} out of range ({num} graphs)")
        start, end = bounds[i], bounds[i + 1]
        tail, (nts, ets, ntypes, etypes) = _locate_tail(buf, start, end)
        if len(ntypes) != 1 or len(etypes) != 1:
            raise ValueError(f"{filename}: graph {i} is a heterograph ({ntypes}, {etypes}): not read")
        # num_verts_per_type: vector<i64> of one entry right before the tensor block
        if tail - 16 < start or struct.unpack_from("<Q", buf, tail - 16)[0] != 1:
            raise ValueError(f"{filename}: graph {i}: no node count before the tensor block")
        n = struct.unpack_from("<q", buf, tail - 8)[0]
        nd = {name: _tensor(arr, code) for name, arr, code in nts[0]}
        ed = {name: _tensor(arr, code) for name, arr, code in ets[0]}
        for name, t in nd.items():
            if t.dim() == 0 or t.shape[0] != n:
                raise ValueError(f"{filename}: graph {i}: ndata[{name!r}] has {tuple(t.shape)[:1]} rows, {n} nodes")
        e_known = next(iter(ed.values())).shape[0] if ed else None
        src, dst = _edge_list(_structure_arrays(buf, start, tail - 16), n, e_known)
        g = RobotGraph(src, dst, num_nodes=n)
        for k, v in nd.items():
            g.ndata[k] = v
        for k, v in ed.items():
            g.edata[k] = v
        graphs.append(g)
    return graphs, labels


def is_dgl_graph_file(filename: str) -> bool:
    with open(filename, "rb") as f:
        head = f.read(8)
    return len(head) == 8 and struct.unpack("<Q", head)[0] == FILE_MAGIC
