#!/usr/bin/env python3
"""Kernel lab (not product code): the aggregation kernels of the product library (A) against a variant
library (B, tools/build_variant_lib.py) in one process, alternated, HIP-graph timed like bench.py's
rooflines (rotating buffer sets over 512 MB), at the headline and configs[1..4] shapes: forward,
backward without a base and the training (DXB) backward; the backward's outputs compared bit for bit.
usage: python tools/ab_libs.py tools/bin/<variant>.so [iters] [rounds]
       python tools/ab_libs.py knob:<name>=<a>,<b> [iters] [rounds]   (the product library at two knob values)"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402
from mrp_gnn_amd import _lib  # noqa: E402

path_b = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
lib_a = _lib.load_library()
knob = None
if path_b.startswith("knob:"):
    knob, vals = path_b[5:].split("=")
    kv = dict(zip(("A", "B"), (int(v) for v in vals.split(","))))
    lib_b = lib_a
else:
    lib_b = ctypes.CDLL(os.path.abspath(path_b))
    _lib._declare(lib_b)


def use(lab, lib):
    _lib._lib = lib
    if knob:
        assert lib.mrp_tuning_set(knob.encode(), kv[lab]) == 0
dev = torch.device("cuda:0")
SHAPES = [("north_star", 32, 8, 512, 32, None), ("cfg1", 16, 8, 512, 32, None), ("cfg2", 32, 8, 1280, 8, None),
          ("cfg3", 8, 8, 2048, 8, None), ("cfg4", 8, 16, 1024, 16, 4)]
mode = _lib.MODE_FILM_MEAN | _lib.GB_LOGITS
for name, B, N, C, H, knn in SHAPES:
    g = bench.make_workload(B, N, C, H, H, seed=3, device=dev, knn=knn)
    x = g.ndata["image"]
    csr = g.csr(dev)
    torch.manual_seed(0)
    z = torch.randn(g.num_edges(), 2 * C, device=dev)
    plane = x.numel() * 4
    nb = bench.rotating_sets(4 * plane)
    sets = [(torch.randn_like(x), x if i == 0 else torch.randn_like(x), torch.randn_like(x)) for i in range(nb)]
    res = {}

    def run(lib, kind):
        if kind == "fwd":
            fs = [lambda xi=xi, oi=G: mrp.film_mean_forward_into(xi, z, csr, mode, oi) for G, xi, _ in sets]
        elif kind == "bwd":
            fs = [lambda G=G, xi=xi: mrp.aggregate.film_mean_backward(G, xi, z, csr, mode, True, True) for G, xi, _ in sets]
        else:
            fs = [lambda G=G, xi=xi, bs=bs: mrp.aggregate.film_mean_backward(G, xi, z, csr, mode, True, True,
                                                                             grad_x_base=bs) for G, xi, bs in sets]
        return bench.time_launches(fs, iters, dev)

    for _ in range(rounds):
        for lab, lib in (("A", lib_a), ("B", lib_b)):
            use(lab, lib)
            for kind in ("fwd", "bwd", "dxb"):
                res.setdefault((lab, kind), []).append(run(lib, kind))
    outs = {}
    for lab, lib in (("A", lib_a), ("B", lib_b)):
        use(lab, lib)
        G, xi, bs = sets[0]
        o = mrp.aggregate.film_mean_backward(G, xi, z, csr, mode, True, True, grad_x_base=bs)
        outs[lab] = [t.clone() for t in (o if isinstance(o, (tuple, list)) else (o,)) if t is not None]
    same = all(torch.equal(a, b) for a, b in zip(outs["A"], outs["B"]))
    _lib._lib = lib_a
    if knob:
        lib_a.mrp_tuning_set(b"reset", 0)
    print(f"{name:10s} " + "  ".join(f"{k[1]} {k[0]} {min(v) * 1e6:7.1f} us" for k, v in sorted(res.items(), key=lambda t: (t[0][1], t[0][0])))
          + f"  outputs bit-identical {same}", flush=True)
    del sets
    torch.cuda.empty_cache()
