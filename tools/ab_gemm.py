#!/usr/bin/env python3
"""Kernel lab (not product code): the compress GEMMs of the product library (A) against a variant
library (B, tools/build_variant_lib.py) in one process, alternated per round, HIP-graph timed
(bench.time_launches) at the configs[1..4] layer shapes and the headline layer shape: forward, data
gradient, weight gradient, and the three back to back (one graph: the order a training step runs
them, where the chip's power limit sets the clock).
usage: python tools/ab_gemm.py tools/bin/<variant>.so [iters] [rounds] [shapes, e.g. cfg1,cfg3]
       python tools/ab_gemm.py knob:<name>=<a>,<b> ...   (the product library at two knob values)"""
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
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
only = sys.argv[4].split(",") if len(sys.argv) > 4 else None
lib_a = _lib.load_library()
if path_b.startswith("knob:"):
    knob, vals = path_b[5:].split("=")
    va, vb = (int(v) for v in vals.split(","))
    lib_b = lib_a
else:
    knob = None
    lib_b = ctypes.CDLL(os.path.abspath(path_b))
    _lib._declare(lib_b)
dev = torch.device("cuda:0")
cm = mrp.compress
cm.set_compress_path("split")
SHAPES = [("cfg1", 128, 512, 32), ("cfg2", 256, 1280, 8), ("cfg3", 64, 2048, 8), ("cfg4", 128, 1024, 16)]
for name, n, C, H in SHAPES:
    if only and name not in only:
        continue
    torch.manual_seed(0)
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    b = torch.randn(C, device=dev)
    x, a, gy = (torch.randn(n, C, H, H, device=dev) for _ in range(3))
    flop = 2.0 * C * 2 * C * n * H * H
    ops = {
        "fwd": lambda: cm.compress_forward(w, b, x, a),
        "dgrad": lambda: cm.compress_backward_data(w, gy),
        "wgrad": lambda: cm.compress_backward_weight(gy, x, a),
    }
    ops["step"] = lambda: (ops["fwd"](), ops["dgrad"](), ops["wgrad"]())
    res = {}
    outs = {}
    for _ in range(rounds):
        for lab, lib in (("A", lib_a), ("B", lib_b)):
            _lib._lib = lib
            if knob:
                assert lib.mrp_tuning_set(knob.encode(), va if lab == "A" else vb) == 0
            for k, f in ops.items():
                res.setdefault((lab, k), []).append(bench.time_launches([f], iters, dev))
                if k != "step" and (lab, k) not in outs:
                    o = f()
                    outs[(lab, k)] = [t.clone() for t in (o if isinstance(o, tuple) else (o,)) if t is not None]
    _lib._lib = lib_a
    if knob:
        lib_a.mrp_tuning_set(b"reset", 0)
    line = [f"{name} n={n} C={C} {H}x{H}"]
    for k in ops:
        ta, tb = min(res[("A", k)]), min(res[("B", k)])
        fl = flop * (3 if k == "step" else 1)
        same = ""
        if k != "step":
            same = " same" if all(torch.equal(p, q) for p, q in zip(outs[("A", k)], outs[("B", k)])) else " DIFF"
        line.append(f"{k} A {ta * 1e6:7.1f} B {tb * 1e6:7.1f} us ({(tb / ta - 1) * 100:+5.1f} %, "
                    f"{fl / tb / 1e12:5.1f} TF/s{same})")
    print(" | ".join(line), flush=True)
