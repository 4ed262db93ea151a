"""Kernel lab (not product code): the compress forward / data-gradient GEMM forms side by side per
BASELINE config shape — gemm_split 4 (32-k stages, 32x32x16 MFMAs), 5 (the pipelined default) and 7
(32-k stages on 16x16x32 MFMAs) — HIP-graph timed (bench.time_launches), with the max relative error
against float64 and a repeat-launch bit-identity check.

usage: python tools/exp_nn_forms.py [--iters N] [--forms 4,5,7]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import time_launches  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--forms", default="4,5,7")
args = ap.parse_args()
forms = [int(v) for v in args.forms.split(",")]
dev = torch.device("cuda:0")
cm = mrp.compress
lib = mrp.load_library()
cm.set_compress_path("split")
SHAPES = [("cfg1", 128, 512, 32), ("cfg2", 256, 1280, 8), ("cfg3", 64, 2048, 8), ("cfg4", 128, 1024, 16),
          ("head", 256, 512, 32)]
for name, n, C, H in SHAPES:
    torch.manual_seed(0)
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    b = torch.randn(C, device=dev)
    x, a, gy = (torch.randn(n, C, H, H, device=dev) for _ in range(3))
    flop = 2.0 * C * 2 * C * n * H * H
    yref = cm._lib_forward(w.double(), b.double(), x.double(), a.double())
    gref = cm._lib_backward_data(w.double(), gy.double())
    row = [f"{name} n={n} C={C} {H}x{H}"]
    for v in forms:
        assert lib.mrp_tuning_set(b"gemm_split", v) == 0
        f = lambda: cm.compress_forward(w, b, x, a)
        d = lambda: cm.compress_backward_data(w, gy)
        y, g = f(), d()
        same = torch.equal(y, f()) and all(torch.equal(p, q) for p, q in zip(g, d()))
        ey = float((y.double() - yref).abs().max() / yref.abs().max())
        eg = max(float((p.double() - r).abs().max() / r.abs().max()) for p, r in zip(g, gref))
        tf = time_launches([f], args.iters, dev)
        td = time_launches([d], args.iters, dev)
        row.append(f"{v}: fwd {tf * 1e6:7.1f} us {flop / tf / 1e12:5.1f} TF/s dgrad {td * 1e6:7.1f} us "
                   f"{flop / td / 1e12:5.1f} (err {ey:.1e}/{eg:.1e} repeat {same})")
    lib.mrp_tuning_set(b"gemm_split", -1)
    print(" | ".join(row), flush=True)
