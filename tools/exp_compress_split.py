"""Kernel lab (not product code): the compress forward and data gradient per BASELINE config shape on
the split-bf16 matrix cores (compress_split.hip) against the fp32 MFMA (compress_gemm.hip) and torch's
library GEMM, HIP-graph timed (bench.time_launches); TF/s counts the fp32 product's 2 M N K flops.

usage: python tools/exp_compress_split.py [--iters N]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import time_launches  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
dev = torch.device("cuda:0")
cm = mrp.compress
SHAPES = [("cfg1", 128, 512, 32), ("cfg2", 256, 1280, 8), ("cfg3", 64, 2048, 8), ("cfg4", 128, 1024, 16),
          ("head", 256, 512, 32)]
for name, n, C, H in SHAPES:
    torch.manual_seed(0)
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    b = torch.randn(C, device=dev)
    x, a, gy = (torch.randn(n, C, H, H, device=dev) for _ in range(3))
    flop = 2.0 * C * 2 * C * n * H * H
    row = [f"{name} n={n} C={C} {H}x{H}"]
    ref = None
    lib = mrp.load_library()
    for path in ("split4", "split2", "hip", "library"):
        cm.set_compress_path("split" if path.startswith("split") else path)
        lib.mrp_tuning_set(b"gemm_split", 4 if path == "split4" else 2)
        if path == "library":
            f = lambda: cm._lib_forward(w, b, x, a)
            d = lambda: cm._lib_backward_data(w, gy)
        else:
            f = lambda: cm.compress_forward(w, b, x, a)
            d = lambda: cm.compress_backward_data(w, gy)
        y = f()
        if ref is None:
            ref = cm._lib_forward(w.double(), b.double(), x.double(), a.double())
        err = float((y.double() - ref).abs().max() / ref.abs().max())
        if path == "library":
            wg = lambda: cm._lib_backward_weight(gy, x, a, True)
        else:
            wg = lambda: cm.compress_backward_weight(gy, x, a)
        tf = time_launches([f], args.iters, dev)
        td = time_launches([d], args.iters, dev)
        tw = time_launches([wg], args.iters, dev) if path != "split2" else float("nan")
        row.append(f"{path}: fwd {tf * 1e6:7.1f} us {flop / tf / 1e12:5.1f} TF/s (err {err:.1e}) "
                   f"dgrad {td * 1e6:7.1f} us {flop / td / 1e12:5.1f} wgrad {tw * 1e6:7.1f} us {flop / tw / 1e12:5.1f}")
    cm.set_compress_path("split")
    lib.mrp_tuning_set(b"gemm_split", -1)
    print(" | ".join(row), flush=True)
