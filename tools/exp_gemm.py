"""Kernel lab (not product code): the matrix-core compress kernels of csrc/compress_gemm.hip
(forward, data gradient, weight gradient) — every variant of the kernel family (mrp_tuning_set
"gemm_nn" / "gemm_nt") — against the library GEMMs torch uses for the same products at every
BASELINE config's per-GPU layer shape, HIP-graph timed (bench.time_launches).
TF/s = 2 Nt P C 2C / t for each of the three products.  Each variant is also checked against the
library result (max |d| / max |ref|), so a broken variant shows as a large error, not a fast time.

usage: python tools/exp_gemm.py [shape ...] [--variants 0,1,...] [--library]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import time_launches  # noqa: E402
from mrp_gnn_amd import compress as cp  # noqa: E402

SHAPES = {"cfg1": (128, 512, 32), "cfg2": (256, 1280, 8), "cfg3": (64, 2048, 8), "cfg4": (128, 1024, 16),
          "head": (256, 512, 32)}
ap = argparse.ArgumentParser()
ap.add_argument("shapes", nargs="*", default=["cfg1", "cfg2", "cfg3", "cfg4"])
ap.add_argument("--variants", default="0,1,2,3,4,5")
ap.add_argument("--library", action="store_true", help="also time torch's library GEMMs")
ap.add_argument("--iters", type=int, default=10)
args = ap.parse_args()
dev = torch.device("cuda:0")
lib = mrp.load_library()


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


for name in args.shapes:
    n, C, H = SHAPES[name]
    torch.manual_seed(0)
    x = torch.randn(n, C, H, H, device=dev)
    a = torch.randn(n, C, H, H, device=dev)
    gy = torch.randn(n, C, H, H, device=dev)
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    b = torch.randn(C, device=dev)
    cat = torch.cat((x, a), 1)
    P = H * H
    flop = 2.0 * n * P * C * 2 * C
    w2 = w.reshape(C, 2 * C)
    tf = lambda t: flop / t / 1e12  # noqa: E731
    with torch.no_grad():
        ref_y = torch.baddbmm(b.view(1, C, 1), w2.expand(n, C, 2 * C), cat.view(n, 2 * C, P)).view(n, C, H, H)
        ref_d = torch.bmm(w2.t().expand(n, 2 * C, C), gy.view(n, C, P)).view(n, 2 * C, H, H)
        ref_w = cp._lib_backward_weight(gy, x, a, False)[0]
        if args.library:
            it = args.iters
            t_fl = time_launches([lambda: torch.baddbmm(b.view(1, C, 1), w2.expand(n, C, 2 * C), cat.view(n, 2 * C, P))],
                                 it, dev)
            t_dl = time_launches([lambda: torch.bmm(w2.t().expand(n, 2 * C, C), gy.view(n, C, P))], it, dev)
            t_wl = time_launches([lambda: cp._lib_backward_weight(gy, x, a, True)], it, dev)
            print(f"{name} Nt={n} C={C} {H}x{H} library: fwd {t_fl * 1e6:7.1f} us {tf(t_fl):5.1f} | data {t_dl * 1e6:7.1f} "
                  f"{tf(t_dl):5.1f} | weight {t_wl * 1e6:7.1f} {tf(t_wl):5.1f}", flush=True)
        for v in [int(s) for s in args.variants.split(",")]:
            assert lib.mrp_tuning_set(b"gemm_nn", v) == 0 and lib.mrp_tuning_set(b"gemm_nt", v) == 0
            y = cp.compress_forward(w, b, x, a)
            gx, ga = cp.compress_backward_data(w, gy)
            dw, db = cp.compress_backward_weight(gy, x, a)
            err = max(rel(y, ref_y), rel(torch.cat((gx, ga), 1), ref_d), rel(dw, ref_w), rel(db, gy.sum((0, 2, 3))))
            it = args.iters
            t_f = time_launches([lambda: cp.compress_forward(w, b, x, a)], it, dev)
            t_d = time_launches([lambda: cp.compress_backward_data(w, gy)], it, dev)
            t_w = time_launches([lambda: cp.compress_backward_weight(gy, x, a)], it, dev)
            print(f"{name} Nt={n} C={C} {H}x{H} v{v}: fwd {t_f * 1e6:7.1f} us {tf(t_f):5.1f} TF/s | data {t_d * 1e6:7.1f} "
                  f"{tf(t_d):5.1f} | weight {t_w * 1e6:7.1f} {tf(t_w):5.1f} | ws "
                  f"{lib.mrp_compress_bwd_weight_workspace(n, C, P, C * P) / 2**20:.1f} MiB | err {err:.2e}", flush=True)
        lib.mrp_tuning_set(b"reset", 0)
    del x, a, gy, cat, ref_y, ref_d
    torch.cuda.empty_cache()
