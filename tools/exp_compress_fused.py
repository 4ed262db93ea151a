"""Experiment (not product code): the fused aggregation + compress kernel against the unfused path
(cat kernel + batched library GEMM) at the BASELINE config shapes, HIP-graph-timed like bench.py."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload, time_launches  # noqa: E402
from mrp_gnn_amd.compress import compress_1x1, compress_dual, compress_film_fused  # noqa: E402

dev = torch.device("cuda:0")
MODE = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
lib = mrp.load_library()
lib.mrp_compress_film_debug.argtypes = [__import__("ctypes").c_int]
for name, (B, N, C, H) in {"cfg1": (16, 8, 512, 32), "cfg2": (32, 8, 1280, 8), "cfg3": (8, 8, 2048, 8)}.items():
    g = make_workload(B, N, C, H, H, seed=1, device=dev)
    x = g.ndata["image"]
    torch.manual_seed(0)
    gcn = mrp.GCN(type("O", (), {"feature_dim": C})()).to(dev)
    conv = torch.nn.Conv2d(2 * C, C, 1).to(dev)
    csr = g.csr(dev)
    with torch.no_grad():
        z = gcn.edge_encoder.logits(g.edata["pose"])
        cat = torch.empty(x.shape[0], 2 * C, H, H, device=dev)
        t_cat = time_launches([lambda: mrp.film_mean_cat_forward_into(x, z, csr, MODE, cat)], 20, dev)
        t_gemm = time_launches([lambda: compress_1x1(conv, cat)], 20, dev)
        flop = 2 * x.shape[0] * H * H * C * 2 * C
        t_fused = time_launches([lambda: compress_film_fused(conv, x, z, csr, MODE)], 20, dev)
        agg = torch.empty_like(x)
        t_agg = time_launches([lambda: mrp.film_mean_forward_into(x, z, csr, MODE, agg)], 20, dev)
        t_dual = time_launches([lambda: compress_dual(conv, x, agg)], 20, dev)
        print(f"{name}: two-pass: aggregate {t_agg * 1e6:8.1f} us + dual GEMM {t_dual * 1e6:8.1f} us "
              f"({flop / t_dual / 1e12:6.1f} TF/s) = {(t_agg + t_dual) * 1e6:8.1f} us", flush=True)
        lab = []
        for mode in (1, 2):  # 1: consumers only (MFMA bound), 2: producers only
            lib.mrp_compress_film_debug(mode)
            lab.append(time_launches([lambda: compress_film_fused(conv, x, z, csr, MODE)], 20, dev))
        lib.mrp_compress_film_debug(32)
        t_noprio = time_launches([lambda: compress_film_fused(conv, x, z, csr, MODE)], 20, dev)
        lib.mrp_compress_film_debug(64)
        t_bm256 = time_launches([lambda: compress_film_fused(conv, x, z, csr, MODE)], 20, dev)
        lib.mrp_compress_film_debug(0)
        print(f"{name}: fused without producer priority {t_noprio * 1e6:8.1f} us, with BM 256 {t_bm256 * 1e6:8.1f} us",
              flush=True)
        print(f"{name}: lab consumers-only {lab[0] * 1e6:8.1f} us ({flop / lab[0] / 1e12:6.1f} TF/s)  "
              f"producers-only {lab[1] * 1e6:8.1f} us", flush=True)
        print(f"{name}: cat {t_cat * 1e6:8.1f} us + gemm {t_gemm * 1e6:8.1f} us ({flop / t_gemm / 1e12:6.1f} TF/s) "
              f"= {(t_cat + t_gemm) * 1e6:8.1f} us | fused {t_fused * 1e6:8.1f} us ({flop / t_fused / 1e12:6.1f} TF/s)",
              flush=True)
    del g, x, z, cat, conv, gcn
    torch.cuda.empty_cache()
