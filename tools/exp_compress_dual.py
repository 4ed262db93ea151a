"""Kernel lab (not product code): the layer's compress without the cat buffer — aggregate kernel +
mrp_compress_dual_fwd — against cat kernel + batched library GEMM at every BASELINE config shape
(including the k-NN one), HIP-graph timed (bench.time_launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload, time_launches  # noqa: E402
from mrp_gnn_amd.compress import compress_1x1, compress_dual  # noqa: E402

dev = torch.device("cuda:0")
MODE = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
SHAPES = {"cfg1": (16, 8, 512, 32, None), "cfg2": (32, 8, 1280, 8, None), "cfg3": (8, 8, 2048, 8, None),
          "cfg4": (8, 16, 1024, 16, 4)}
for name, (B, N, C, H, knn) in SHAPES.items():
    g = make_workload(B, N, C, H, H, seed=1, device=dev, knn=knn)
    x = g.ndata["image"]
    torch.manual_seed(0)
    gcn = mrp.GCN(type("O", (), {"feature_dim": C})()).to(dev)
    conv = torch.nn.Conv2d(2 * C, C, 1).to(dev)
    csr = g.csr(dev)
    with torch.no_grad():
        z = gcn.edge_encoder.logits(g.edata["pose"])
        cat = torch.empty(x.shape[0], 2 * C, H, H, device=dev)
        agg = torch.empty_like(x)
        t_cat = time_launches([lambda: mrp.film_mean_cat_forward_into(x, z, csr, MODE, cat)], 20, dev)
        t_gemm = time_launches([lambda: compress_1x1(conv, cat)], 20, dev)
        t_agg = time_launches([lambda: mrp.film_mean_forward_into(x, z, csr, MODE, agg)], 20, dev)
        t_dual = time_launches([lambda: compress_dual(conv, x, agg)], 20, dev)
        lib = mrp.load_library()
        lib.mrp_compress_film_debug(128)  # W fragments by ds_read_b128 (the four-b32 form is the default)
        t_wide = time_launches([lambda: compress_dual(conv, x, agg)], 20, dev)
        lib.mrp_compress_film_debug(0)
        flop = 2 * x.shape[0] * H * H * C * 2 * C
        print(f"{name}: dual GEMM narrow-A {t_dual * 1e6:7.1f} us ({flop / t_dual / 1e12:5.1f} TF/s), "
              f"wide-A {t_wide * 1e6:7.1f} us ({flop / t_wide / 1e12:5.1f} TF/s)", flush=True)
        print(f"{name}: cat {t_cat * 1e6:7.1f} + library GEMM {t_gemm * 1e6:7.1f} us ({flop / t_gemm / 1e12:5.1f} TF/s)"
              f" = {(t_cat + t_gemm) * 1e6:7.1f} us | aggregate {t_agg * 1e6:7.1f} + dual {t_dual * 1e6:7.1f} us "
              f"({flop / t_dual / 1e12:5.1f} TF/s) = {(t_agg + t_dual) * 1e6:7.1f} us", flush=True)
    del g, x, z, cat, agg, conv, gcn
    torch.cuda.empty_cache()
