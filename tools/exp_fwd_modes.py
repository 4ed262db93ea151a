"""Kernel lab (not product code): the forward aggregation at the config shapes with gamma/beta as
logits (product), post-sigmoid (no sigmoid in the prologue) and copy_mean (no gamma/beta loads at
all), to price the prologue.  HIP-graph timing on rotating buffers (bench.time_launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import alg_bytes_fwd, rotating_sets, time_launches  # noqa: E402
from tools.sweep_geometry import SHAPES, setup  # noqa: E402

dev = torch.device("cuda:0")
L = mrp._lib
for name in ("cfg1", "cfg2", "cfg3", "north_star"):
    g, z, csr = setup(name)
    x = g.ndata["image"]
    Nt, C, H, W = x.shape
    gb = torch.sigmoid(z)
    nf = rotating_sets(2 * x.numel() * 4)
    sets = [(x if i == 0 else torch.randn_like(x), torch.empty_like(x)) for i in range(nf)]
    row = []
    for label, gbt, mode in (("logits", z, L.MODE_FILM_MEAN | L.GB_LOGITS), ("post-sigmoid", gb, L.MODE_FILM_MEAN),
                             ("copy_mean", None, L.MODE_COPY_MEAN)):
        launches = [lambda a=a, o=o, gbt=gbt, mode=mode: mrp.film_mean_forward_into(a, gbt, csr, mode, o) for a, o in sets]
        t = time_launches(launches, 40, dev)
        row.append(f"{label} {t * 1e6:6.1f} us ({alg_bytes_fwd(Nt, g.num_edges(), C, H * W) / t / 8e12 * 100:4.1f} %)")
    print(f"{name}: " + " | ".join(row), flush=True)
    del sets, g, z, csr, x
    torch.cuda.empty_cache()
