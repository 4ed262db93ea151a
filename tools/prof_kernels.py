"""Profiling driver (not product code): runs the forward and backward aggregation kernels of every
BASELINE config shape a fixed number of times, on rotating buffer sets (bench.py's method), so one
``rocprofv3 --kernel-trace --stats`` or ``--pmc`` pass sees each kernel at the bench workload's size
without the rest of bench.py.  Usage: python tools/prof_kernels.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload, rotating_sets  # noqa: E402

SHAPES = {  # name: (B, N, C, H, knn) -- bench.py CONFIGS and the headline
    "north_star": (32, 8, 512, 32, None),
    "cfg1": (16, 8, 512, 32, None),
    "cfg2": (32, 8, 1280, 8, None),
    "cfg3": (8, 8, 2048, 8, None),
    "cfg4": (8, 16, 1024, 16, 4),
}
MODE = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else list(SHAPES)
    dev = torch.device("cuda:0")
    for name in only:
        B, N, C, H, knn = SHAPES[name]
        g = make_workload(B, N, C, H, H, seed=1, device=dev, knn=knn)
        torch.manual_seed(0)
        gcn = mrp.GCN(type("O", (), {"feature_dim": C})()).to(dev)
        csr = g.csr(dev)
        x = g.ndata["image"]
        with torch.no_grad():
            z = gcn.edge_encoder.logits(g.edata["pose"])
        plane = x.numel() * 4
        nf = rotating_sets(2 * plane)
        sets = [(x if i == 0 else torch.randn_like(x), torch.empty_like(x)) for i in range(nf)]
        for i in range(iters):
            a, o = sets[i % nf]
            mrp.film_mean_forward_into(a, z, csr, MODE, o)
        torch.cuda.synchronize()
        del sets
        nb = rotating_sets(3 * plane)
        bsets = [(torch.randn_like(x), x if i == 0 else torch.randn_like(x)) for i in range(nb)]
        for i in range(iters):
            G, a = bsets[i % nb]
            mrp.aggregate.film_mean_backward(G, a, z, csr, MODE, True, True)
        torch.cuda.synchronize()
        del bsets, g, gcn, csr, x, z
        torch.cuda.empty_cache()
        print(f"{name}: {iters} forward + {iters} backward launches", flush=True)


if __name__ == "__main__":
    main()
