"""Kernel lab (not product code): the aggregation backward at the headline and configs[1..3] shapes with
both outputs, dx only and d(gamma, beta) only, HIP-graph timed on rotating buffers like bench.py, to
price the Gram / lane reduction / d(gamma, beta) epilogue against the dx stream.
usage: python tools/exp_bwd_parts.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402
from mrp_gnn_amd import _lib  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
mode = _lib.MODE_FILM_MEAN | _lib.GB_LOGITS
for name, B, N, C, H in [("north_star", 32, 8, 512, 32), ("cfg1", 16, 8, 512, 32), ("cfg2", 32, 8, 1280, 8),
                         ("cfg3", 8, 8, 2048, 8)]:
    g = bench.make_workload(B, N, C, H, H, seed=3, device=dev)
    x = g.ndata["image"]
    csr = g.csr(dev)
    torch.manual_seed(0)
    z = torch.randn(g.num_edges(), 2 * C, device=dev)
    nb = bench.rotating_sets(3 * x.numel() * 4)
    sets = [(torch.randn_like(x), x if i == 0 else torch.randn_like(x)) for i in range(nb)]
    res = {}
    for _ in range(3):
        for dx, dgb in ((True, True), (True, False), (False, True)):
            fs = [lambda G=G, xi=xi, dx=dx, dgb=dgb: mrp.aggregate.film_mean_backward(G, xi, z, csr, mode, dx, dgb)
                  for G, xi in sets]
            res.setdefault((dx, dgb), []).append(bench.time_launches(fs, iters, dev))
    print(f"{name:10s} both {min(res[(True, True)]) * 1e6:7.1f} us  dx only {min(res[(True, False)]) * 1e6:7.1f}"
          f"  dgb only {min(res[(False, True)]) * 1e6:7.1f}", flush=True)
    del sets
    torch.cuda.empty_cache()
