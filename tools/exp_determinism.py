"""Kernel lab (not product code): run-to-run determinism of the compress kernels and the aggregate.

Each kernel is launched REPS times on the same inputs; every output is compared with the first and the
fused kernel with the two-source one.  Prints the number of differing runs and the largest difference.

Usage: python tools/exp_determinism.py
"""
import os
import sys
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as m  # noqa: E402
from mrp_gnn_amd.compress import compress_dual, compress_film_fused  # noqa: E402

REPS = int(os.environ.get("REPS", "40"))
dev = torch.device("cuda:0")


def frames(B, N, C, H, seed):
    rng = np.random.RandomState(seed)
    gs = [m.frame_graph(np.concatenate([rng.uniform(-10, 10, (N, 3)), rng.standard_normal((N, 4))], 1)
                        .astype(np.float32)) for _ in range(B)]
    g = m.batch(gs)
    torch.manual_seed(seed)
    g.ndata["image"] = torch.randn(g.num_nodes(), C, H, H)
    return g


def check(name, fn):
    ref = fn().clone()
    bad, worst = 0, 0.0
    for _ in range(REPS):
        y = fn()
        if not torch.equal(y, ref):
            bad += 1
            worst = max(worst, float((y - ref).abs().max()))
    print(f"{name:40s} differing runs {bad}/{REPS}  max |diff| {worst:.3e}", flush=True)
    return ref


def main():
    for (B, N, C, H) in [(3, 8, 256, 8), (3, 8, 128, 4), (16, 8, 512, 32), (3, 5, 256, 8)]:
        g = frames(B, N, C, H, seed=4).to(dev)
        x = g.ndata["image"]
        csr = g.csr(dev)
        torch.manual_seed(1)
        conv = torch.nn.Conv2d(2 * C, C, 1).to(dev)
        z = torch.randn(g.num_edges(), 2 * C, device=dev)
        mode = m._lib.MODE_FILM_MEAN | m._lib.GB_LOGITS
        tag = f"B{B} N{N} C{C} {H}x{H}"
        with torch.no_grad():
            agg = check(f"aggregate {tag}", lambda: m.film_mean(x, z, csr, logits=True))
            dual = check(f"dual {tag}", lambda: compress_dual(conv, x, agg))
            if N <= 8:
                fused = check(f"fused {tag}", lambda: compress_film_fused(conv, x, z, csr, mode))
                print(f"{'fused == dual ' + tag:40s} {torch.equal(fused, dual)}  "
                      f"max |diff| {float((fused - dual).abs().max()):.3e}", flush=True)
            opt = types.SimpleNamespace(feature_dim=C, compress_gcn=True, multi_gcn=True)
            torch.manual_seed(1)
            net = m.GCNBlock(opt).to(dev)
            prev = m.models.fused_compress_setting()
            try:
                for s in ("fused", True):
                    m.models.set_fused_compress(s)
                    check(f"stack[{s}] {tag}", lambda: net(g, x))
            finally:
                m.models.set_fused_compress(prev)


if __name__ == "__main__":
    main()
