"""Kernel lab (not product code): the configs[1] training step (GCNBlock, 2 layers, B=16, N=8, C=512,
32x32) through the concatenation-free layer (FilmCompressFunction) against the cat kernel + batched
GEMM path, timed alternately; plus a torch-profiler op table of one step of each.

Usage: python tools/exp_train_dual.py
"""
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload  # noqa: E402

dev = torch.device("cuda:0")


def main():
    B, N, C, H = 16, 8, 512, 32
    g = make_workload(B, N, C, H, H, seed=1, device=dev)
    x0 = g.ndata["image"]
    torch.manual_seed(0)
    net = mrp.GCNBlock(types.SimpleNamespace(feature_dim=C, compress_gcn=True, multi_gcn=True)).to(dev)
    G = torch.randn_like(x0)

    def step():
        net.zero_grad(set_to_none=True)
        x = x0.detach().requires_grad_(True)
        (net(g, x) * G).sum().backward()

    def timeit(n=10):
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            step()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / n

    res = {True: [], False: []}
    for _ in range(4):
        for setting in (True, False):
            mrp.models.set_training_compress(setting)
            res[setting].append(timeit())
    for k, v in res.items():
        print(f"set_training_compress({k}): train step {sorted(v)[len(v) // 2]:.3f} ms  (all {['%.3f' % t for t in v]})")
    for setting in (True, False):
        mrp.models.set_training_compress(setting)
        step()
        torch.cuda.synchronize()
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            step()
            torch.cuda.synchronize()
        print(f"--- set_training_compress({setting})")
        print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=14))
    mrp.models.set_training_compress(False)


if __name__ == "__main__":
    main()
