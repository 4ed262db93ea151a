"""Experiment: overlap the encoder's second Linear (library GEMM) with the aggregation by splitting
the batch into graph chunks on two streams.  Not product code."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload  # noqa: E402

dev = torch.device("cuda:0")
B, N, C, HW = 32, 8, 512, 32
g = make_workload(B, N, C, HW, HW, seed=0, device=dev)
x = g.ndata["image"]
torch.manual_seed(0)
gcn = mrp.GCN(type("O", (), {"feature_dim": C})()).to(dev)
pose = g.edata["pose"]
csr = g.csr(dev)
E = g.num_edges()
l1, l2 = gcn.edge_encoder.layers[0], gcn.edge_encoder.layers[2]
mode = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


h = mrp.encoder.hidden_forward(pose, l1.weight, l1.bias)
W2t = l2.weight.t()
for lib in ["default", "cublaslt", "cublas"]:
    if lib != "default":
        torch.backends.cuda.preferred_blas_library(lib)
    print(f"addmm {lib:9s} {timeit(lambda: torch.addmm(l2.bias, h, W2t)):8.1f} us", flush=True)
torch.backends.cuda.preferred_blas_library("default") if hasattr(torch.backends.cuda, "preferred_blas_library") else None

with torch.no_grad():
    print(f"GCN forward        {timeit(lambda: gcn(g, x)):8.1f} us", flush=True)
    z = gcn.edge_encoder.logits(pose)
    out = torch.empty_like(x)
    print(f"aggregation only   {timeit(lambda: mrp.film_mean_forward_into(x, z, csr, mode, out)):8.1f} us", flush=True)

    # chunked pipeline
    side = torch.cuda.Stream(dev)
    for S in [2, 4, 8]:
        gpc = B // S
        chunks = []
        for i in range(S):
            sub = mrp.batch([mrp.complete_graph(N) for _ in range(gpc)])
            chunks.append((i * gpc * N, (i + 1) * gpc * N, i * gpc * N * (N - 1), (i + 1) * gpc * N * (N - 1),
                           sub.csr(dev)))
        zbuf = torch.empty(E, 2 * C, device=dev)
        evs = [torch.cuda.Event() for _ in range(S)]

        def pipelined():
            hh = mrp.encoder.hidden_forward(pose, l1.weight, l1.bias)
            o = torch.empty_like(x)
            ready = torch.cuda.Event()
            ready.record()
            with torch.cuda.stream(side):
                side.wait_event(ready)
                for i, (n0, n1, e0, e1, _) in enumerate(chunks):
                    torch.addmm(l2.bias, hh[e0:e1], W2t, out=zbuf[e0:e1])
                    evs[i].record(side)
            for i, (n0, n1, e0, e1, c) in enumerate(chunks):
                torch.cuda.current_stream().wait_event(evs[i])
                mrp.film_mean_forward_into(x[n0:n1], zbuf[e0:e1].view(-1, C, 2), c, mode, o[n0:n1])
            return o

        ref = gcn(g, x)
        got = pipelined()
        torch.cuda.synchronize()
        print(f"pipelined S={S}     {timeit(pipelined):8.1f} us  equal={torch.equal(ref, got)}", flush=True)
