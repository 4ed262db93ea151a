"""Experiment (not product code): one GCN forward with the encoder's second Linear split into graph
chunks on a HIGH-PRIORITY side stream, so chunk i+1's GEMM (MFMA-bound) runs beside chunk i's
aggregation (HBM-bound) instead of before it.  (tools/exp_overlap.py did the same on a
default-priority stream and lost: 283 vs 243 us.)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
W2t = l2.weight.t()


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


print("stream priority range", torch.cuda.Stream.priority_range(), flush=True)
with torch.no_grad():
    ref = gcn(g, x)
    print(f"GCN forward (serial)   {timeit(lambda: gcn(g, x)):8.1f} us", flush=True)
    z = gcn.edge_encoder.logits(pose)
    out = torch.empty_like(x)
    print(f"aggregation only       {timeit(lambda: mrp.film_mean_forward_into(x, z, csr, mode, out)):8.1f} us",
          flush=True)
    hh = mrp.encoder.hidden_forward(pose, l1.weight, l1.bias)
    print(f"hidden kernel          {timeit(lambda: mrp.encoder.hidden_forward(pose, l1.weight, l1.bias)):8.1f} us",
          flush=True)
    print(f"addmm (all edges)      {timeit(lambda: torch.addmm(l2.bias, hh, W2t)):8.1f} us", flush=True)

    for prio in (-1, 0):
        side = torch.cuda.Stream(dev, priority=prio)
        for S in (2, 4, 8):
            gpc = B // S
            sub = csr._replace(num_graphs=gpc, num_nodes=gpc * N, num_edges=gpc * N * (N - 1))
            ecut = [i * gpc * N * (N - 1) for i in range(S + 1)]
            ncut = [i * gpc * N for i in range(S + 1)]
            evs = [torch.cuda.Event() for _ in range(S)]
            zbuf = torch.empty(E, 2 * C, device=dev)

            def pipelined(first_on_main):
                cur = torch.cuda.current_stream(dev)
                h = mrp.encoder.hidden_forward(pose, l1.weight, l1.bias)
                o = torch.empty_like(x)
                start = 0
                if first_on_main:
                    torch.addmm(l2.bias, h[ecut[0]:ecut[1]], W2t, out=zbuf[ecut[0]:ecut[1]])
                    start = 1
                ready = torch.cuda.Event()
                ready.record(cur)
                side.wait_event(ready)
                with torch.cuda.stream(side):
                    for i in range(start, S):
                        torch.addmm(l2.bias, h[ecut[i]:ecut[i + 1]], W2t, out=zbuf[ecut[i]:ecut[i + 1]])
                        evs[i].record(side)
                for i in range(S):
                    if i >= start:
                        cur.wait_event(evs[i])
                    mrp.film_mean_forward_into(x[ncut[i]:ncut[i + 1]], zbuf[ecut[i]:ecut[i + 1]].view(-1, C, 2), sub,
                                               mode, o[ncut[i]:ncut[i + 1]])
                h.record_stream(side)
                return o

            for fom in (False, True):
                got = pipelined(fom)
                torch.cuda.synchronize()
                print(f"prio={prio:2d} S={S} first_on_main={int(fom)}  {timeit(lambda: pipelined(fom)):8.1f} us  "
                      f"equal={torch.equal(ref, got)}", flush=True)
