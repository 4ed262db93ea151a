"""Experiment (not product code): where the north-star step's time goes, and which way of running
the edge encoder beside the aggregation shortens it.

Variants, each timed like bench.py (host clock around K back-to-back steps, synchronised):
  serial        encoder (hidden kernel + addmm) then the aggregation, eager
  *_graph       the same sequence captured once in a HIP graph and replayed
  chan[a|b|..]  channel chunks: the encoder GEMM of chunk i+1 on a side stream beside the
                aggregation of chunk i (x / out read and written through channel-sliced views)
  graphs S      graph chunks (round 1's negative result, re-measured under graph replay)
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload  # noqa: E402

dev = torch.device("cuda:0")
B, N, C, HW = 32, 8, 512, 32
K = int(os.environ.get("STEPS", "50"))
g = make_workload(B, N, C, HW, HW, seed=0, device=dev)
x = g.ndata["image"]
torch.manual_seed(0)
gcn = mrp.GCN(type("O", (), {"feature_dim": C})()).to(dev)
pose = g.edata["pose"]
csr = g.csr(dev)
E = g.num_edges()
l1, l2 = gcn.edge_encoder.layers[0], gcn.edge_encoder.layers[2]
W1, b1, W2, b2 = l1.weight.detach(), l1.bias.detach(), l2.weight.detach(), l2.bias.detach()
MODE = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
P = HW * HW


def timeit(fn, iters=K):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def graphed(fn):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    cg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(cg):
        res = fn()
    cg.replay()
    torch.cuda.synchronize()
    return cg, res


side = torch.cuda.Stream(dev)


def make_chan(bounds):
    nck = len(bounds) - 1
    evs = [torch.cuda.Event() for _ in range(nck)]

    def step():
        cur = torch.cuda.current_stream(dev)
        side.wait_stream(cur)
        out = torch.empty_like(x)
        zs = []
        with torch.cuda.stream(side):
            h = mrp.encoder.hidden_forward(pose, W1, b1)
            for i in range(nck):
                r0, r1 = 2 * bounds[i], 2 * bounds[i + 1]
                zs.append(torch.addmm(b2[r0:r1], h, W2[r0:r1].t()))
                evs[i].record(side)
        for i in range(nck):
            c0, c1 = bounds[i], bounds[i + 1]
            cur.wait_event(evs[i])
            zs[i].record_stream(cur)
            mrp.film_mean_forward_into(x[:, c0:c1], zs[i].view(E, c1 - c0, 2), csr, MODE, out[:, c0:c1])
        h.record_stream(side)
        return out

    return step


def make_graph_chunks(S):
    gpc = B // S
    sub = csr._replace(num_graphs=gpc, num_nodes=gpc * N, num_edges=gpc * N * (N - 1))
    ecut = [i * gpc * N * (N - 1) for i in range(S + 1)]
    ncut = [i * gpc * N for i in range(S + 1)]
    evs = [torch.cuda.Event() for _ in range(S)]

    def step():
        cur = torch.cuda.current_stream(dev)
        side.wait_stream(cur)
        out = torch.empty_like(x)
        z = torch.empty(E, 2 * C, device=dev)
        with torch.cuda.stream(side):
            h = mrp.encoder.hidden_forward(pose, W1, b1)
            for i in range(S):
                torch.addmm(b2, h[ecut[i]:ecut[i + 1]], W2.t(), out=z[ecut[i]:ecut[i + 1]])
                evs[i].record(side)
        for i in range(S):
            cur.wait_event(evs[i])
            mrp.film_mean_forward_into(x[ncut[i]:ncut[i + 1]], z[ecut[i]:ecut[i + 1]].view(-1, C, 2), sub, MODE,
                                       out[ncut[i]:ncut[i + 1]])
        h.record_stream(side)
        return out

    return step


def main():
    with torch.no_grad():
        ref = gcn(g, x)
        z = gcn.edge_encoder.logits(pose)
        out = torch.empty_like(x)
        h = mrp.encoder.hidden_forward(pose, W1, b1)
        variants = {
            "aggregation only": lambda: mrp.film_mean_forward_into(x, z, csr, MODE, out),
            "encoder only (eager)": lambda: gcn.edge_encoder.logits(pose),
            "serial eager": lambda: gcn(g, x),
        }
        cg_serial, o = graphed(lambda: gcn(g, x))
        assert torch.equal(o, ref)
        variants["serial graph"] = cg_serial.replay
        for bounds in ([0, 32, 512], [0, 64, 512], [0, 128, 512], [0, 32, 128, 512]):
            st = make_chan(bounds)
            assert torch.equal(st(), ref)
            variants[f"chan {bounds[1:-1]} eager"] = st
            cg, o = graphed(st)
            assert torch.equal(o, ref)
            variants[f"chan {bounds[1:-1]} graph"] = cg.replay
        for S in (2,):
            st = make_graph_chunks(S)
            assert torch.equal(st(), ref)
            variants[f"graphs S={S} eager"] = st
            cg, o = graphed(st)
            variants[f"graphs S={S} graph"] = cg.replay
        res = {k: [] for k in variants}
        for rep in range(int(os.environ.get("REPS", "4"))):
            for k, fn in variants.items():
                res[k].append(timeit(fn))
        for k, v in res.items():
            v = sorted(v)
            print(f"{k:28s} min {v[0]:8.1f}  median {v[len(v) // 2]:8.1f}  all {' '.join(f'{t:.1f}' for t in v)}",
                  flush=True)


if __name__ == "__main__":
    main()
