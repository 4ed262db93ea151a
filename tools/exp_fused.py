#!/usr/bin/env python3
"""Kernel lab (not product code): the no-grad GCN layer at the headline shape (bench.py's step) as ONE
launch (mrp_gcn_fwd_fused) against the two launches (encoder + film_fwd), interleaved in one process:
eager steps timed like bench.py (barrier-free, synchronize on both sides) and HIP-graph replays, plus a
sweep of the producer count.
usage: python tools/exp_fused.py [steps] [rounds] [producers,...]"""
import os
import sys
import time
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

lib = mrp.load_library()

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
# producer counts, each optionally with lab bits: "128" or "128:6" (Tuning::fused_lab)
prods = sys.argv[3].split(",") if len(sys.argv) > 3 else ["128"]


def setp(spec):
    p, _, lab = spec.partition(":")
    assert lib.mrp_tuning_set(b"fused_producers", int(p)) == 0
    assert lib.mrp_tuning_set(b"fused_lab", int(lab or 0)) == 0
B, N, C, H = int(os.environ.get("B", 32)), 8, int(os.environ.get("C", 512)), int(os.environ.get("H", 32))
dev = torch.device("cuda:0")
g = bench.make_workload(B, N, C, H, H, seed=0, device=dev)
torch.manual_seed(0)
gcn = mrp.GCN(types.SimpleNamespace(feature_dim=C)).to(dev)
x = g.ndata["image"]


def step():
    return gcn(g, x)


def eager(n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def graphed(n):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=side):
        for _ in range(n):
            step()
    gr.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        gr.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / n)
    return sorted(ts)[1]


with torch.no_grad():
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:  # clock ramp (bench.py spinup)
        for _ in range(20):
            step()
        torch.cuda.synchronize()
    ref = None
    mrp.fused.set_fused_forward(False)
    ref = step().clone()
    mrp.fused.set_fused_forward(True)
    for p in prods:
        setp(p)
        out = step()
        print(f"producers {p}: bit-identical {torch.equal(out, ref)}, err word {mrp.fused.error_word(dev)}", flush=True)
    res = {}
    for r in range(rounds):
        for label in ["two"] + [f"fused{p}" for p in prods]:
            if label == "two":
                mrp.fused.set_fused_forward(False)
            else:
                mrp.fused.set_fused_forward(True)
                setp(label[5:])
            for _ in range(10):
                step()
            e = eager(steps)
            gt = graphed(min(steps, 50))
            res.setdefault(label, []).append((e, gt))
            print(f"round {r} {label:10s} eager {e:7.2f} us/step  graph {gt:7.2f} us/step", flush=True)
    mrp.fused.set_fused_forward(True)
    setp("128")
    for k, v in res.items():
        es = sorted(a for a, _ in v)
        gs = sorted(b for _, b in v)
        print(f"median {k:10s} eager {es[len(es) // 2]:7.2f}  graph {gs[len(gs) // 2]:7.2f}  "
              f"-> {B * N * C * H * H / es[len(es) // 2] * 1e6:.4e} elems/s eager")
