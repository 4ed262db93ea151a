"""Experiment (not product code): how long a fresh process needs before the aggregation kernel runs
at its steady-state speed (clock / memory power-state ramp).  Launches the north-star aggregation
back to back from a cold start and prints the mean launch time per window of launches (HIP events)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload  # noqa: E402

dev = torch.device("cuda:0")
g = make_workload(32, 8, 512, 32, 32, seed=0, device=dev)
x = g.ndata["image"]
torch.manual_seed(0)
gcn = mrp.GCN(type("O", (), {"feature_dim": 512})()).to(dev)
csr = g.csr(dev)
MODE = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
with torch.no_grad():
    z = gcn.edge_encoder.logits(g.edata["pose"])
    out = torch.empty_like(x)
    torch.cuda.synchronize()
    time.sleep(float(os.environ.get("IDLE", "2")))  # idle like bench.py's host-side setup
    W = 25
    t_start = time.perf_counter()
    for w in range(int(os.environ.get("WINDOWS", "60"))):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(W):
            mrp.film_mean_forward_into(x, z, csr, MODE, out)
        b.record()
        b.synchronize()
        print(f"window {w:3d} t={time.perf_counter() - t_start:7.3f}s  {a.elapsed_time(b) / W * 1e3:7.1f} us/launch",
              flush=True)
    # steps of the layer, cold again after an idle second
    time.sleep(1.0)
    for w in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            gcn(g, x)
        torch.cuda.synchronize()
        print(f"step window {w:2d}: {(time.perf_counter() - t0) / 20 * 1e6:7.1f} us/step", flush=True)
