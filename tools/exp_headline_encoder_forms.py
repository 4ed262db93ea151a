"""Kernel lab (not product code): the headline step (bench.py's no-grad GCN.forward, B = 32, N = 8,
C = 512, 32 x 32) per setting of an encoder knob (default edge_split_v: -1, 1, 3; or the knob and values
given), timed like bench.py (spin-up, warmup, barrier-free synchronize-bracketed steps), settings
interleaved over rounds.
usage: python tools/exp_headline_encoder_forms.py [steps] [knob] [values, e.g. 0,1]"""
import os
import sys
import time
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
knob = sys.argv[2] if len(sys.argv) > 2 else "edge_split_v"
values = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [-1, 1, 3]
dev = torch.device("cuda:0")
g = bench.make_workload(32, 8, 512, 32, 32, seed=0, device=dev)
x = g.ndata["image"]
torch.manual_seed(0)
gcn = mrp.GCN(types.SimpleNamespace(feature_dim=512)).to(dev)
lib = mrp.load_library()
res = {}
with torch.no_grad():
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _ in range(20):
            gcn(g, x)
        torch.cuda.synchronize()
    for rnd in range(4):
        for v in values:
            assert lib.mrp_tuning_set(knob.encode(), v) == 0
            for _ in range(10):
                gcn(g, x)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(steps):
                gcn(g, x)
            torch.cuda.synchronize()
            res.setdefault(v, []).append((time.perf_counter() - t) / steps * 1e6)
lib.mrp_tuning_set(b"reset", 0)
for v, ts in res.items():
    print(f"{knob} {v:2d}: " + " ".join(f"{t:6.1f}" for t in ts) + f"  min {min(ts):6.1f} us/step", flush=True)
