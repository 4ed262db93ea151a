"""Kernel lab (not product code): the headline layer's training step (bench.py's ``train_step``: forward,
backward through the HIP kernels and the encoder, B = 32, N = 8, C = 512, 32 x 32) per value of a tuning
knob, timed like bench.py (spin-up, warmup, synchronize-bracketed steps), values interleaved over rounds.
usage: python tools/exp_train_knob.py <knob> <values, e.g. 0,1,2> [steps] [rounds]"""
import os
import sys
import time
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

knob = sys.argv[1]
values = [int(v) for v in sys.argv[2].split(",")]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 4
dev = torch.device("cuda:0")
g = bench.make_workload(32, 8, 512, 32, 32, seed=0, device=dev)
x = g.ndata["image"]
torch.manual_seed(0)
gcn = mrp.GCN(types.SimpleNamespace(feature_dim=512)).to(dev)
lib = mrp.load_library()
xr = x.detach().clone().requires_grad_(True)
gy = torch.randn_like(x)


def step():
    for p in gcn.parameters():
        p.grad = None
    xr.grad = None
    gcn(g, xr).backward(gy)


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    step()
torch.cuda.synchronize()
res = {}
grads = {}
for rnd in range(rounds):
    for v in values:
        assert lib.mrp_tuning_set(knob.encode(), v) == 0
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        res.setdefault(v, []).append((time.perf_counter() - t) / steps * 1e6)
        if rnd == 0:
            grads[v] = [xr.grad.clone()] + [p.grad.clone() for p in gcn.parameters()]
lib.mrp_tuning_set(b"reset", 0)
ref = grads[values[0]]
for v, ts in res.items():
    same = all(torch.equal(a, b) for a, b in zip(grads[v], ref))
    print(f"{knob} {v:2d}: " + " ".join(f"{t:7.1f}" for t in ts) + f"  min {min(ts):7.1f} us/step  "
          f"gradients bit-identical to {knob}={values[0]}: {same}", flush=True)
