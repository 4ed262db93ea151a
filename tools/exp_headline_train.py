"""Kernel lab (not product code): the headline training step (bench.train_step_time's step: one GCN
layer, B = 32 complete 8-robot graphs, C = 512, 32 x 32, forward + backward) with the encoder's
training path on the split-bf16 kernels with the fused single-stream backward ("fused") or the
two-stream one ("split2s"), and on hidden + fp32-MFMA logits + hipBLASLt ("hip"); wall time per step
and the GPU time of the step's stream (events).
usage: python tools/exp_headline_train.py [steps]"""
import os
import sys
import time
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
g = bench.make_workload(32, 8, 512, 32, 32, seed=1, device=dev)
x = g.ndata["image"]
torch.manual_seed(0)
gcn = mrp.GCN(types.SimpleNamespace(feature_dim=512)).to(dev)
xr = x.detach().clone().requires_grad_(True)
grad = torch.randn_like(x)


def step():
    for p in gcn.parameters():
        p.grad = None
    xr.grad = None
    gcn(g, xr).backward(grad)


for path in ("fused", "split2s", "hip", "fused", "split2s", "hip"):
    mrp.encoder.set_logits_path("hip" if path == "hip" else "split")
    mrp.encoder.set_fused_backward(path == "fused")
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    # host-only cost: the same calls with the GPU already busy would hide it; measure enqueue time
    torch.cuda._sleep(int(2e8))
    t1 = time.perf_counter()
    for _ in range(10):
        step()
    host = (time.perf_counter() - t1) / 10
    torch.cuda.synchronize()
    print(f"{path:8s} wall {wall * 1e3:.3f} ms  events {e0.elapsed_time(e1) / steps:.3f} ms  host enqueue {host * 1e3:.3f} ms",
          flush=True)
mrp.encoder.set_logits_path("split")
mrp.encoder.set_fused_backward(True)
