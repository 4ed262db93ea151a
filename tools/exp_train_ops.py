"""torch.profiler op table of the layer's training step at the north-star size (which aten ops and
copies run besides the HIP kernels).  Not product code."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload  # noqa: E402

dev = torch.device("cuda:0")
g = make_workload(32, 8, 512, 32, 32, seed=0, device=dev)
x = g.ndata["image"].detach().clone().requires_grad_(True)
gcn = mrp.GCN(type("O", (), {"feature_dim": 512})()).to(dev)
G = torch.randn_like(x)


def step():
    for p in gcn.parameters():
        p.grad = None
    x.grad = None
    gcn(g, x).backward(G)


for _ in range(5):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    for _ in range(5):
        step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=40, max_name_column_width=60))
