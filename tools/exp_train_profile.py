"""Run GCN forward+backward steps at the north-star size for a kernel-trace profile. Not product code."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload  # noqa: E402

dev = torch.device("cuda:0")
g = make_workload(32, 8, 512, 32, 32, seed=0, device=dev)
x = g.ndata["image"].requires_grad_(True)
gcn = mrp.GCN(type("O", (), {"feature_dim": 512})()).to(dev)
G = torch.randn_like(x)
for _ in range(20):
    for p in gcn.parameters():
        p.grad = None
    x.grad = None
    gcn(g, x).backward(G)
torch.cuda.synchronize()
print("done")
