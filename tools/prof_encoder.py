"""Profiling driver (not product code): the split-bf16 edge encoder forward at the headline shape
(E = 1792, C = 512), N launches, for one rocprofv3 --kernel-trace or --pmc pass.
Usage: python tools/prof_encoder.py [launches] [edge_split_v (-1: the per-shape default)]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
v = int(sys.argv[2]) if len(sys.argv) > 2 else -1
dev = torch.device("cuda:0")
torch.manual_seed(0)
layers = mrp.edge_encoder([512, 512]).to(dev).layers
pose = torch.randn(1792, 9, device=dev)
mrp.load_library().mrp_tuning_set(b"edge_split_v", v)
with torch.no_grad():
    for _ in range(n):
        mrp.encoder.encoder_forward_split(pose, layers[0], layers[2])
torch.cuda.synchronize()
print("done")
