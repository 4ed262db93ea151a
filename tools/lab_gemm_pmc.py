"""Kernel lab (not product code): a short fixed workload for rocprofv3 --pmc passes over the compress
GEMM kernels and the library GEMM of the same product (configs[3] per-GPU shape by default).
usage: python tools/lab_gemm_pmc.py [cfg] [variant]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from mrp_gnn_amd import compress as cp  # noqa: E402

SHAPES = {"cfg1": (128, 512, 32), "cfg2": (256, 1280, 8), "cfg3": (64, 2048, 8), "cfg4": (128, 1024, 16)}
name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dev = torch.device("cuda:0")
lib = mrp.load_library()
if name == "enc":  # the headline's edge encoder: fused kernel (edge_fused = variant) and addmm
    from mrp_gnn_amd import encoder as enc
    E, C = 1792, 512
    layers = mrp.edge_encoder([C, C]).to(dev).layers
    pose = torch.randn(E, 9, device=dev)
    h = torch.relu(torch.randn(E, C, device=dev))
    p = [t.detach() for t in (pose, layers[0].weight, layers[0].bias, layers[2].weight, layers[2].bias)]
    lib.mrp_tuning_set(b"edge_fused", variant)
    for _ in range(30):
        enc.encoder_forward_fused(*p)
    torch.cuda.synchronize()
    for _ in range(5):
        enc.encoder_forward_fused(*p)
        torch.addmm(p[4], h, p[3].t())
    torch.cuda.synchronize()
    print("done")
    sys.exit(0)
n, C, H = SHAPES[name]
lib.mrp_tuning_set(b"gemm_nn", variant)
x = torch.randn(n, C, H, H, device=dev)
a = torch.randn_like(x)
gy = torch.randn_like(x)
w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
w2 = w.reshape(C, 2 * C)
cat = torch.cat((x, a), 1)
for _ in range(30):  # clock ramp
    cp.compress_forward(w, None, x, a)
torch.cuda.synchronize()
for _ in range(5):
    cp.compress_forward(w, None, x, a)
    torch.bmm(w2.expand(n, C, 2 * C), cat.view(n, 2 * C, H * H))
    cp.compress_backward_data(w, gy)
    torch.bmm(w2.t().expand(n, 2 * C, C), gy.view(n, C, H * H))
torch.cuda.synchronize()
print("done")
