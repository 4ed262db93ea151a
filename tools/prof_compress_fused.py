"""Profiling driver (not product code): the fused aggregation + compress kernel at the configs[1]
shape, ``iters`` launches with a kernel-lab debug mode (0 = product, 1 = consumers only, 2 = producers
only, 64 = BM 256), for one ``rocprofv3 --pmc`` pass.  Usage: python tools/prof_compress_fused.py mode [iters]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload  # noqa: E402
from mrp_gnn_amd.compress import compress_film_fused  # noqa: E402

mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda:0")
lib = mrp.load_library()
lib.mrp_compress_film_debug.argtypes = [ctypes.c_int]
B, N, C, H = 16, 8, 512, 32
g = make_workload(B, N, C, H, H, seed=1, device=dev)
torch.manual_seed(0)
gcn = mrp.GCN(type("O", (), {"feature_dim": C})()).to(dev)
conv = torch.nn.Conv2d(2 * C, C, 1).to(dev)
with torch.no_grad():
    z = gcn.edge_encoder.logits(g.edata["pose"])
    lib.mrp_compress_film_debug(mode)
    for _ in range(iters):
        compress_film_fused(conv, g.ndata["image"], z, g.csr(dev), mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS)
    torch.cuda.synchronize()
print(f"mode {mode}: {iters} launches", flush=True)
