#!/usr/bin/env python3
"""Kernel lab (not product code): the one-launch layer's timeline at the headline shape (fused_lab
bit 64): when each producer item starts and publishes, and each graph's first aggregation workgroup's
wait window, in microseconds from the earliest stamp.
usage: python tools/timeline_fused.py [producers] [extra lab bits]"""
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

nprod = int(sys.argv[1]) if len(sys.argv) > 1 else 128
extra = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dev = torch.device("cuda:0")
B, N, C, H = 32, 8, 512, 32
g = bench.make_workload(B, N, C, H, H, seed=0, device=dev)
torch.manual_seed(0)
gcn = mrp.GCN(types.SimpleNamespace(feature_dim=C)).to(dev)
x = g.ndata["image"]
lib = mrp.load_library()
enc = gcn.edge_encoder.layers
csr = g.csr(dev)
pose = g.edata["pose"]
nb = int(lib.mrp_gcn_fwd_fused_workspace_bytes(B, N, C, H * H))
stream = torch.cuda.current_stream(dev).cuda_stream
nitems = (nb - 256) // 4  # upper bound on items (state words are padded)
ws = mrp.fused._workspace(dev, stream, nb + 256 + 16 * (4096 + 64))
lib.mrp_tuning_set(b"fused_producers", nprod)
with torch.no_grad():
    for _ in range(30):
        mrp.fused.gcn_forward_fused(x, pose, csr, enc[0], enc[2])
    lib.mrp_tuning_set(b"fused_lab", 64 | extra)
    mrp.fused.gcn_forward_fused(x, pose, csr, enc[0], enc[2])
    torch.cuda.synchronize()
    lib.mrp_tuning_set(b"fused_lab", 0)
lib.mrp_tuning_set(b"fused_producers", 128)
items = (B * 2 + 3) // 4 * (2 * C // 32)
tl = ws.view(torch.int64)[nb // 8:].cpu()  # past the zeroed block: err word's 256 B then the stamps
prod = tl[:2 * items].view(items, 2).double()
cons = tl[2 * items:2 * items + 2 * B].view(B, 2).double()
t0 = min(prod[prod > 0].min(), cons[cons > 0].min())
prod = (prod - t0) / 100.0  # 100 MHz -> us
cons = (cons - t0) / 100.0
per_ebg = prod.view(-1, 2 * C // 32, 2)
for e in range(per_ebg.shape[0]):
    s, f = per_ebg[e, :, 0], per_ebg[e, :, 1]
    print(f"items of graphs {2 * e},{2 * e + 1}: start {s.min():6.1f}-{s.max():6.1f} us, published "
          f"{f.min():6.1f}-{f.max():6.1f} us, item time {float((f - s).mean()):5.1f} us")
for b in range(B):
    print(f"graph {b:2d}: first workgroup waits {cons[b, 0]:6.1f} -> {cons[b, 1]:6.1f} us "
          f"({cons[b, 1] - cons[b, 0]:5.1f})")
