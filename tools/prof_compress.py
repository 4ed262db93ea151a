"""Profiling driver (not product code): the split-bf16 compress forward at the configs[3] layer shape
(64 nodes, C=2048, 8x8), N launches, for one rocprofv3 --kernel-trace or --pmc pass.
Usage: python tools/prof_compress.py [launches] [op: fwd|dgrad|wgrad|wgrad3]  (wgrad: the default weight
gradient — at C = 2048 dy split once, split_rows + gemm_nt_psa; wgrad3: both operands split in the
kernel, gemm_nt_split_w4_mf16)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402

n_launch = int(sys.argv[1]) if len(sys.argv) > 1 else 10
op = sys.argv[2] if len(sys.argv) > 2 else "fwd"
dev = torch.device("cuda:0")
torch.manual_seed(0)
n, C, H = 64, 2048, 8
w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
b = torch.randn(C, device=dev)
x, a, gy = (torch.randn(n, C, H, H, device=dev) for _ in range(3))
cm = mrp.compress
if op == "wgrad3":
    assert mrp.load_library().mrp_tuning_set(b"split_nt", 3) == 0
for _ in range(n_launch):
    if op == "fwd":
        cm.compress_forward(w, b, x, a)
    elif op == "dgrad":
        cm.compress_backward_data(w, gy)
    else:
        cm.compress_backward_weight(gy, x, a)
torch.cuda.synchronize()
print("done")
