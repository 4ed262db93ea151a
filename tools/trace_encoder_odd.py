#!/usr/bin/env python3
"""Kernel-name evidence for VERDICT r5 #7: the edge encoder's odd shapes (E or C not a multiple of 32)
run forward + backward, in every backward form, with NOTHING else in the process (no reference
evaluation), so that a kernel trace of this script lists only what the product path launches.

    rocprofv3 --kernel-trace --stats -d gpurun_out/odd -o odd -- python tools/trace_encoder_odd.py

then no ``Cijk_*`` (hipBLASLt / rocBLAS GEMM) name may appear in the stats (profiles/r06_encoder_odd_*)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as m  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = [(1, 1), (7, 3), (100, 130), (33, 1281), (1000, 48), (1792, 500), (1793, 512)]
for E, C in SHAPES:
    torch.manual_seed(E + C)
    enc = m.edge_encoder([C, C]).to(dev)
    for form in ("fused", "two_stream", "pose_grad"):
        m.encoder.set_fused_backward(form != "two_stream")
        pose = (torch.randn(E, 9, device=dev) * 8).requires_grad_(form == "pose_grad")
        z = m.encoder.edge_logits(enc.layers, pose)
        z.backward(torch.ones_like(z))
    with torch.no_grad():
        m.encoder.edge_logits(enc.layers, pose)
m.encoder.set_fused_backward(True)
torch.cuda.synchronize()
print("paths", dict(m.encoder.PATH_COUNTS))
assert m.encoder.PATH_COUNTS["autograd"] == 0, "an odd shape left the split kernels"
