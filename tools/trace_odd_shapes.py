#!/usr/bin/env python3
"""Kernel-name evidence for VERDICT r5 #7: the edge encoder's odd shapes (E or C not a multiple of 32)
run forward + backward, in every backward form, then whole GCN stacks (encoder, aggregation, 1x1
compress) at channel counts and planes no BASELINE config has, with NOTHING else in the process (no
reference evaluation), so that a kernel trace of this script lists only what the product path launches.

    rocprofv3 --kernel-trace --stats -d gpurun_out/odd -o odd -- python tools/trace_odd_shapes.py

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
import types  # noqa: E402

import numpy as np  # noqa: E402
for B, N, C, H, layers, knn in [(3, 5, 48, 7, 2, None), (2, 8, 100, 6, 1, None), (2, 10, 40, 5, 2, 3)]:
    rng = np.random.RandomState(B + N + C)
    g = m.batch([m.frame_graph(np.concatenate([rng.uniform(-10, 10, (N, 3)), rng.standard_normal((N, 4))], 1)
                               .astype(np.float32), knn=knn) for _ in range(B)]).to(dev)
    torch.manual_seed(C)
    net = m.GCNStack(types.SimpleNamespace(feature_dim=C, compress_gcn=True, multi_gcn=False, gcn_layers=layers,
                                           gcn_combine="cat_compress")).to(dev)
    x = torch.randn(g.num_nodes(), C, H, H, device=dev, requires_grad=True)
    net(g, x).square().mean().backward()
    with torch.no_grad():
        net(g, x)
torch.cuda.synchronize()
print("paths", dict(m.encoder.PATH_COUNTS))
assert m.encoder.PATH_COUNTS["autograd"] == 0, "an odd shape left the split kernels"
