"""Kernel lab (not product code): the encoder's fused training backward (mrp_edge_encoder_bwd_fused) at
forced split counts (knobs enc_s1 / enc_s2) against the planner's, HIP-graph timed, per encoder shape.
usage: python tools/ab_enc_splits.py E C s1,s2 [s1,s2 ...]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import time_launches  # noqa: E402
from mrp_gnn_amd.aggregate import _ptr  # noqa: E402

E, C = int(sys.argv[1]), int(sys.argv[2])
plans = [(0, 0)] + [tuple(int(v) for v in a.split(",")) for a in sys.argv[3:]]
dev = torch.device("cuda:0")
lib = mrp.load_library()
g = torch.Generator().manual_seed(E + C)
dz = torch.randn(E, 2 * C, generator=g).to(dev)
w2 = (torch.randn(2 * C, C, generator=g) / C ** 0.5).to(dev)
w2t = w2.t().contiguous()
hT = torch.randn(C, E, generator=g).to(dev)
pose = (torch.randn(E, 9, generator=g) * 8).to(dev)
outs = [torch.empty(n, device=dev) for n in (C * 9, C, 2 * C * C, 2 * C)]
img = torch.empty((int(lib.mrp_compress_split_pack_bytes(C, 2 * C)) + 3) // 4, device=dev)
mrp._lib.check(lib.mrp_compress_split_pack(_ptr(w2), C, 1, C, 2 * C, _ptr(img), None), "pack")
res = {}
for _ in range(3):
    for s1, s2 in plans:
        assert lib.mrp_tuning_set(b"enc_s1", s1) == 0 and lib.mrp_tuning_set(b"enc_s2", s2) == 0
        ws = torch.empty((int(lib.mrp_edge_encoder_bwd_fused_workspace(E, C)) + 3) // 4, device=dev)

        def call():
            mrp._lib.check(lib.mrp_edge_encoder_bwd_fused(
                _ptr(dz), _ptr(w2t), _ptr(img), _ptr(hT), _ptr(pose), E, C, *(_ptr(o) for o in outs), _ptr(ws),
                ws.numel() * 4, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "bwd_fused")

        res.setdefault((s1, s2), []).append(time_launches([call], 20, dev))
lib.mrp_tuning_set(b"reset", 0)
print(f"E={E} C={C}: " + "  ".join(f"{k}: {min(v) * 1e6:.1f} us" for k, v in res.items()), flush=True)
