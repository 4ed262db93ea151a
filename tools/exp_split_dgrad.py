"""Accuracy lab (not product code): the split-bf16 data gradient [gx; ga] = W^T gy at the configs[4]
layer shape against float64 — element errors, the error of pixel/node sums (what bias gradients and
Gram sums see), and the packed W^T image decoded back to fp64 (representation error of the split)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as m  # noqa: E402

dev = torch.device("cuda:0")
cm = m.compress
torch.manual_seed(0)
n, C, H = 128, 1024, 16
w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
gy = torch.randn(n, C, H, H, device=dev) * 1e-3
ref = torch.einsum("oc,nohw->nchw", w.reshape(C, 2 * C).double(), gy.double())
for path in ("split", "hip"):
    cm.set_compress_path(path)
    gx, ga = cm.compress_backward_data(w, gy)
    got = torch.cat((gx, ga), 1).double()
    e = float((got - ref).abs().max() / ref.abs().max())
    s_got, s_ref = got.sum((0, 2, 3)), ref.sum((0, 2, 3))
    es = float((s_got - s_ref).abs().max() / s_ref.abs().max())
    print(f"{path}: element err {e:.3e}  channel-sum err {es:.3e}")
f32 = torch.einsum("oc,nohw->nchw", w.reshape(C, 2 * C), gy).double()
print(f"torch fp32: element err {float((f32 - ref).abs().max() / ref.abs().max()):.3e}  channel-sum err "
      f"{float((f32.sum((0, 2, 3)) - ref.sum((0, 2, 3))).abs().max() / ref.sum((0, 2, 3)).abs().max()):.3e}")
# decode the packed images
for kind, M, K, A in (("fwd", C, 2 * C, w.reshape(C, 2 * C)), ("bwd", 2 * C, C, w.reshape(C, 2 * C).t())):
    img = cm.packed_weight(w, kind)
    raw = img.view(torch.int16).cpu().numpy().astype(np.uint16).astype(np.uint32) << 16
    vals = raw.view(np.float32).astype(np.float64).reshape(M // 32, K // 16, 3, 64, 8)
    s = vals.sum(2)  # (mb, ks, lane, j)
    lane = np.arange(64)
    rows = 32 * np.arange(M // 32)[:, None, None, None] + (lane & 31)[None, None, :, None]
    ks = 16 * np.arange(K // 16)[None, :, None, None] + 8 * (lane >> 5)[None, None, :, None] + np.arange(8)[None, None, None, :]
    Ad = A.double().cpu().numpy()
    rec = Ad[np.broadcast_to(rows, s.shape), np.broadcast_to(ks, s.shape)]
    print(f"pack {kind}: max |A - (p0+p1+p2)| / |A| = {np.max(np.abs(rec - s) / np.maximum(np.abs(rec), 1e-30)):.3e}")
cm.set_compress_path("split")
