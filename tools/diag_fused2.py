#!/usr/bin/env python3
"""Kernel lab (not product code): which pixels of the one-launch layer's output differ (lane /
segment pattern), and whether the aggregation side alone (producers idle, no wait, z pre-filled with
the correct logits) reproduces the two launches."""
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

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
with torch.no_grad():
    mrp.fused.set_fused_forward(False)
    ref = gcn(g, x).clone()
    zref = mrp.encoder.edge_logits(enc, pose).clone()
    mrp.fused.set_fused_forward(True)


def run(label, nprod, lab=0, prefill=False, reps=3, detail=False):
    lib.mrp_tuning_set(b"fused_producers", nprod)
    lib.mrp_tuning_set(b"fused_lab", lab)
    for it in range(reps):
        z = zref.clone() if prefill else torch.empty_like(zref)
        with torch.no_grad():
            out = mrp.fused.gcn_forward_fused(x, pose, csr, enc[0], enc[2], z_out=z)
        torch.cuda.synchronize()
        d = (out != ref).reshape(B * N, C, H * H)
        print(f"{label} it{it}: z equal {torch.equal(z, zref)}, mismatching elems {int(d.sum())}", flush=True)
        if detail and it == 0:
            idx = d.nonzero()[:64].tolist()
            rows = {}
            for n_, c_, p_ in idx:
                rows.setdefault((n_, c_), []).append(p_)
            for (n_, c_), ps in list(rows.items())[:8]:
                lanes = sorted({(p // 4) % 64 for p in ps})
                segs = sorted({p // 256 for p in ps})
                vals = [(float(out.reshape(B * N, C, -1)[n_, c_, p]), float(ref.reshape(B * N, C, -1)[n_, c_, p])) for p in ps[:4]]
                print(f"   node {n_} (graph {n_ // N}) ch {c_}: pixels {ps[:12]} lanes {lanes} segs {segs} got/ref {vals}")
            # per destination node-in-graph and per pixel-in-slice
            nz = d.nonzero()
            print("   by node-in-graph", torch.bincount(nz[:, 0] % N, minlength=N).tolist(),
                  " by pixel%4", torch.bincount(nz[:, 2] % 4, minlength=4).tolist(),
                  " by lane-group (lane//16)", torch.bincount((nz[:, 2] // 4) % 64 // 16, minlength=4).tolist(),
                  " by segment", torch.bincount(nz[:, 2] // 256, minlength=4).tolist(),
                  " by channel%4", torch.bincount(nz[:, 1] % 4, minlength=4).tolist())
    lib.mrp_tuning_set(b"fused_producers", 128)
    lib.mrp_tuning_set(b"fused_lab", 0)


import sys as _s
for spec in (_s.argv[1] if len(_s.argv) > 1 else "2,10,18,26,34,6").split(","):
    lab = int(spec)
    run(f"lab{lab}(prefill)", 128, lab=lab, prefill=True, reps=2, detail=(lab == 2))
