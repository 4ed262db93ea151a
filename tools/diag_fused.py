#!/usr/bin/env python3
"""Kernel lab (not product code): where the one-launch layer differs from the two launches at the
headline shape — mismatching elements per graph and iteration, by producer count and workspace
handling (launcher memset vs torch zero_; fresh vs reused workspace)."""
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


def run(label, nprod, lab=0, fresh=False, reps=5):
    lib.mrp_tuning_set(b"fused_producers", nprod)
    lib.mrp_tuning_set(b"fused_lab", lab)
    for it in range(reps):
        if fresh:
            mrp.fused._workspaces.clear()
        if lab & 1:
            stream = torch.cuda.current_stream(dev).cuda_stream
            nb = int(lib.mrp_gcn_fwd_fused_workspace_bytes(B, N, C, H * H))
            mrp.fused._workspace(dev, stream, nb).zero_()
        z = torch.empty_like(zref)
        with torch.no_grad():
            out = mrp.fused.gcn_forward_fused(x, pose, csr, enc[0], enc[2], z_out=z)
        err = mrp.fused.error_word(dev)
        d = (out != ref).reshape(B, N, C, -1)
        per_graph = d.any(-1).sum((1, 2)).tolist()
        per_ch = d.any(-1).any(1).any(0).nonzero().flatten().tolist()
        print(f"{label} it{it}: z equal {torch.equal(z, zref)}, err {err}, mismatching elems {int(d.sum())}, "
              f"(node,channel) pairs per graph {per_graph}, first channels {per_ch[:16]}", flush=True)
    lib.mrp_tuning_set(b"fused_producers", 128)
    lib.mrp_tuning_set(b"fused_lab", 0)


run("p128", 128)
run("p512", 512)
run("p128-fresh", 128, fresh=True)
run("p128-torchzero", 128, lab=1)
run("p0", 0, reps=2)
run("p1", 1, reps=2)
