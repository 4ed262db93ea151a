#!/usr/bin/env python3
"""Kernel lab (not product code): the one-launch layer from a variant library (tools/bin/<name>.so)
against the product library's two launches at the headline shape, mismatches per run."""
import ctypes
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402
from mrp_gnn_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
B, N, C, H = 32, 8, 512, 32
g = bench.make_workload(B, N, C, H, H, seed=0, device=dev)
torch.manual_seed(0)
gcn = mrp.GCN(types.SimpleNamespace(feature_dim=C)).to(dev)
x = g.ndata["image"]
enc = gcn.edge_encoder.layers
csr = g.csr(dev)
pose = g.edata["pose"]
lib_a = _lib.load_library()
with torch.no_grad():
    mrp.fused.set_fused_forward(False)
    ref = gcn(g, x).clone()
    zref = mrp.encoder.edge_logits(enc, pose).clone()
    mrp.fused.set_fused_forward(True)
for path in sys.argv[1:]:
    lib = lib_a if path == "product" else ctypes.CDLL(os.path.abspath(path))
    if lib is not lib_a:
        _lib._declare(lib)
    _lib._lib = lib
    for lab in (0, 2):
        lib.mrp_tuning_set(b"fused_lab", lab)
        for it in range(3):
            z = zref.clone() if lab else torch.empty_like(zref)
            with torch.no_grad():
                out = mrp.fused.gcn_forward_fused(x, pose, csr, enc[0], enc[2], z_out=z)
            torch.cuda.synchronize()
            d = (out != ref).reshape(B * N, C, H * H)
            nz = d.nonzero()
            print(f"{path} lab{lab} it{it}: mismatches {int(d.sum())} lanes//16 "
                  f"{torch.bincount((nz[:, 2] // 4) % 64 // 16, minlength=4).tolist()} pixel%4 "
                  f"{torch.bincount(nz[:, 2] % 4, minlength=4).tolist()}", flush=True)
        lib.mrp_tuning_set(b"fused_lab", 0)
    _lib._lib = lib_a
