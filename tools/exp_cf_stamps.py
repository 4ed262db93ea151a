"""Kernel lab (not product code): s_memtime stamps around the first 16 barriers of workgroup 0 of the
fused aggregation + compress kernel at the configs[1] shape, per wave, in the product mode and the
producers-only / consumers-only lab modes.  Prints, per role, the median work time between barriers
and the median wait inside them (shader cycles)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload  # noqa: E402
from mrp_gnn_amd.compress import compress_film_fused  # noqa: E402

dev = torch.device("cuda:0")
lib = mrp.load_library()
lib.mrp_compress_film_debug.argtypes = [ctypes.c_int]
lib.mrp_compress_film_debug_stamps.argtypes = [ctypes.c_void_p]
shape = sys.argv[1] if len(sys.argv) > 1 else "cfg1"
B, N, C, H = {"cfg1": (16, 8, 512, 32), "cfg3": (8, 8, 2048, 8)}[shape]
g = make_workload(B, N, C, H, H, seed=1, device=dev)
torch.manual_seed(0)
gcn = mrp.GCN(type("O", (), {"feature_dim": C})()).to(dev)
conv = torch.nn.Conv2d(2 * C, C, 1).to(dev)
MODE = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
st = torch.zeros(16 * 32 + 16 * 64, dtype=torch.int64, device=dev)
with torch.no_grad():
    z = gcn.edge_encoder.logits(g.edata["pose"])
    x, csr = g.ndata["image"], g.csr(dev)
    for mode in (0, 2, 1, 64):  # product (BM 128), producers only, consumers only, BM 256
        lib.mrp_compress_film_debug(mode)
        lib.mrp_compress_film_debug_stamps(None)
        for _ in range(30):  # clocks up
            compress_film_fused(conv, x, z, csr, MODE)
        st.zero_()
        lib.mrp_compress_film_debug_stamps(ctypes.c_void_p(st.data_ptr()))
        compress_film_fused(conv, x, z, csr, MODE)
        torch.cuda.synchronize()
        lib.mrp_compress_film_debug_stamps(None)
        raw = st.cpu().numpy()
        a = raw[:16 * 32].reshape(16, 16, 2)  # wave, barrier, (before, after)
        q = raw[16 * 32:].reshape(16, 16, 4)  # wave, barrier index at produce time, (operands stored, aggregate stored)
        nw = int((a[:, 0, 0] != 0).sum())
        nc = nw - 4
        t0 = a[:nw, 0, 1].min()
        rows = []
        for role, ws in (("consumer", range(nc)), ("producer", range(nc, nw))):
            wait = np.median([a[w, k, 1] - a[w, k, 0] for w in ws for k in range(2, 15)])
            work = np.median([a[w, k + 1, 0] - a[w, k, 1] for w in ws for k in range(2, 14)])
            rows.append(f"{role}: work {work:7.0f} wait {wait:7.0f}")
        stage = np.median(np.diff(a[0, 2:15, 1]))
        if mode != 1:
            ws = range(nc, nw)
            st_ops = np.median([q[w, k, 0] - a[w, k - 1, 1] for w in ws for k in range(3, 14)])
            agg = np.median([q[w, k, 1] - q[w, k, 0] for w in ws for k in range(3, 14)])
            rest = np.median([a[w, k, 0] - q[w, k, 1] for w in ws for k in range(3, 14)])
            rows.append(f"producer split: barrier->operands stored {st_ops:6.0f}, aggregate {agg:6.0f}, loads issue {rest:6.0f}")
        print(f"{shape} mode {mode:3d} ({nw} waves): stage {stage:7.0f} cyc | " + " | ".join(rows), flush=True)
    lib.mrp_compress_film_debug(0)
