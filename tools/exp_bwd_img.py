#!/usr/bin/env python3
"""Kernel lab (not product code): the compress backward with dy split once for both GEMMs
(mrp_compress_bwd_img: split_rows_bt -> gemm_nn_img data gradient -> gemm_nt_psa weight gradient)
against the product's two calls (mrp_compress_bwd_data_split + mrp_compress_bwd_weight_split), at the
configs[1..4] layer shapes: bit-identity of gx, ga, dW, db and HIP-graph time of the pair.  Needs
tools/lab_patches/r05_dgrad_bt_image.patch applied to csrc/compress_split.hip (not in the product library).
usage: python tools/exp_bwd_img.py [iters] [rounds]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402
from mrp_gnn_amd import _lib  # noqa: E402
from mrp_gnn_amd.aggregate import _ptr, _stream  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
lib = _lib.load_library()
P_, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
lib.mrp_compress_bwd_img_workspace.argtypes = [I32, I32, I32]
lib.mrp_compress_bwd_img_workspace.restype = I64
lib.mrp_compress_bwd_img.argtypes = [P_, I64, P_, I64, P_, I64, I32, I32, I32, P_, P_, I64, P_, I64, P_, P_, P_, I64,
                                     P_]
lib.mrp_compress_bwd_img.restype = ctypes.c_int
dev = torch.device("cuda:0")
cm = mrp.compress
cm.set_compress_path("split")
SHAPES = [("cfg1", 128, 512, 32), ("cfg2", 256, 1280, 8), ("cfg3", 64, 2048, 8), ("cfg4", 128, 1024, 16)]
for name, n, C, H in SHAPES:
    torch.manual_seed(0)
    P = H * H
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    x, a, gy = (torch.randn(n, C, H, H, device=dev) for _ in range(3))
    nb = int(lib.mrp_compress_bwd_img_workspace(n, C, P))
    if nb == 0:
        print(f"{name}: declined", flush=True)
        continue
    ws = torch.empty((nb + 3) // 4, device=dev)
    img = cm.packed_weight(w, "bwd")
    gx, ga = torch.empty_like(x), torch.empty_like(x)
    dw, db = torch.empty(C, 2 * C, device=dev), torch.empty(C, device=dev)

    def two():
        return cm.compress_backward_data(w, gy) + cm.compress_backward_weight(gy, x, a, True)

    def one():
        _lib.check(lib.mrp_compress_bwd_img(_ptr(gy), C * P, _ptr(x), C * P, _ptr(a), C * P, n, C, P, _ptr(img),
                                            _ptr(gx), C * P, _ptr(ga), C * P, _ptr(dw), _ptr(db), _ptr(ws), nb,
                                            _stream(dev)),
                   "mrp_compress_bwd_img")
        return gx, ga, dw, db

    ref = [t.clone() for t in two()]
    got = [t.clone() for t in one()]
    torch.cuda.synchronize()
    same = [torch.equal(p.reshape(-1), q.reshape(-1)) for p, q in zip(ref, got)]
    diff = [float((p.reshape(-1) - q.reshape(-1)).abs().max()) for p, q in zip(ref, got)]
    res = {"two": [], "one": []}
    for _ in range(rounds):
        res["two"].append(bench.time_launches([two], iters, dev))
        res["one"].append(bench.time_launches([one], iters, dev))
    ta, tb = min(res["two"]), min(res["one"])
    print(f"{name} n={n} C={C} {H}x{H}: two {ta * 1e6:7.1f} us  one {tb * 1e6:7.1f} us ({(tb / ta - 1) * 100:+5.1f} %)"
          f"  same gx/ga/dW/db={same} maxdiff={diff}", flush=True)
