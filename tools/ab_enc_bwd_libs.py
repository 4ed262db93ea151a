"""Kernel lab (not product code): the edge encoder's fused training backward (mrp_edge_encoder_bwd_fused,
default form) of the product library (A) against variant libraries (tools/build_variant_lib.py) at the
headline and configs[1..4] encoder shapes, HIP-graph timed, libraries interleaved over rounds, the four
gradients compared bit for bit.  usage: python tools/ab_enc_bwd_libs.py tools/bin/<variant>.so [...]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import time_launches  # noqa: E402
from mrp_gnn_amd import _lib  # noqa: E402
from mrp_gnn_amd.aggregate import _ptr  # noqa: E402

dev = torch.device("cuda:0")
libs = [("A", _lib.load_library())]
for p in sys.argv[1:]:
    lb = ctypes.CDLL(os.path.abspath(p))
    _lib._declare(lb)
    libs.append((os.path.basename(p), lb))
for E, C in ((1792, 512), (896, 512), (1792, 1280), (448, 2048), (512, 1024)):
    g = torch.Generator().manual_seed(E + C)
    dz = torch.randn(E, 2 * C, generator=g).to(dev)
    w2t = (torch.randn(C, 2 * C, generator=g) / C ** 0.5).to(dev)
    hT = torch.randn(C, E, generator=g).to(dev)
    pose = (torch.randn(E, 9, generator=g) * 8).to(dev)
    outs = [torch.empty(n, device=dev) for n in (C * 9, C, 2 * C * C, 2 * C)]
    lib0 = libs[0][1]
    ws = torch.empty((int(lib0.mrp_edge_encoder_bwd_fused_workspace(E, C)) + 3) // 4, device=dev)
    w2 = w2t.t().contiguous()
    img = torch.empty((int(lib0.mrp_compress_split_pack_bytes(C, 2 * C)) + 3) // 4, device=dev)
    _lib.check(lib0.mrp_compress_split_pack(_ptr(w2), C, 1, C, 2 * C, _ptr(img), None), "pack")

    def call(lb):
        _lib.check(lb.mrp_edge_encoder_bwd_fused(
            _ptr(dz), _ptr(w2t), _ptr(img), _ptr(hT), _ptr(pose), E, C, *(_ptr(o) for o in outs), _ptr(ws),
            ws.numel() * 4, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "bwd_fused")

    res, snap = {}, {}
    for _ in range(5):
        for lab, lb in libs:
            res.setdefault(lab, []).append(time_launches([lambda lb=lb: call(lb)], 50, dev))
            if lab not in snap:
                call(lb)
                torch.cuda.synchronize()
                snap[lab] = [o.clone() for o in outs]
    line = [f"E={E} C={C}"]
    for lab, _ in libs:
        same = "" if lab == "A" else (" same" if all(torch.equal(a, b) for a, b in zip(snap[lab], snap["A"])) else " DIFF")
        line.append(f"{lab} {min(res[lab]) * 1e6:6.1f} us{same}")
    print(" | ".join(line), flush=True)
