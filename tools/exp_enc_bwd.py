"""Kernel lab (not product code): the edge encoder's fused training backward alone
(``mrp_edge_encoder_bwd_fused``: prep, dual split-K product, reduce, final) at the BASELINE encoder
shapes, HIP-graph timed (bench.time_launches) on fixed inputs, with the gradients' checksum so two
builds can be compared; with W2^T's packed image (the default since round 5: the dh^T product reads it
by LDS-DMA) against the in-kernel split of W2^T (knob enc_bwd_psa 0), alternated, and their
gradients compared bit for bit (and dz^T written as an image too, enc_bwd_psa 2).  usage: python tools/exp_enc_bwd.py [iters]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import time_launches  # noqa: E402
from mrp_gnn_amd.aggregate import _ptr  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda:0")
lib = mrp.load_library()
for E, C in ((1792, 512), (896, 512), (1792, 1280), (448, 2048), (512, 1024)):
    g = torch.Generator().manual_seed(E + C)
    dz = torch.randn(E, 2 * C, generator=g).to(dev)
    w2t = (torch.randn(C, 2 * C, generator=g) / C ** 0.5).to(dev)
    hT = torch.randn(C, E, generator=g).to(dev)
    pose = (torch.randn(E, 9, generator=g) * 8).to(dev)
    outs = [torch.empty(n, device=dev) for n in (C * 9, C, 2 * C * C, 2 * C)]
    ws = torch.empty((int(lib.mrp_edge_encoder_bwd_fused_workspace(E, C)) + 3) // 4, device=dev)

    w2 = w2t.t().contiguous()
    img = torch.empty((int(lib.mrp_compress_split_pack_bytes(C, 2 * C)) + 3) // 4, device=dev)
    mrp._lib.check(lib.mrp_compress_split_pack(_ptr(w2), C, 1, C, 2 * C, _ptr(img), None), "pack")

    def call():
        mrp._lib.check(lib.mrp_edge_encoder_bwd_fused(
            _ptr(dz), _ptr(w2t), _ptr(img), _ptr(hT), _ptr(pose), E, C, *(_ptr(o) for o in outs), _ptr(ws), ws.numel() * 4,
            ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "mrp_edge_encoder_bwd_fused")

    call()
    torch.cuda.synchronize()
    ref = [o.double() for o in outs]
    # float64 reference of the four gradients
    d = dz.double()
    dh = (d @ w2t.double().t()).t() * (hT > 0).double()  # (C, E): W2^T dz masked by the ReLU
    r64 = [(dh @ pose.double()).reshape(-1), dh.sum(1), (d.t() @ hT.double().t()).reshape(-1), d.sum(0)]
    err = max(float((a - b).abs().max() / b.abs().max()) for a, b in zip(ref, r64))
    res = {0: [], 1: [], 2: []}
    snap = {}
    for _ in range(3):
        for v in (2, 1, 0):
            assert lib.mrp_tuning_set(b"enc_bwd_psa", v) == 0
            res[v].append(time_launches([call], iters, dev))
            call()
            torch.cuda.synchronize()
            snap[v] = [o.clone() for o in outs]
    lib.mrp_tuning_set(b"reset", 0)
    same = all(torch.equal(a, b) for a, b in zip(snap[0][:3], snap[2][:3]))
    print(f"E={E} C={C}: both images {min(res[2]) * 1e6:6.1f} us, W2^T image {min(res[1]) * 1e6:6.1f} us, "
          f"in-kernel split {min(res[0]) * 1e6:6.1f} us ({(min(res[2]) / min(res[0]) - 1) * 100:+5.1f} %), "
          f"dW1/db1/dW2 bit-identical {same}, max rel err vs float64 {err:.1e}", flush=True)
