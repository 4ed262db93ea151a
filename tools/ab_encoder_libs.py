"""Kernel lab (not product code): the one-launch encoder forward of the product library (A) against
variant libraries (tools/build_variant_lib.py) at the headline and configs[1..4] encoder shapes,
HIP-graph timed, libraries interleaved over rounds, logits compared for bit-identity; with --train the
training form (mrp_edge_encoder_fwd_split_train: logits and h^T, both compared).
usage: python tools/ab_encoder_libs.py [--train] tools/bin/<variant>.so [...]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402
from mrp_gnn_amd import _lib  # noqa: E402
from mrp_gnn_amd.aggregate import _ptr  # noqa: E402

dev = torch.device("cuda:0")
args = sys.argv[1:]
train = "--train" in args
args = [a for a in args if a != "--train"]
libs = [("A", _lib.load_library())]
for p in args:
    lb = ctypes.CDLL(os.path.abspath(p))
    _lib._declare(lb)
    libs.append((os.path.basename(p), lb))
for name, E, C in [("head", 1792, 512), ("cfg1", 896, 512), ("cfg2", 1792, 1280), ("cfg3", 448, 2048),
                   ("cfg4", 512, 1024)]:
    torch.manual_seed(0)
    enc = mrp.edge_encoder([C, C]).to(dev)
    pose = (torch.randn(E, 9) * 8).to(dev)
    l1, l2 = enc.layers[0], enc.layers[2]

    img = mrp.encoder.packed_weights(l1, l2)
    z = torch.empty(E, 2 * C, device=dev)
    hT = torch.empty(C, E, device=dev)
    b2 = l2.bias.detach().contiguous()

    def f():
        if not train:
            with torch.no_grad():
                return mrp.encoder.encoder_forward_split(pose, l1, l2)
        lb = _lib._lib
        _lib.check(lb.mrp_edge_encoder_fwd_split_train(
            _ptr(pose), _ptr(img), _ptr(b2), E, C, _ptr(z), _ptr(hT), E,
            ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "fwd_split_train")
        return z, hT
    res, outs = {}, {}
    for _ in range(5):
        for lab, lb in libs:
            _lib._lib = lb
            res.setdefault(lab, []).append(bench.time_launches([f], 20, dev))
            if lab not in outs:
                o = f()
                outs[lab] = torch.cat([t.reshape(-1).clone() for t in (o if isinstance(o, tuple) else (o,))])
    _lib._lib = libs[0][1]
    line = [f"{name} E={E} C={C}"]
    for lab, _ in libs:
        same = "" if lab == "A" else (" same" if torch.equal(outs[lab], outs["A"]) else " DIFF")
        line.append(f"{lab} {min(res[lab]) * 1e6:6.1f} us{same}")
    print(" | ".join(line), flush=True)
