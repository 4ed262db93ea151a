"""Kernel lab (not product code): the edge encoder's second Linear z = h W2^T + b2 — the matrix-core
kernel mrp_edge_logits_fwd (mrp_tuning_set "edge_gemm" 0 / 1) against torch.addmm (hipBLASLt) —
the one-launch encoder mrp_edge_encoder_fwd ("edge_fused" 0..4), its split-bf16 form
mrp_edge_encoder_fwd_split, and the whole encoder forward per
path (library / hidden + logits kernels / fused), HIP-graph timed (bench.time_launches), at
the headline size (B = 32 complete graphs of 8: E = 1792, C = 512) and the BASELINE configs.

usage: python tools/exp_encoder.py [--iters N]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import time_launches  # noqa: E402
from mrp_gnn_amd import encoder as enc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=50)
args = ap.parse_args()
dev = torch.device("cuda:0")
lib = mrp.load_library()
# (E, C): headline, configs[1..4] per GPU (complete graphs: E = B n (n - 1); k-NN: B n k)
SHAPES = [("head", 1792, 512), ("cfg1", 1792 * 2, 512), ("cfg2", 256 * 3, 1280), ("cfg3", 64 * 7, 2048),
          ("cfg4", 128 * 4, 1024)]
for name, E, C in SHAPES:
    torch.manual_seed(0)
    layers = mrp.edge_encoder([C, C]).to(dev).layers
    pose = torch.randn(E, 9, device=dev)
    h = torch.relu(torch.randn(E, C, device=dev))
    w2, b2 = layers[2].weight.detach(), layers[2].bias.detach()
    flop = 2.0 * E * C * 2 * C
    ref = torch.addmm(b2, h, w2.t())
    row = [f"{name} E={E} C={C}"]
    with torch.no_grad():
        enc.set_logits_path("library")
        t = time_launches([lambda: enc.logits_forward(h, w2, b2)], args.iters, dev)
        row.append(f"addmm {t * 1e6:6.1f} us {flop / t / 1e12:5.1f} TF/s")
        enc.set_logits_path("hip")
        for v in (0, 1):
            lib.mrp_tuning_set(b"edge_gemm", v)
            z = enc.logits_forward(h, w2, b2)
            err = float((z - ref).abs().max() / ref.abs().max())
            t = time_launches([lambda: enc.logits_forward(h, w2, b2)], args.iters, dev)
            row.append(f"v{v} {t * 1e6:6.1f} us {flop / t / 1e12:5.1f} TF/s (err {err:.1e})")
        lib.mrp_tuning_set(b"reset", 0)
        l1 = layers[0]
        ref_full = enc.logits_forward(enc.hidden_forward(pose, l1.weight, l1.bias), w2, b2)
        for v in range(5):
            lib.mrp_tuning_set(b"edge_fused", v)
            args_f = (pose, l1.weight, l1.bias, w2, b2)
            z = enc.encoder_forward_fused(*args_f)
            if z is None:
                row.append(f"fused{v} declined")
                continue
            same = bool(torch.equal(z, ref_full))
            t = time_launches([lambda: enc.encoder_forward_fused(*args_f)], args.iters, dev)
            row.append(f"fused{v} {t * 1e6:6.1f} us{'' if same else ' MISMATCH'}")
        lib.mrp_tuning_set(b"reset", 0)
        for cb, ks in ((1, 1), (2, 1), (1, 2), (2, 2)):
            lib.mrp_tuning_set(b"edge_split_cb", cb)
            lib.mrp_tuning_set(b"edge_split_k", ks)
            zs = enc.encoder_forward_split(pose, l1, layers[2])
            err = float((zs - ref_full).abs().max() / ref_full.abs().max())
            t = time_launches([lambda: enc.encoder_forward_split(pose, l1, layers[2])], args.iters, dev)
            row.append(f"split cb{cb} k{ks} {t * 1e6:6.1f} us (vs fused {err:.1e})")
        lib.mrp_tuning_set(b"reset", 0)
        for path in ("library", "hip", "fused", "split"):
            enc.set_logits_path(path)
            t = time_launches([lambda: enc.edge_logits(layers, pose)], args.iters, dev)
            row.append(f"encoder[{path}] {t * 1e6:6.1f} us")
    print(" | ".join(row), flush=True)
