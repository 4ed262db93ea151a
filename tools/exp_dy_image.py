"""Kernel lab (not product code): the compress backward (data gradient + weight gradient, as
FilmCompressFunction runs them) per BASELINE config layer shape in three forms, HIP-graph timed
(bench.time_launches), alternated:
  both-split  the data gradient, then the weight gradient splitting dy and [x; agg] in every workgroup (split_nt 3)
  split-rows  the data gradient, then split_rows (dy split once into its packed image) + gemm_nt_psa (split_nt 4)
  dgrad-img   the data gradient writing dy's image itself, then gemm_nt_psa (the training default)
usage: python tools/exp_dy_image.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import time_launches  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
lib = mrp.load_library()
cm = mrp.compress
cm.set_compress_path("split")
SHAPES = [("cfg1", 128, 512, 32), ("cfg2", 256, 1280, 8), ("cfg3", 64, 2048, 8), ("cfg4", 128, 1024, 16)]
for name, n, C, H in SHAPES:
    torch.manual_seed(0)
    x, a, gy = (torch.randn(n, C, H, H, device=dev) for _ in range(3))
    w = torch.randn(C, 2 * C, 1, 1, device=dev) / (2 * C) ** 0.5
    flop = 2 * 2.0 * C * 2 * C * n * H * H

    def both(nt):
        def f():
            cm.compress_backward_data(w, gy)
            cm.compress_backward_weight(gy, x, a)
        return f

    def img_path():
        img = cm.dy_image(gy)
        cm.compress_backward_data(w, gy, dy_image=img)
        cm.compress_backward_weight(gy, x, a, dy_image=img)

    def dgrad_only():
        cm.compress_backward_data(w, gy)

    res = {}
    for _ in range(2):
        for label, nt, fn in (("both-split", 3, both(3)), ("split-rows", 4, both(4)), ("dgrad-img", -1, img_path),
                              ("dgrad alone", -1, dgrad_only)):
            assert lib.mrp_tuning_set(b"split_nt", nt) == 0
            t = time_launches([fn], iters, dev)
            res.setdefault(label, []).append(t)
    lib.mrp_tuning_set(b"split_nt", -1)
    print(f"{name} n={n} C={C} {H}x{H}: " + " | ".join(
        f"{k} {min(v) * 1e6:7.1f} us" + ("" if k == "dgrad alone" else f" {flop / min(v) / 1e12:5.1f} TF/s")
        for k, v in res.items()), flush=True)
lib.mrp_tuning_set(b"reset", 0)
