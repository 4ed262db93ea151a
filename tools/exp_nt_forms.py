"""Kernel lab (not product code): the split-bf16 weight gradient (compress_backward_weight) per BASELINE
config shape with the 32-k-stage NT kernel (split_nt 1), the pipelined one (split_nt 2) and the
32-k-stage one on 16x16x32 MFMAs (split_nt 3) and that one with dy pre-split once (split_nt 4), HIP-graph
timed (bench.time_launches), plus the edge encoder's two backward products at the headline; dW
outputs compared between the forms (bit-identical at equal splits).
usage: python tools/exp_nt_forms.py [iters] [forms, e.g. 1,2,3]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import time_launches  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
FORMS = tuple(int(v) for v in sys.argv[2].split(",")) if len(sys.argv) > 2 else (3, 4)
dev = torch.device("cuda:0")
lib = mrp.load_library()
cm = mrp.compress
cm.set_compress_path("split")
SHAPES = [("cfg1", 128, 512, 32), ("cfg2", 256, 1280, 8), ("cfg3", 64, 2048, 8), ("cfg4", 128, 1024, 16)]
for name, n, C, H in SHAPES:
    torch.manual_seed(0)
    x, a, gy = (torch.randn(n, C, H, H, device=dev) for _ in range(3))
    flop = 2.0 * C * 2 * C * n * H * H
    res, outs = [], []
    for v in FORMS * 2:
        assert lib.mrp_tuning_set(b"split_nt", v) == 0
        outs.append(cm.compress_backward_weight(gy, x, a))
        t = time_launches([lambda: cm.compress_backward_weight(gy, x, a)], iters, dev)
        res.append(f"nt{v} {t * 1e6:7.1f} us {flop / t / 1e12:6.1f} TF/s")
    diffs = [float((o[0] - outs[0][0]).abs().max() / outs[0][0].abs().max()) for o in outs[1:len(FORMS)]]
    print(f"{name} n={n} C={C} {H}x{H}: " + " | ".join(res) + " | max rel diff vs the first form " +
          ", ".join(f"{d:.2e}" for d in diffs), flush=True)
# the encoder's backward products at the headline (E = 1792, C = 512)
E, C = 1792, 512
torch.manual_seed(1)
enc = mrp.edge_encoder([C, C]).to(dev)
pose = (torch.randn(E, 9) * 8).to(dev)
gz = torch.randn(E, 2 * C, device=dev)
for v in (1, 2, 1, 2):
    assert lib.mrp_tuning_set(b"split_nt", v) == 0
    for _ in range(5):
        enc.zero_grad(set_to_none=True)
        mrp.encoder.edge_logits(enc.layers, pose).backward(gz)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        enc.zero_grad(set_to_none=True)
        mrp.encoder.edge_logits(enc.layers, pose).backward(gz)
    e1.record()
    torch.cuda.synchronize()
    print(f"encoder fwd+bwd E={E} C={C} nt{v}: {e0.elapsed_time(e1) / iters * 1e3:7.1f} us (eager, events)", flush=True)
lib.mrp_tuning_set(b"reset", 0)
