"""Kernel lab (not product code): the backward of COMPLETE graphs of more than 8 nodes — film_bwd_dx +
the Gram pass (default) against the matrix-core film_bwd_mfma (mrp_tuning_set bwd_complete_mfma 1) —
to decide whether the matrix-core kernel earns a default for complete graphs anywhere.
HIP-graph timed over rotating buffers (bench.time_launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import make_workload, rotating_sets, time_launches  # noqa: E402

dev = torch.device("cuda:0")
lib = mrp.load_library()
MODE = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
for B, N, C, H in ((8, 16, 1024, 16), (32, 12, 512, 8), (8, 8, 2048, 8)):
    g = make_workload(B, N, C, H, H, seed=3, device=dev)
    x = g.ndata["image"]
    csr = g.csr(dev)
    torch.manual_seed(0)
    enc = mrp.edge_encoder([C, C]).to(dev)
    with torch.no_grad():
        z = enc.logits(g.edata["pose"])
    nb = rotating_sets(3 * x.numel() * 4)
    sets = [(torch.randn_like(x), x if i == 0 else torch.randn_like(x)) for i in range(nb)]
    res = {}
    for knob in (0, 1):
        assert lib.mrp_tuning_set(b"bwd_complete_mfma", knob) == 0
        launches = [lambda G=G, xi=xi: mrp.aggregate.film_mean_backward(G, xi, z, csr, MODE, True, True) for G, xi in sets]
        res[knob] = time_launches(launches, 30, dev)
        out = mrp.aggregate.film_mean_backward(sets[0][0], sets[0][1], z, csr, MODE, True, True)
        res[f"out{knob}"] = [t.clone() for t in out]
    lib.mrp_tuning_set(b"reset", 0)
    d = max(float((a - b).abs().max() / b.abs().max()) for a, b in zip(res["out0"], res["out1"]))
    print(f"complete B={B} N={N} C={C} {H}x{H}: VALU {res[0] * 1e6:7.1f} us | matrix-core {res[1] * 1e6:7.1f} us "
          f"| max rel diff {d:.1e}", flush=True)
    del sets, x, g
    torch.cuda.empty_cache()
