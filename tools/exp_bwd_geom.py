"""Kernel lab (not product code): the training aggregation backward (grad_x base added in-kernel,
the DXB instantiation) at the 8x8 BASELINE configs per backward geometry / prefetch knob,
HIP-graph timed over rotating buffer sets; fraction of 8 TB/s on the algorithmic bytes.
usage: python tools/exp_bwd_geom.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

dev = torch.device("cuda:0")
lib = mrp.load_library()
VARIANTS = [("default", {}), ("lo16", {"bwd_fused_lo": 16}), ("pre2", {"bwd_pre2": 1}),
            ("cap8", {"bwd_fused_cap": 8}), ("cap32", {"bwd_fused_cap": 32}), ("lo16cap8", {"bwd_fused_lo": 16, "bwd_fused_cap": 8})]
for cid in (2, 3):
    cfg = bench.CONFIGS[cid]
    N, C, H, B = cfg["N"], cfg["C"], cfg["H"], cfg["per_gpu"]
    g = bench.make_workload(B, N, C, H, H, seed=5, device=dev, knn=cfg["knn"])
    x = g.ndata["image"]
    csr = g.csr(dev)
    Nt, E, P = g.num_nodes(), g.num_edges(), H * H
    gcn = mrp.GCN(type("o", (), {"feature_dim": C})()).to(dev)
    with torch.no_grad():
        z = gcn.edge_encoder.logits(g.edata["pose"])
    mode = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
    plane = Nt * C * P * 4
    nb = bench.rotating_sets(4 * plane + 2 * E * 2 * C * 4)
    sets = [(torch.randn_like(x), torch.randn_like(x), torch.randn_like(x)) for _ in range(nb)]
    res = []
    ref = None
    for name, knobs in VARIANTS + VARIANTS[:1]:
        lib.mrp_tuning_set(b"reset", 0)
        for k, v in knobs.items():
            assert lib.mrp_tuning_set(k.encode(), v) == 0, (k, v)
        G, xi, bs = sets[0]
        o = mrp.aggregate.film_mean_backward(G, xi, z, csr, mode, True, True, grad_x_base=bs)
        if ref is None:
            ref = [t.clone() for t in o]
        same = all(torch.equal(a, b) for a, b in zip(ref, o))
        launches = [lambda G=G, xi=xi, bs=bs: mrp.aggregate.film_mean_backward(G, xi, z, csr, mode, True, True,
                                                                               grad_x_base=bs) for G, xi, bs in sets]
        t = bench.time_launches(launches, 40, dev)
        byts = bench.alg_bytes_bwd(Nt, E, C, P, base=True)
        res.append(f"{name} {t * 1e6:6.1f} us {byts / t / 8e12:5.3f}{'' if same else ' DIFF'}")
    lib.mrp_tuning_set(b"reset", 0)
    print(f"configs[{cid}]: " + " | ".join(res), flush=True)
    del sets
    torch.cuda.empty_cache()
