"""Kernel lab (not product code): the aggregation backward with and without the grad_x base (the DXB
instantiation training runs through FilmCompressFunction) at the BASELINE config shapes, HIP-graph
timed over rotating buffer sets (bench.time_launches); fraction of 8 TB/s on the algorithmic bytes
(bench.alg_bytes_bwd).

usage: python tools/exp_bwd_dxb.py [cfg ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
want = sys.argv[1:] or ["1", "2", "3", "4"]
for cid in want:
    cfg = bench.CONFIGS[int(cid)]
    N, C, H, knn = cfg["N"], cfg["C"], cfg["H"], cfg["knn"]
    B = cfg["per_gpu"]
    g = bench.make_workload(B, N, C, H, H, seed=5, device=dev, knn=knn)
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
    lib = mrp.load_library()
    for base, pre2 in ((False, 1), (True, 1), (True, 2)):
        assert lib.mrp_tuning_set(b"bwd_pre2", pre2) == 0
        launches = [lambda G=G, xi=xi, bs=bs: mrp.aggregate.film_mean_backward(
            G, xi, z, csr, mode, True, True, grad_x_base=bs if base else None) for G, xi, bs in sets]
        t = bench.time_launches(launches, 40, dev)
        byts = bench.alg_bytes_bwd(Nt, E, C, P, base=base)
        res.append(f"{'base' if base else 'no base'} pre2={pre2}: {t * 1e6:7.1f} us {byts / t / 8e12:5.3f}")
    lib.mrp_tuning_set(b"reset", 0)
    print(f"configs[{cid}] N={N} C={C} {H}x{H} B={B}: " + " | ".join(res), flush=True)
    del sets
    torch.cuda.empty_cache()
