"""Kernel lab (not product code): launch-geometry sweeps of the aggregation kernels at the BASELINE
config shapes, through the product entry points and ``mrp_tuning_set`` knobs, timed with HIP events
over rotating buffer sets larger than 2x the 256 MB Infinity Cache (bench.py's method).

Usage: python tools/sweep_geometry.py [fwd|bwd|all]
"""
import itertools
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import alg_bytes_bwd, alg_bytes_fwd, make_workload, rotating_sets, time_launches  # noqa: E402

dev = torch.device("cuda:0")
lib = mrp.load_library()
MODE = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
ITERS = int(os.environ.get("ITERS", "40"))

SHAPES = {  # name: (B, N, C, H, knn)
    "north_star": (32, 8, 512, 32, None),
    "cfg1": (16, 8, 512, 32, None),
    "cfg2": (32, 8, 1280, 8, None),
    "cfg3": (8, 8, 2048, 8, None),
    "cfg4": (8, 16, 1024, 16, 4),
}


def knobs(**kw):
    lib.mrp_tuning_set(b"reset", 0)
    for k, v in kw.items():
        code = lib.mrp_tuning_set(k.encode(), int(v))
        if code != 0:
            raise ValueError(f"knob {k}={v} rejected")


def setup(name):
    B, N, C, H, knn = SHAPES[name]
    g = make_workload(B, N, C, H, H, seed=1, device=dev, knn=knn)
    torch.manual_seed(0)
    gcn = mrp.GCN(type("O", (), {"feature_dim": C})()).to(dev)
    with torch.no_grad():
        z = gcn.edge_encoder.logits(g.edata["pose"])
    return g, z, g.csr(dev)


def fwd_time(g, z, csr):
    x = g.ndata["image"]
    Nt, C, H, W = x.shape
    plane = x.numel() * 4
    nf = rotating_sets(2 * plane)
    sets = [(x if i == 0 else torch.randn_like(x), torch.empty_like(x)) for i in range(nf)]
    launches = [lambda a=a, o=o: mrp.film_mean_forward_into(a, z, csr, MODE, o) for a, o in sets]
    t = time_launches(launches, ITERS, dev)
    return t, alg_bytes_fwd(Nt, g.num_edges(), C, H * W) / t / 8e12


def bwd_time(g, z, csr, need_dx=True, need_dgb=True):
    x = g.ndata["image"]
    Nt, C, H, W = x.shape
    plane = x.numel() * 4
    nb = rotating_sets(3 * plane)
    sets = [(torch.randn_like(x), x if i == 0 else torch.randn_like(x)) for i in range(nb)]
    launches = [lambda G=G, a=a: mrp.aggregate.film_mean_backward(G, a, z, csr, MODE, need_dx, need_dgb)
                for G, a in sets]
    t = time_launches(launches, ITERS, dev)
    return t, alg_bytes_bwd(Nt, g.num_edges(), C, H * W) / t / 8e12


def sweep(label, name, fn, grid):
    g, z, csr = setup(name)
    keys = list(grid)
    res = []
    for vals in itertools.product(*(grid[k] for k in keys)):
        kw = dict(zip(keys, vals))
        try:
            knobs(**kw)
            t, frac = fn(g, z, csr)
        except (ValueError, RuntimeError) as e:
            print(f"{label} {name} {kw}: {e}", flush=True)
            continue
        res.append((t, kw, frac))
        print(f"{label} {name:10s} {kw}  {t * 1e6:8.1f} us  {frac * 100:5.1f} %", flush=True)
    res.sort(key=lambda r: r[0])
    print(f"BEST {label} {name}: {res[0][1]} {res[0][0] * 1e6:.1f} us {res[0][2] * 100:.1f} %", flush=True)
    knobs()
    del g, z, csr
    torch.cuda.empty_cache()


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    # warm the clocks
    g, z, csr = setup("cfg2")
    out = torch.empty_like(g.ndata["image"])
    for _ in range(2000):
        mrp.film_mean_forward_into(g.ndata["image"], z, csr, MODE, out)
    torch.cuda.synchronize()
    del g, z, csr, out
    if what == "vec2":  # 8-byte slices on small planes (fewer registers, more waves)
        for name in ("cfg2", "cfg3", "cfg4", "cfg1"):
            sweep("fwd", name, fwd_time, {"fwd_vec2_below": [0, 1 << 20], "fwd_lo": [16, 32]})
        return
    if what == "fwdall":  # the forward at every config shape, default geometry
        for name in ("north_star", "cfg1", "cfg2", "cfg3", "cfg4"):
            sweep("fwd", name, fwd_time, {"fwd_cap": [16]})
        return
    if what == "cfg4fwd":  # repeated k-NN forward timings (A/B between library builds)
        for _ in range(3):
            sweep("fwd", "cfg4", fwd_time, {"fwd_regular_split": [0]})
        return
    if what == "cfg4":  # repeated k-NN forward and backward timings
        for _ in range(3):
            sweep("fwd", "cfg4", fwd_time, {"fwd_regular_split": [0]})
            sweep("bwd", "cfg4", bwd_time, {"bwd_regular_vec": [2]})
        return
    if what == "cfg4bwd":  # k-NN backward: matrix-core kernel against the VALU kernel
        for _ in range(2):
            sweep("bwd", "cfg4", bwd_time, {"bwd_regular_mfma": [0, 1], "bwd_mfma_cpw": [1, 2, 4]})
        for dx, dgb in ((True, False), (False, True)):
            sweep(f"bwd dx={int(dx)} dgb={int(dgb)}", "cfg4",
                  lambda g, z, csr, dx=dx, dgb=dgb: bwd_time(g, z, csr, dx, dgb), {"bwd_regular_mfma": [0, 1]})
        return
    if what == "mfmabwd":  # complete graphs: matrix-core backward against film_bwd_fused
        for name in ("cfg3", "cfg2", "cfg1"):
            sweep("bwd", name, bwd_time, {"bwd_complete_mfma": [0]})
            sweep("bwd", name, bwd_time, {"bwd_complete_mfma": [1], "bwd_mfma_cpw": [1, 2]})
        sweep("bwd", "cfg4", bwd_time, {"bwd_regular_mfma": [1], "bwd_mfma_cpw": [1, 2]})
        return
    # "gramparts" (removed with its kernel hooks): film_bwd_fused at configs[3] with the lane reduction,
    # the d gamma/beta stores or the Gram FMAs skipped: 25.2 us -> 23.3 / 23.2 / 23.1, all three 21.0
    if what == "bigbwd1":  # 32x32 backward with one slice per lane (a plane over 4 waves)
        for name in ("cfg1", "north_star"):
            sweep("bwd", name, bwd_time, {"bwd_fused_lo": [128, 256], "bwd_fused_hi": [256], "bwd_fused_cap": [1]})
        return
    if what == "bigbwd":  # 32x32-plane backward geometry (headline / configs[1])
        for name in ("cfg1",):
            sweep("bwd", name, bwd_time, {"bwd_fused_lo": [32, 64, 128], "bwd_fused_hi": [64, 128, 256],
                                          "bwd_fused_cap": [1, 2, 4], "bwd_pre2": [0, 1]})
        return
    if what == "smallcap":  # 8x8-plane backward: channels per workgroup
        for name in ("cfg3", "cfg2"):
            sweep("bwd", name, bwd_time, {"bwd_fused_cap": [8, 16, 32, 64], "bwd_pre2": [0, 1]})
        return
    if what == "smallbwd":  # 8x8-plane backward geometry (configs[2] / [3])
        for name in ("cfg3", "cfg2"):
            sweep("bwd", name, bwd_time, {"bwd_fused_lo": [4, 8, 16], "bwd_fused_hi": [8, 16],
                                          "bwd_fused_cap": [2, 4, 8, 16], "bwd_pre2": [0, 1]})
        return
    if what == "cfg4fwdgeo":  # k-NN forward geometry after the compile-time-degree specialisation
        sweep("fwd", "cfg4", fwd_time, {"fwd_regular_split": [0, 1], "fwd_regular_lo": [16, 32, 64],
                                        "fwd_regular_hi": [32, 64], "fwd_regular_cap": [4, 8, 16]})
        return
    if what == "bwdparts":  # the backward's two halves alone: grad_x only, d gamma/beta only
        for name in ("cfg4", "cfg1", "cfg3"):
            for dx, dgb in ((True, True), (True, False), (False, True)):
                sweep(f"bwd dx={int(dx)} dgb={int(dgb)}", name,
                      lambda g, z, csr, dx=dx, dgb=dgb: bwd_time(g, z, csr, dx, dgb), {"bwd_regular_vec": [2]})
        return
    if what == "pre2":  # backward with / without the two-slice prefetch
        for name in ("north_star", "cfg1", "cfg2", "cfg3"):
            sweep("bwd", name, bwd_time, {"bwd_pre2": [0, 1, 0, 1]})
        return
    if what == "bwdall":  # the backward at every config shape, default geometry
        for name in ("north_star", "cfg1", "cfg2", "cfg3"):
            sweep("bwd", name, bwd_time, {"bwd_fused_cap": [8]})
        sweep("bwd", "cfg4", bwd_time, {"bwd_regular_vec": [2]})
        return
    if what == "capfwd":  # small workgroups (round 2: a 1-float4-per-thread copy streams at 82 %)
        for name in ("north_star", "cfg2", "cfg3"):
            sweep("fwd", name, fwd_time, {"fwd_cap": [1, 2, 4, 8, 16]})
        sweep("fwd", "north_star", fwd_time, {"fwd_lo": [16, 32], "fwd_hi": [16, 32, 64], "fwd_cap": [1, 2, 4]})
        sweep("bwd", "cfg2", bwd_time, {"bwd_fused_cap": [1, 2, 4, 8]})
        sweep("bwd", "cfg3", bwd_time, {"bwd_fused_cap": [1, 2, 4, 8]})
        return
    if what == "regbwd":
        sweep("bwd", "cfg4", bwd_time, {"bwd_regular_vec": [1, 2], "bwd_regular_lanes": [8, 16, 32]})
        for name in ("cfg2", "cfg3", "cfg1"):
            sweep("bwd", name, bwd_time, {"bwd_fused_cap": [8]})
            sweep("fwd", name, fwd_time, {"fwd_cap": [16]})
        sweep("fwd", "cfg4", fwd_time, {"fwd_regular_split": [0, 1]})
    if what in ("fwd", "all"):
        for name in ("cfg2", "cfg3"):
            sweep("fwd", name, fwd_time, {"fwd_lo": [4, 8, 16], "fwd_hi": [4, 8, 16], "fwd_cap": [4, 8, 16]})
        sweep("fwd", "north_star", fwd_time, {"fwd_lo": [16, 32, 64], "fwd_hi": [32, 64, 128, 256], "fwd_cap": [8, 16]})
        sweep("fwd", "cfg4", fwd_time, {"fwd_regular_split": [0, 1], "fwd_regular_lo": [8, 16, 32, 64],
                                        "fwd_regular_hi": [16, 32, 64], "fwd_regular_cap": [4, 8, 16]})
    if what in ("bwd", "all"):
        for name in ("cfg2", "cfg3"):
            sweep("bwd", name, bwd_time, {"bwd_fused_lo": [4, 8, 16], "bwd_fused_hi": [4, 8, 16],
                                          "bwd_fused_cap": [8, 16, 32, 64]})
        sweep("bwd", "cfg1", bwd_time, {"bwd_fused_lo": [32, 64], "bwd_fused_hi": [64, 128, 256],
                                        "bwd_fused_cap": [2, 4, 8]})
        sweep("bwd", "cfg4", bwd_time, {"bwd_regular_vec": [1, 2], "bwd_regular_lanes": [8, 16, 32]})


if __name__ == "__main__":
    main()
