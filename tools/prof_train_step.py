"""Profiling driver (not product code): a few GCN-stack training steps (forward + backward + every
parameter gradient) and no-grad forwards of every BASELINE config, so one
``rocprofv3 --kernel-trace --stats`` pass shows which kernels a step launches (the compress must be
``gemm_nn``/``gemm_nt``/``split_sum``, no ``Cijk_*``/MIOpen).
Usage: python tools/prof_train_step.py [steps] [config ids, default all] [--no-fwd]"""
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mrp_gnn_amd as mrp  # noqa: E402
from bench import CONFIGS, make_workload  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(args[0]) if args else 5
    ids = [int(c) for c in args[1:]] or list(CONFIGS)
    fwd = "--no-fwd" not in sys.argv
    dev = torch.device("cuda:0")
    for cid in ids:
        cfg = CONFIGS[cid]
        B = cfg["per_gpu"]
        g = make_workload(B, cfg["N"], cfg["C"], cfg["H"], cfg["H"], seed=cid, device=dev, knn=cfg["knn"])
        opt = types.SimpleNamespace(feature_dim=cfg["C"], compress_gcn=True, multi_gcn=False,
                                    gcn_layers=cfg["layers"], gcn_combine="cat_compress")
        torch.manual_seed(0)
        net = mrp.GCNStack(opt).to(dev)
        x = g.ndata["image"].detach().clone().requires_grad_(True)
        gy = torch.randn_like(x)
        for _ in range(steps):
            for p in net.parameters():
                p.grad = None
            x.grad = None
            net(g, x).backward(gy)
        if fwd:
            with torch.no_grad():
                for _ in range(steps):
                    net(g, x)
        torch.cuda.synchronize()
        print(f"configs[{cid}] done", flush=True)
        del g, net, x, gy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
