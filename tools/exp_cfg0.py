"""Kernel lab (not product code): configs[0] (8 complete 4-robot graphs, C = 64, 32 x 32) no-grad GCN
forward per encoder form (edge_split_v), wall time per call and the encoder path taken."""
import os
import sys
import time
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

dev = torch.device("cuda:0")
g = bench.make_workload(8, 4, 64, 32, 32, seed=77, device=dev)
torch.manual_seed(0)
gcn = mrp.GCN(types.SimpleNamespace(feature_dim=64)).to(dev)
x = g.ndata["image"]
lib = mrp.load_library()
for v in (-1, 0, 1, 2, 3, 4, -1):
    assert lib.mrp_tuning_set(b"edge_split_v", v) == 0
    with torch.no_grad():
        for _ in range(200):
            gcn(g, x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            gcn(g, x)
        torch.cuda.synchronize()
    print(f"edge_split_v {v:2d}: {(time.perf_counter() - t0) / 200 * 1e6:8.1f} us/call  paths {dict(mrp.encoder.PATH_COUNTS)}",
          flush=True)
lib.mrp_tuning_set(b"reset", 0)
