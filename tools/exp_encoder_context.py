"""Kernel lab (not product code): the headline encoder kernel (mrp_edge_encoder_fwd_split, E = 1792,
C = 512) timed per launch by the kernel trace (run under rocprofv3 --kernel-trace) in four contexts:
  alone      encoder launches back to back
  after_agg  each after the headline aggregation (the bench step's order)
  after_copy each after a 1 GiB device copy (caches cold, no MFMA load before)
  after_tiny each after a tiny kernel
Each block is tagged by a distinctive fill kernel so the trace can be split.
usage: rocprofv3 --kernel-trace -d out -- python tools/exp_encoder_context.py"""
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

dev = torch.device("cuda:0")
g = bench.make_workload(32, 8, 512, 32, 32, seed=0, device=dev)
x = g.ndata["image"]
torch.manual_seed(0)
gcn = mrp.GCN(types.SimpleNamespace(feature_dim=512)).to(dev)
pose = g.edata["pose"]
csr = g.csr(dev)
mode = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
out = torch.empty_like(x)
big_a = torch.empty(1 << 28, device=dev)
big_b = torch.empty(1 << 28, device=dev)
tiny = torch.empty(64, device=dev)
marker = torch.empty(1 << 10, device=dev, dtype=torch.int64)
with torch.no_grad():
    z = gcn.edge_encoder.logits(pose)
    for _ in range(200):  # clocks up
        gcn(g, x)
    torch.cuda.synchronize()
    for tag, pre in (("alone", None), ("after_agg", lambda: mrp.film_mean_forward_into(x, z, csr, mode, out)),
                     ("after_copy", lambda: big_b.copy_(big_a)), ("after_tiny", lambda: tiny.fill_(1.0))):
        marker.fill_(len(tag))  # FillFunctor<long> marks the block start in the trace
        for _ in range(40):
            if pre is not None:
                pre()
            gcn.edge_encoder.logits(pose)
        torch.cuda.synchronize()
print("done")
