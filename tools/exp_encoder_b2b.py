"""Kernel lab (not product code): the one-launch encoder at the headline shape back to back and after a
tiny elementwise kernel, HIP-graph timed (run under rocprofv3 --kernel-trace for per-launch durations)."""
import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import bench, mrp_gnn_amd as mrp
dev = torch.device("cuda:0")
torch.manual_seed(0)
E, C = 1792, 512
enc = mrp.edge_encoder([C, C]).to(dev); pose = (torch.randn(E, 9) * 8).to(dev)
l1, l2 = enc.layers[0], enc.layers[2]
tiny = torch.zeros(64, device=dev)
def f():
    with torch.no_grad():
        return mrp.encoder.encoder_forward_split(pose, l1, l2)
def g():
    tiny.add_(1.0)
    return f()
for lab, fn in (("b2b", f), ("tiny", g), ("b2b2", f)):
    t = bench.time_launches([fn], 40, dev)
    print(lab, round(t * 1e6, 2), flush=True)
