"""Kernel lab (not product code): the one-launch encoder forward with 4- vs 8-wave workgroups (knob
edge_split_v 1 / 3) at the headline and configs[1..4] encoder shapes, HIP-graph timed."""
import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import bench, mrp_gnn_amd as mrp
dev = torch.device("cuda:0"); lib = mrp.load_library()
for name, E, C in [("head", 1792, 512), ("cfg1", 896, 512), ("cfg2", 1792, 1280), ("cfg3", 448, 2048), ("cfg4", 512, 1024)]:
    torch.manual_seed(0)
    enc = mrp.edge_encoder([C, C]).to(dev); pose = (torch.randn(E, 9) * 8).to(dev)
    l1, l2 = enc.layers[0], enc.layers[2]
    def f():
        with torch.no_grad():
            return mrp.encoder.encoder_forward_split(pose, l1, l2)
    res = {}
    for _ in range(3):
        for v in (1, 3):
            assert lib.mrp_tuning_set(b"edge_split_v", v) == 0
            res.setdefault(v, []).append(bench.time_launches([f], 20, dev))
    lib.mrp_tuning_set(b"reset", 0)
    print(name, E, C, {v: round(min(t) * 1e6, 1) for v, t in res.items()}, flush=True)
