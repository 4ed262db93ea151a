"""Kernel lab (not product code): the headline step (bench.py's no-grad GCN.forward, B = 32, N = 8, C = 512,
32 x 32) with the inference encoder on its own stream (``encoder.set_encoder_stream(True)``, the default)
at normal and high priority, against the caller's stream, timed like bench.py, settings interleaved over rounds; outputs compared.
usage: python tools/exp_encoder_stream.py [steps] [rounds]"""
import os
import sys
import time
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = torch.device("cuda:0")
g = bench.make_workload(32, 8, 512, 32, 32, seed=0, device=dev)
x = g.ndata["image"]
torch.manual_seed(0)
gcn = mrp.GCN(types.SimpleNamespace(feature_dim=512)).to(dev)
res, outs = {}, {}
with torch.no_grad():
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _ in range(20):
            gcn(g, x)
        torch.cuda.synchronize()
    # (own stream, priority, device-scope join)
    settings = [(False, 0, True), (True, 0, False), (True, -1, False), (True, 0, True), (True, -1, True)]
    for rnd in range(rounds):
        for on, prio, fj in settings:
            mrp.encoder.set_encoder_stream(on)
            mrp.encoder.set_encoder_stream_priority(prio)
            mrp.encoder.set_fast_join(fj)
            for _ in range(10):
                gcn(g, x)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(steps):
                out = gcn(g, x)
            torch.cuda.synchronize()
            res.setdefault((on, prio, fj), []).append((time.perf_counter() - t) / steps * 1e6)
            outs[(on, prio, fj)] = out.clone()
mrp.encoder.set_encoder_stream(True)
mrp.encoder.set_encoder_stream_priority(-1)
mrp.encoder.set_fast_join(True)
for (on, prio, fj), ts in res.items():
    print(f"encoder stream {'own' if on else 'caller'} priority {prio} join {'device' if fj else 'torch'}: "
          + " ".join(f"{t:6.1f}" for t in ts) + f"  min {min(ts):6.1f} us/step", flush=True)
print("outputs bit-identical:", all(torch.equal(o, outs[settings[0]]) for o in outs.values()))
