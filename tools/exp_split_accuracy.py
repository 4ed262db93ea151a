"""Accuracy lab (not product code): the configs[4] stack (3 layers, k-NN(4), C=1024, 16x16, B=8)
forward and backward with the compress products on the fp32 MFMA or the split-bf16 kernels, per
product, error of every output/gradient against the float64 restatement, beside the fp32
restatement's own error (tests/stack_ref.py).  usage: python tools/exp_split_accuracy.py [B]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mrp_gnn_amd as m  # noqa: E402
import stack_ref  # noqa: E402
from test_gpu_configs import frames, model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda:0")
g = frames(B, 16, 1024, 16, 16, seed=B * 7 + 16 + 1024, knn=4).to(dev)
net = model(1024, 3).to(dev)
params = {k: v.detach() for k, v in net.named_parameters()}
x0 = g.ndata["image"].detach().clone()
torch.manual_seed(1)
G = None
src, dst = (t.to(dev) for t in g.edges())
pose = g.edata["pose"]
for variant, ops in (("hip", None), ("split all", {"fwd", "dgrad", "wgrad"}), ("split fwd", {"fwd"}),
                     ("split dgrad", {"dgrad"}), ("split wgrad", {"wgrad"})):
    m.compress.set_compress_path("hip" if ops is None else "split", split_ops=ops or {"fwd", "dgrad", "wgrad"})
    x = x0.clone().requires_grad_(True)
    for p in net.parameters():
        p.grad = None
    out = net(g, x)
    if G is None:
        torch.manual_seed(1)
        G = torch.randn_like(out)
        kw = dict(layers=3, combine="cat_compress", alpha=0.25)
        f64 = stack_ref.run(params, x0, pose, src, dst, G, torch.float64, **kw)
        f32 = stack_ref.run(params, x0, pose, src, dst, G, torch.float32, **kw)
    out.backward(G)
    rows = [("forward", out, f32[0], f64[0]), ("dx", x.grad, f32[1], f64[1])]
    rows += [(k, p.grad, f32[2][k], f64[2][k]) for k, p in net.named_parameters()]
    worst = max(rows, key=lambda r: stack_ref.err(r[1], r[3]) / max(1e-5, 4 * stack_ref.err(r[2], r[3])))
    print(f"== {variant}: worst {worst[0]}")
    for name, o, a32, a64 in rows:
        e, e32 = stack_ref.err(o, a64), stack_ref.err(a32, a64)
        flag = "" if e <= max(1e-5, 4 * e32) else "  FAIL"
        print(f"   {name:34s} ours {e:.3e}  fp32 {e32:.3e}{flag}", flush=True)
m.compress.set_compress_path("split", split_ops={"fwd", "dgrad", "wgrad"})
