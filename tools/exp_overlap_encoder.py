"""Kernel lab (not product code): can the edge encoder of one half of the batch run under the
aggregation forward of the other half?  The headline no-grad step (encoder, then film_fwd) against
  split-k: the batch's graphs in k contiguous chunks; chunk i's encoder on a side stream while
           chunk i-1's aggregation runs on the main stream (the first chunk's encoder exposed).
Timed as HIP graphs of the whole step (bench.time_launches); outputs checked equal to the one-shot
step's.  usage: python tools/exp_overlap_encoder.py [iters]"""
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mrp_gnn_amd as mrp  # noqa: E402
from mrp_gnn_amd.dist import shard_graph  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
g = bench.make_workload(32, 8, 512, 32, 32, seed=1, device=dev)
x = g.ndata["image"]
torch.manual_seed(0)
gcn = mrp.GCN(types.SimpleNamespace(feature_dim=512)).to(dev).eval()
enc = gcn.edge_encoder
csr = g.csr(dev)
side = torch.cuda.Stream(dev)


def one_shot():
    with torch.no_grad():
        return [gcn(g, x)]


def chunks(k):
    parts = [shard_graph(g, i, k)[0] for i in range(k)]
    csrs = [p.csr(dev) for p in parts]
    poses = [p.edata["pose"] for p in parts]
    xs = [p.ndata["image"] for p in parts]

    def step():
        outs = []
        main = torch.cuda.current_stream(dev)
        with torch.no_grad():
            z = enc.logits(poses[0])
            for i in range(k):
                znext = None
                if i + 1 < k:
                    side.wait_stream(main)
                    with torch.cuda.stream(side):
                        znext = enc.logits(poses[i + 1])
                outs.append(mrp.film_mean(xs[i], z, csrs[i], "film_mean", logits=True))
                if znext is not None:
                    main.wait_stream(side)
                    z = znext
        return outs
    return step


ref = torch.cat(one_shot())
forms = [("one-shot", one_shot)] + [(f"split-{k}", chunks(k)) for k in (2, 4)]
for name, f in forms:
    out = torch.cat(f())
    torch.cuda.synchronize()
    same = torch.equal(out, ref)
    ts = [bench.time_launches([f], iters, dev) for _ in range(3)]
    print(f"{name:9s} {min(ts) * 1e6:7.1f} us (runs {', '.join(f'{t * 1e6:.1f}' for t in ts)})  equal {same}",
          flush=True)
