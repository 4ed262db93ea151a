#!/usr/bin/env python3
"""Generate the golden fixtures in ``tests/golden/*.npz`` FROM THE REFERENCE ITSELF.

Run in the survey/build container only (needs the read-only reference at /root/reference; never
runs on the GPU box and is not collected by pytest):

    python tests/golden/make_golden.py

How: ``/root/reference/dgl/model/models.py`` is imported with empty stub modules for the
absent third-party packages (``dgl``, ``dgl.nn.pytorch``, ``dgl.function``, ``dgl.ops``,
``torchvision``), which it imports only at module level.  Its own ``edge_encoder``,
``edge_udf``, ``node_udf`` and ``GCN`` classes/functions then run unchanged, driven by
:class:`DGLGraphShim`, a restatement of the DGL graph semantics they use (``local_scope`` and
``update_all`` with DGL's UDF degree bucketing: mailboxes per in-degree bucket, in-edges sorted
by edge id, zero-in-degree nodes zero-filled).  Edge poses come from the reference's
``dgl/utils.py:cal_relative_pose`` on float32 arrays, exactly as its dataset builder calls it
(``dgl/dataloader.py:116-122``).  Backward vectors come from torch autograd through those
reference UDFs.  Only data (inputs + outputs) is written; no reference source is copied.
"""
from __future__ import annotations

import contextlib
import os
import sys
import types

import numpy as np
import torch

REF_DGL = "/root/reference/dgl"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    sys.dont_write_bytecode = True  # the reference tree is read-only
    stubs = {}
    tv = types.ModuleType("torchvision")
    tv.models = types.ModuleType("torchvision.models")
    stubs["torchvision"] = tv
    stubs["torchvision.models"] = tv.models
    dgl = types.ModuleType("dgl")
    dgl.nn = types.ModuleType("dgl.nn")
    dgl.nn.pytorch = types.ModuleType("dgl.nn.pytorch")
    dgl.nn.pytorch.GraphConv = type("GraphConv", (), {})  # imported, never used (models.py:7)
    dgl.function = types.ModuleType("dgl.function")
    dgl.ops = types.ModuleType("dgl.ops")
    for name, mod in [("dgl", dgl), ("dgl.nn", dgl.nn), ("dgl.nn.pytorch", dgl.nn.pytorch),
                      ("dgl.function", dgl.function), ("dgl.ops", dgl.ops)]:
        stubs[name] = mod
    for k, v in stubs.items():
        sys.modules.setdefault(k, v)
    sys.path.insert(0, REF_DGL)
    from model import models  # noqa: E402  (reference dgl/model/models.py)
    import utils  # noqa: E402  (reference dgl/utils.py; needs pandas, present)
    return models, utils


class _Batch:
    def __init__(self, src=None, data=None, mailbox=None):
        self.src, self.data, self.mailbox = src, data, mailbox


class DGLGraphShim:
    """The DGLGraph surface ``GCN.forward`` touches, with DGL's semantics."""

    def __init__(self, src, dst, num_nodes):
        self.src = torch.as_tensor(src, dtype=torch.int64)
        self.dst = torch.as_tensor(dst, dtype=torch.int64)
        self.n = num_nodes
        self.ndata, self.edata = {}, {}

    @contextlib.contextmanager
    def local_scope(self):
        sn, se = dict(self.ndata), dict(self.edata)
        try:
            yield
        finally:
            self.ndata, self.edata = sn, se

    def update_all(self, message_func, reduce_func):
        msgs = message_func(_Batch(src={k: v[self.src] for k, v in self.ndata.items()}, data=self.edata))
        deg = np.bincount(self.dst.numpy(), minlength=self.n)
        dst_np = self.dst.numpy()
        results, nodes = [], []
        for d in np.unique(deg):
            if d == 0:
                continue
            bkt = np.nonzero(deg == d)[0]
            eids = np.stack([np.sort(np.nonzero(dst_np == v)[0]) for v in bkt]).reshape(-1)
            mb = {k: m[torch.from_numpy(eids)].reshape((len(bkt), int(d)) + tuple(m.shape[1:])) for k, m in msgs.items()}
            results.append(reduce_func(_Batch(mailbox=mb)))
            nodes.append(torch.from_numpy(bkt))
        if results:
            idx = torch.cat(nodes)
            for k in results[0]:
                val = torch.cat([r[k] for r in results])
                full = torch.zeros((self.n,) + tuple(val.shape[1:]), dtype=val.dtype)
                self.ndata[k] = full.index_copy(0, idx, val)


def complete_edges(n):
    return [i for i in range(n) for j in range(n) if i != j], [j for i in range(n) for j in range(n) if i != j]


def knn_edges(pos, k):
    n = len(pos)
    d = np.linalg.norm(pos[:, None] - pos[None], axis=-1)
    src, dst = [], []
    for v in range(n):
        cand = sorted((u for u in range(n) if u != v), key=lambda u: (d[u, v], u))[:k]
        for u in sorted(cand):
            src.append(u)
            dst.append(v)
    return src, dst


def random_poses(rng, n):
    t = rng.uniform(-10, 10, size=(n, 3))
    q = rng.standard_normal((n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    # the dataset path holds poses as float32 tensors (dataloader_utils.py:114-116)
    return np.concatenate([t, q], 1).astype(np.float32)


def make_case(models, utils, name, graphs, C, H, W, seed, mode="film_mean"):
    """graphs: list of (num_nodes, src, dst, poses) per frame; batched like dgl.batch."""
    torch.manual_seed(seed)
    src, dst, pose, bnn = [], [], [], []
    off = 0
    for n, s, d, p in graphs:
        for u, v in zip(s, d):
            src.append(u + off)
            dst.append(v + off)
            pose.append(utils.cal_relative_pose(p[u], p[v]))  # dataloader.py:119-120 argument order
        bnn.append(n)
        off += n
    Nt, E = off, len(src)
    pose = torch.from_numpy(np.stack(pose)).float() if E else torch.zeros(0, 9)
    opt = types.SimpleNamespace(feature_dim=C)
    gcn = models.GCN(opt)  # reference class; default nn.Linear init under the seed
    enc = gcn.edge_encoder
    x = torch.randn(Nt, C, H, W)
    G = torch.randn(Nt, C, H, W)

    # (1) the reference GCN exactly as shipped (returns g.ndata['image'], models.py:226)
    g = DGLGraphShim(src, dst, Nt)
    g.ndata["image"] = x
    g.edata["pose"] = pose
    ref_returns_input = bool(torch.equal(gcn(g), x))

    # (2) the aggregate update_all computes, with the reference UDFs, forward + autograd backward
    xg = x.clone().requires_grad_(True)
    g = DGLGraphShim(src, dst, Nt)
    g.ndata["image"] = xg
    g.edata["pose"] = pose
    gam, bet = enc(g.edata["pose"])
    gam.retain_grad()
    bet.retain_grad()
    g.edata["pose_gamma"], g.edata["pose_beta"] = gam, bet
    if mode == "copy_mean":
        g.update_all(lambda edges: {"m": edges.src["image"]}, models.node_udf)
    else:
        g.update_all(models.edge_udf, models.node_udf)
    out = g.ndata["images"]
    (out * G).sum().backward()
    gb = torch.stack([gam.detach()[:, :, 0, 0], bet.detach()[:, :, 0, 0]], -1)
    zeros = torch.zeros(E, C)
    dgam = gam.grad[:, :, 0, 0] if gam.grad is not None else zeros
    dbet = bet.grad[:, :, 0, 0] if bet.grad is not None else zeros
    dgb = torch.stack([dgam, dbet], -1)
    sd = {k: v.detach().numpy() for k, v in enc.state_dict().items()}
    pg = {k: p.grad.numpy() if p.grad is not None else np.zeros(p.shape, np.float32) for k, p in enc.named_parameters()}
    arrays = dict(
        x=x.numpy(), pose=pose.numpy(), src=np.asarray(src, np.int64), dst=np.asarray(dst, np.int64),
        batch_num_nodes=np.asarray(bnn, np.int64), gb=gb.numpy(), out=out.detach().numpy(), grad_out=G.numpy(),
        dx=xg.grad.numpy(), dgb=dgb.numpy(), mode=np.array(mode), ref_gcn_returns_input=np.array(ref_returns_input),
    )
    for k, v in sd.items():
        arrays["param." + k] = v
    for k, v in pg.items():
        arrays["grad." + k] = v
    path = os.path.join(OUT_DIR, f"{name}.npz")
    np.savez_compressed(path, **arrays)
    print(f"{name}: Nt={Nt} E={E} C={C} {H}x{W} mode={mode} ref_returns_input={ref_returns_input} "
          f"-> {os.path.getsize(path)} B")


def make_checkpoint(models, utils, seed=11):
    """A checkpoint in the reference harness's format (``torch.save({'model': module, ...})``,
    dgl/training.py:350-353) holding reference ``GCN`` modules (class path ``model.models.GCN``),
    plus the reference's aggregate for a small complete batch computed with them.  Loaded by
    tests/test_compat.py through the ``model.models`` alias (mrp_gnn_amd.compat)."""
    import argparse
    torch.manual_seed(seed)
    C, H, W, n = 8, 4, 4, 4
    opt = argparse.Namespace(feature_dim=C, compress_gcn=True, multi_gcn=True, camera_num=n, image_size=128,
                             skip_level=False, task="depth")
    holder = torch.nn.Module()  # stands in for multi_view_dgl_model's GCN part (its encoder needs torchvision)
    holder.gcn1 = models.GCN(opt)
    holder.conv1 = torch.nn.Conv2d(2 * C, C, kernel_size=1)
    holder.gcn2 = models.GCN(opt)
    holder.conv2 = torch.nn.Conv2d(2 * C, C, kernel_size=1)
    rng = np.random.RandomState(seed)
    graphs = []
    for _ in range(2):
        p = random_poses(rng, n)
        graphs.append((n, *complete_edges(n), p))
    src, dst, pose = [], [], []
    for b, (nn_, s, d, p) in enumerate(graphs):
        src += [u + b * n for u in s]
        dst += [v + b * n for v in d]
        pose += [utils.cal_relative_pose(p[u], p[v]) for u, v in zip(s, d)]
    pose = torch.from_numpy(np.stack(pose)).float()
    x = torch.randn(2 * n, C, H, W)
    with torch.no_grad():
        outs = []
        for gcn in (holder.gcn1, holder.gcn2):
            g = DGLGraphShim(src, dst, 2 * n)
            g.ndata["image"] = x
            g.edata["pose"] = pose
            g.edata["pose_gamma"], g.edata["pose_beta"] = gcn.edge_encoder(pose)
            g.update_all(models.edge_udf, models.node_udf)
            outs.append(g.ndata["images"])
    path = os.path.join(OUT_DIR, "ref_gcn_checkpoint.pt")
    torch.save({"model": holder.gcn1, "stack": holder, "n_iter": 3}, path)
    np.savez_compressed(os.path.join(OUT_DIR, "ref_gcn_checkpoint_io.npz"), x=x.numpy(), pose=pose.numpy(),
                        src=np.asarray(src, np.int64), dst=np.asarray(dst, np.int64),
                        out_gcn1=outs[0].numpy(), out_gcn2=outs[1].numpy(),
                        **{"gcn1." + k: v.numpy() for k, v in holder.gcn1.state_dict().items()})
    print(f"ref_gcn_checkpoint: {os.path.getsize(path)} B")


def main():
    models, utils = import_reference()
    if "--checkpoint-only" in sys.argv:
        make_checkpoint(models, utils)
        return
    rng = np.random.RandomState(0)

    def frames(n, count, knn=None):
        out = []
        for _ in range(count):
            p = random_poses(rng, n)
            s, d = complete_edges(n) if knn is None else knn_edges(p[:, :3].astype(np.float64), knn)
            out.append((n, s, d, p))
        return out

    make_case(models, utils, "complete_n4_c8_4x4_b2", frames(4, 2), 8, 4, 4, seed=1)
    make_case(models, utils, "complete_n8_c16_8x8_b2", frames(8, 2), 16, 8, 8, seed=2)
    make_case(models, utils, "complete_n5_c32_8x8_b3", frames(5, 3), 32, 8, 8, seed=3)
    make_case(models, utils, "complete_n8_c16_16x16_b1", frames(8, 1), 16, 16, 16, seed=4)
    make_case(models, utils, "knn4_n16_c8_4x4_b1", frames(16, 1, knn=4), 8, 4, 4, seed=5)
    make_case(models, utils, "complete_n16_c4_4x4_b1", frames(16, 1), 4, 4, 4, seed=6)
    # ragged batch: mixed in-degrees, a zero-in-degree node (node 5), a multi-edge (0->1 twice),
    # a self-loop (3->3), odd plane size P = 15 (exercises the scalar path)
    p6, p3 = random_poses(rng, 6), random_poses(rng, 3)
    s6 = [0, 0, 2, 3, 4, 1, 0, 2, 3, 4, 1]
    d6 = [1, 1, 1, 3, 3, 0, 2, 4, 4, 0, 2]
    make_case(models, utils, "mixed_ragged_c4_3x5", [(6, s6, d6, p6), (3, [0, 1, 2], [1, 2, 0], p3)], 4, 3, 5, seed=7)
    make_case(models, utils, "copyu_complete_n5_c8_4x4_b2", frames(5, 2), 8, 4, 4, seed=8, mode="copy_mean")

    # relative pose: the reference's own self-check pair (float64, dgl/utils.py:80-85) + float32 pairs
    a = np.array([-5.902101516723632812e+01, 1.927141571044921875e+02, 5.996415138244628906e+00,
                  -2.683681845664978027e-01, 2.737782299518585205e-01, 6.468879580497741699e-01,
                  6.592115163803100586e-01])
    b = np.array([-5.506656265258789062e+01, 1.961531982421875000e+02, 5.998308658599853516e+00,
                  -4.198011383414268494e-02, 3.792373836040496826e-01, 1.026619002223014832e-01,
                  9.186278581619262695e-01])
    p1 = random_poses(rng, 64)
    p2 = random_poses(rng, 64)
    np.savez_compressed(
        os.path.join(OUT_DIR, "relpose.npz"),
        selfcheck_p1=a, selfcheck_p2=b, selfcheck_out=utils.cal_relative_pose(a, b),
        p1=p1, p2=p2, out=np.stack([utils.cal_relative_pose(u, v) for u, v in zip(p1, p2)]),
        quat=p1[:, 3:], so3=np.stack([utils.quat_to_so3(q) for q in p1[:, 3:]]),
    )
    print("relpose: selfcheck", utils.cal_relative_pose(a, b))
    make_checkpoint(models, utils)


if __name__ == "__main__":
    main()
