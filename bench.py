#!/usr/bin/env python3
"""Benchmark: aggregated node-features/sec through the GCN (BASELINE.json ``metric``).

Headline workload (SURVEY.md §8(d) north-star target): per rank B=32 per-frame graphs of N=8 robots
(complete directed graphs, the reference's ``dgl/dataloader.py:88-95``), node features
C=512 x 32 x 32 fp32 (ResNet18 width at H/8 x W/8 of a 256^2 image), synthetic and seeded, already
resident in HBM.  A *step* is one forward pass of the drop-in ``GCN`` layer over that batch, as the
reference's eval loop runs it (no gradient): edge encoder (9 -> C -> 2C Linear/ReLU/Linear on the 1792
edge poses in ONE HIP launch on the bf16 matrix cores at fp32 accuracy, ``mrp_edge_encoder_fwd_split``)
+ the HIP FiLM-mean aggregation (which applies the encoder's sigmoid).  value = elements
(Nt*C*H*W) aggregated per second over all ranks.

Multi-GPU (``torch.distributed.run``, one process per GPU): graphs of a batch are independent, so
each rank runs its own B=32 graphs with no data-path collective ("scaling": "weak"); time is the
max over ranks of the barrier-bracketed K steps.

Extra JSON fields:
* ``roofline`` — the aggregation kernel alone, timed with HIP events on its stream over back-to-back
  launches; achieved = algorithmic bytes per launch / mean launch time (bytes: DESIGN.md §4).
  ``traffic`` is the PMC-measured HBM bytes per launch (rocprofv3 FETCH_SIZE/WRITE_SIZE, corrected
  per MI355X_MICROARCH.md) when ``profiles/pmc_traffic_*.json`` for this workload exists, else null.
* ``configs`` — one record per BASELINE.json config (configs[1..4]): the config's GCN stack (layers,
  1x1 compress, k-NN graphs) forward and training step, and the roofline of its own forward and
  backward aggregation kernels, timed over rotating buffer sets larger than the 256 MB Infinity
  Cache.  configs[3] and [4] are data-parallel configs: with N > 1 ranks their global batch (32 and
  64 graphs) is split over the ranks (``dist.shard_graph``, "strong"), and the training step
  all-reduces the gradients over RCCL; with one rank they run the per-GPU share (8 graphs).
* ``configs[0]`` — the reference's CPU-runnable case (4-robot graphs, 64 x 32 x 32, 1 layer, batch 8):
  the CPU oracle's rate beside the HIP layer's at the same shape (rank 0, N = 1).
* ``cpu_baseline`` — the CPU oracle (a torch restatement of the reference DGL UDF path, same op
  sequence) on the headline workload, rank 0 at N=1 only, bounded in time; threads = the job's CPU
  share (OMP_NUM_THREADS) or the affinity mask, with the host's counts reported beside it.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import statistics
import sys
import time
import types

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import mrp_gnn_amd as mrp  # noqa: E402
from mrp_gnn_amd.dist import GradAllReducer, env_rank_world, shard_graph  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
MALL_BYTES = 256 << 20  # Infinity Cache: rotating buffer sets must exceed 2x this
METRIC = "aggregated node-features/sec (N×C×H×W elems through GCN) at 1/2/4/8 MI355X"

# BASELINE.json configs[1..4] (configs[0] is the reference's CPU-only case: cpu_baseline).
# SURVEY.md §8(d) fixes the shapes; "per_gpu" is the graphs one GPU holds in the config.
CONFIGS = {
    1: dict(name="configs[1]: 8-robot warehouse, ResNet18 512 x H/8 x W/8 (32x32), 2-layer GCN "
                 "(multi_gcn + compress), batch 16, 1 GPU",
            batch=16, per_gpu=16, N=8, C=512, H=32, layers=2, knn=None, split=False),
    2: dict(name="configs[2]: 8-robot airsim, gcn_compress (FiLM e_mul_u, 1x1 compress), MobileNetV2 "
                 "1280 x 8x8, batch 32, 1 GPU",
            batch=32, per_gpu=32, N=8, C=1280, H=8, layers=1, knn=None, split=False),
    3: dict(name="configs[3]: 8-robot warehouse, ResNet50 2048 x 8x8, 2-layer GCN (multi_gcn + compress; "
                 "GCN2Conv mapped per SURVEY §8(d)), batch 32, DP over 4 GPUs",
            batch=32, per_gpu=8, N=8, C=2048, H=8, layers=2, knn=None, split=True),
    4: dict(name="configs[4]: 16-robot synthetic k-NN(4), 1024 x 16x16, 3 GCN layers, batch 64, DP over 8 "
                 "GPUs with RCCL gradient all-reduce",
            batch=64, per_gpu=8, N=16, C=1024, H=16, layers=3, knn=4, split=True),
}


def make_workload(B, N, C, H, W, seed, device, knn=None, features=True):
    rng = np.random.RandomState(seed)
    graphs = []
    for _ in range(B):
        t = rng.uniform(-10, 10, size=(N, 3))
        q = rng.standard_normal((N, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        graphs.append(mrp.frame_graph(np.concatenate([t, q], 1).astype(np.float32), knn=knn))
    g = mrp.batch(graphs)
    if features:
        gen = torch.Generator().manual_seed(seed)
        g.ndata["image"] = torch.randn(B * N, C, H, W, generator=gen)
    return g.to(device)


def alg_bytes_fwd(Nt, E, C, P):
    """Algorithmic HBM bytes of one forward aggregation launch: every source plane read once,
    gamma/beta read once, every output plane written once."""
    return Nt * C * P * 4 + E * 2 * C * 4 + Nt * C * P * 4


def alg_bytes_bwd(Nt, E, C, P, base=False):
    """Backward (dx + d gamma/beta): grad_out and x read once, gamma/beta read once, dx written once,
    d gamma/beta written once; ``base``: the training form, which also reads the
    grad_x base (x's gradient from the 1x1 compress, added into dx) once."""
    return (3 if base else 2) * Nt * C * P * 4 + E * 2 * C * 4 + Nt * C * P * 4 + E * 2 * C * 4


def time_launches(launches, iters, device):
    """Duration of one launch (median over 5 graph replays), HIP events on the launch stream; ``launches`` are closures over
    distinct buffer sets, run round-robin.  The ``iters`` launches are captured once in a HIP graph
    and the events bracket its replay, so a short kernel is timed back to back on the device rather
    than at the rate Python can issue ctypes calls (~15-20 us per call: more than a small config's
    whole kernel)."""
    for f in launches * 2:
        f()
    torch.cuda.synchronize(device)
    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        for i in range(iters):
            launches[i % len(launches)]()
    graph.replay()  # warm
    torch.cuda.synchronize(device)
    stream = torch.cuda.current_stream(device)
    # median of 5 replays: single replays of the same launches differ by up to ~10 % box to box
    # (clock and power state), which one replay would report as a kernel difference
    times = []
    for _ in range(5):
        start = torch.cuda.Event(enable_timing=True)
        end = torch.cuda.Event(enable_timing=True)
        start.record(stream)
        graph.replay()
        end.record(stream)
        end.synchronize()
        times.append(start.elapsed_time(end))
    del graph
    times.sort()
    return times[2] / iters * 1e-3  # seconds


def copy_ceiling(plane_bytes, device, iters):
    """The same box's streaming ceiling at a kernel's plane bytes, timed exactly like the kernels
    (HIP graph over rotating buffer sets > 512 MB, median of replays): ``mrp_stream_copy`` of
    ``plane_bytes`` (one read and one write of each byte, nontemporal float4).  Returns its record;
    ``ceiling_frac`` of a kernel = its achieved GB/s over this copy's (a driver
    number that is low against 8 TB/s but level with this reads as the box, not as a regression)."""
    lib = mrp.load_library()
    n = plane_bytes // 4
    sets = rotating_sets(2 * plane_bytes)
    bufs = [(torch.empty(n, device=device), torch.empty(n, device=device)) for _ in range(sets)]
    for a, _ in bufs:
        a.normal_()
    nb = n * 4 // 16 * 16

    def launch(a, b):
        code = lib.mrp_stream_copy(a.data_ptr(), b.data_ptr(), nb, torch.cuda.current_stream(device).cuda_stream)
        if code != 0:
            raise RuntimeError(f"mrp_stream_copy failed: {code}")

    t = time_launches([lambda a=a, b=b: launch(a, b) for a, b in bufs], iters, device)
    del bufs
    ach = 2 * nb / t / 1e9
    return {"kernel": "mrp_stream_copy (1 read + 1 write, float4, nontemporal)", "bytes": 2 * nb, "us": t * 1e6,
            "achieved": ach, "frac": ach / HBM_PEAK_GBS, "rotating_sets": sets}


def with_ceiling(rec, ceil):
    """Attach the copy yardstick: the kernel's achieved GB/s as a fraction of the copy's on this box."""
    rec["ceiling_frac"] = rec["achieved"] / ceil["achieved"]
    rec["copy_ceiling_frac_of_peak"] = ceil["frac"]
    return rec


def roofline(kernel, bytes_launch, t, traffic=None, traffic_src=None, **extra):
    achieved = bytes_launch / t / 1e9
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": traffic, "kernel": kernel, "kernel_us": t * 1e6, "alg_bytes_per_launch": bytes_launch}
    if traffic_src:
        r["traffic_source"] = traffic_src
    r.update(extra)
    return r


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_threads():
    """Threads for the CPU baseline: the job's CPU share (OMP_NUM_THREADS, which the GPU pool sets to
    the per-GPU share of the host) or else every CPU this process may run on; plus what the host has."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = int(omp) if omp and omp.isdigit() and int(omp) > 0 else aff
    return threads, {"os_cpu_count": os.cpu_count(), "affinity_cpus": aff, "omp_num_threads": omp,
                     "threads_used": threads}


def cpu_oracle_rate(B, N, C, H, W, seconds, knn=None):
    """elems/s of the oracle GCN forward (the reference op sequence on the host) over about
    ``seconds`` of CPU work, with the baseline's thread count."""
    import oracle
    threads, _ = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        g = make_workload(B, N, C, H, W, seed=1234, device="cpu", knn=knn)
        torch.manual_seed(0)
        enc = mrp.edge_encoder([C, C])
        params = dict(enc.named_parameters())
        src, dst = (t.numpy() for t in g.edges())
        x, pose = g.ndata["image"], g.edata["pose"]
        with torch.no_grad():
            reps, t0 = 0, time.perf_counter()
            while True:
                oracle.gcn_forward(params, x, pose, src, dst)
                reps += 1
                el = time.perf_counter() - t0
                if el >= seconds:
                    break
    finally:
        torch.set_num_threads(prev)
    return x.numel() * reps / el, reps, el, threads


def cpu_baseline(B, N, C, H, W, seconds):
    """The reference op sequence on the host (oracle: edge encoder -> gather -> FiLM -> degree
    bucket -> mean) over the headline workload itself, bounded to about ``seconds`` of CPU work."""
    import oracle
    threads, counts = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        g = make_workload(B, N, C, H, W, seed=1234, device="cpu")
        torch.manual_seed(0)
        enc = mrp.edge_encoder([C, C])
        params = dict(enc.named_parameters())
        src, dst = (t.numpy() for t in g.edges())
        x = g.ndata["image"]
        pose = g.edata["pose"]
        elems = x.numel()
        with torch.no_grad():
            reps, t0 = 0, time.perf_counter()
            while True:
                oracle.gcn_forward(params, x, pose, src, dst)
                reps += 1
                el = time.perf_counter() - t0
                if el >= seconds:
                    break
    finally:
        torch.set_num_threads(prev)
    return {"value": elems * reps / el, "unit": "elems/s", "cores": threads, "kind": "port",
            "cpu": cpu_model(), "host": counts,
            "threads_note": "the job's CPU share (OMP_NUM_THREADS, set by the GPU pool to the per-GPU share "
                            "of the host) when set, else every CPU in the process's affinity mask",
            "sample": f"the headline workload itself ({B} graphs x N={N} x C={C} x {H}x{W}), {reps} forward "
                      f"passes in {el:.1f} s, torch CPU fp32, {threads} threads"}


def config0_record(device, args):
    """BASELINE configs[0]: the reference's CPU-runnable case — 4-robot complete graphs, 64 x 32 x 32
    node features, one GCN layer, batch 8 (dgl/training.py:28 default), on the DGL CPU path
    (dgl/training.py:176-218 plumbing).  DGL is absent, so the CPU number is the oracle (the same op
    sequence in torch); beside it the HIP layer on the GPU at the same shape."""
    B, N, C, H = 8, 4, 64, 32
    g = make_workload(B, N, C, H, H, seed=77, device=device)
    torch.manual_seed(0)
    gcn = mrp.GCN(types.SimpleNamespace(feature_dim=C)).to(device)
    x = g.ndata["image"]
    # host-bound steps (~50 us of GPU work): the median of three timed runs
    with torch.no_grad():
        for _ in range(10):
            gcn(g, x)
        t = statistics.median(timed(lambda: gcn(g, x), 50, 1, device, args.dist_backend) for _ in range(3))
    xr = x.detach().clone().requires_grad_(True)
    gy = torch.randn_like(x)

    def train():
        for p in gcn.parameters():
            p.grad = None
        xr.grad = None  # the layer's input is the backbone's output in the reference: never accumulated
        gcn(g, xr).backward(gy)

    for _ in range(5):
        train()
    tt = statistics.median(timed(train, 20, 1, device, args.dist_backend) for _ in range(3))
    rec = {"config": "configs[0]: 4-robot complete graph, random 64x32x32 node feats, 1 GraphConv layer, "
                     "DGL CPU backend (dgl/training.py plumbing)",
           "graphs": B, "robots": N, "channels": C, "H": H, "W": H, "layers": 1,
           "gpu_forward": {"value": x.numel() / t, "unit": "elems/s", "ms_per_step": t * 1e3},
           "gpu_train_step": {"value": x.numel() / tt, "unit": "elems/s", "ms_per_step": tt * 1e3}}
    if not args.no_cpu_baseline:
        rate, reps, el, threads = cpu_oracle_rate(B, N, C, H, H, min(args.cpu_seconds, 5.0))
        rec["cpu_forward"] = {"value": rate, "unit": "elems/s", "kind": "port", "cores": threads,
                              "sample": f"{reps} oracle forward passes in {el:.1f} s, torch CPU fp32"}
        rec["gpu_over_cpu"] = rec["gpu_forward"]["value"] / rate
    return rec


def graph_build_time(B, N, device, reps=20):
    """Per-batch graph construction: the device builder (``frame_batch``: one kernel for edge list,
    relative poses and CSR) against the host path the reference's dataset runs (per-frame
    ``cal_relative_pose`` + ``dgl.batch``, restated by ``frame_graph`` + ``batch``)."""
    rng = np.random.RandomState(7)
    t = rng.uniform(-10, 10, size=(B, N, 3))
    q = rng.standard_normal((B, N, 4))
    q /= np.linalg.norm(q, axis=-1, keepdims=True)
    poses = np.concatenate([t, q], -1).astype(np.float32)
    pd = torch.from_numpy(poses).to(device)
    for _ in range(3):
        mrp.frame_batch(pd)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(reps):
        g = mrp.frame_batch(pd)
    torch.cuda.synchronize(device)
    dev_s = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(3):
        gh = mrp.batch([mrp.frame_graph(p) for p in poses]).to(device)
        gh.csr(device)
    torch.cuda.synchronize(device)
    host_s = (time.perf_counter() - t0) / 3
    assert torch.equal(g.edata["pose"].cpu(), gh.edata["pose"].cpu())
    return {"what": f"build B={B} complete {N}-robot frame graphs (edge poses + CSR), ready on the device",
            "device_us": dev_s * 1e6, "host_us": host_s * 1e6}


def pmc_traffic(workload, kernel="film_fwd"):
    """Per-launch HBM bytes from a committed rocprofv3 PMC summary for this workload, if any."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic_*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for rec in d if isinstance(d, list) else [d]:
            if rec.get("workload") == workload and rec.get("kernel") == kernel:
                return rec.get("hbm_bytes_per_launch"), os.path.basename(f)
    return None, None


def max_over_ranks(seconds, world, device, backend):
    if world == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed(fn, steps, world, device, backend):
    """Barrier + synchronize on both sides of ``steps`` calls; max over ranks (seconds per call)."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    return max_over_ranks((time.perf_counter() - t0) / steps, world, device, backend)


def train_step_time(gcn, g, x, world, device, args):
    """One training step of the layer: forward, backward through the HIP kernels and the edge
    encoder, and (N > 1) the bucketed gradient all-reduce of the replicated parameters."""
    xr = x.detach().clone().requires_grad_(True)
    grad = torch.randn_like(x)
    reducer = GradAllReducer(gcn.parameters()) if world > 1 else None

    def step():
        for p in gcn.parameters():
            p.grad = None
        xr.grad = None
        if reducer is not None:
            reducer.arm()  # the backward kernels write the gradients straight into the buckets
        gcn(g, xr).backward(grad)
        if reducer is not None:
            reducer.synchronize()

    for _ in range(3):
        step()
    t = timed(step, args.train_steps, world, device, args.dist_backend)
    nb = len(reducer.buckets) if reducer is not None else 0
    if reducer is not None:
        reducer.remove()
    return t, nb


def rotating_sets(set_bytes, min_total=2 * MALL_BYTES + (128 << 20), max_sets=64):
    """How many buffer sets of ``set_bytes`` to rotate so the timed launches stream from HBM."""
    return max(1, min(max_sets, -(-min_total // max(set_bytes, 1))))


def config_record(cid, world, rank, device, args):
    """One BASELINE config: its GCN stack's forward and training step, and the roofline of its own
    forward and backward aggregation kernels over rotating buffers."""
    cfg = CONFIGS[cid]
    N, C, H, layers, knn = cfg["N"], cfg["C"], cfg["H"], cfg["layers"], cfg["knn"]
    P = H * H
    if cfg["split"] and world > 1:
        # the global batch's frames on every rank (cheap), this rank's share of them with features
        glob_g = make_workload(cfg["batch"], N, C, H, H, seed=300 + cid, device="cpu", knn=knn, features=False)
        g, (lo, hi) = shard_graph(glob_g, rank, world)
        gen = torch.Generator().manual_seed(1000 * cid + lo)
        g.ndata["image"] = torch.randn(g.num_nodes(), C, H, H, generator=gen)
        g = g.to(device)
        scaling, share = "strong", f"graphs [{lo}, {hi}) of {cfg['batch']}"
    else:
        B = cfg["per_gpu"] if cfg["split"] else cfg["batch"]
        g = make_workload(B, N, C, H, H, seed=300 + cid + 17 * rank, device=device, knn=knn)
        lo, hi = 0, B
        scaling = "weak"
        share = f"{B} graphs per rank" + (f" (the per-GPU share of {cfg['batch']})" if cfg["split"] else "")
    opt = types.SimpleNamespace(feature_dim=C, compress_gcn=True, multi_gcn=False, gcn_layers=layers,
                                gcn_combine="cat_compress")
    torch.manual_seed(0)
    net = mrp.GCNStack(opt).to(device)
    x = g.ndata["image"]
    Nt, E = g.num_nodes(), g.num_edges()
    csr = g.csr(device)
    elems = layers * Nt * C * P  # node features through the GCN layers per step (this rank)
    rec = {"config": cfg["name"], "graphs_per_rank": hi - lo, "share": share, "robots": N, "channels": C,
           "H": H, "W": H, "layers": layers, "graph": f"k-NN({knn})" if knn else "complete",
           "graph_kind": "regular" if knn else "complete", "scaling": scaling}
    # forward and training step on the matrix-core compress kernels (the product path) and, for
    # comparison, on the cat kernel + torch's library GEMMs ("library", the round-2 path): timed
    # alternately, three rounds each, median per path — the first timed block of a sequence runs a
    # few % slow (clocks), which a single A-then-B comparison would credit to the path
    xr = x.detach().clone().requires_grad_(True)
    gy = torch.randn(Nt, C, H, H, device=device)
    reducer = GradAllReducer(net.parameters()) if world > 1 else None
    if reducer is not None:
        reducer.set_local_count(hi - lo)

    def fwd():
        with torch.no_grad():
            net(g, x)

    def train():
        for p in net.parameters():
            p.grad = None
        # the input stands in for the backbone's output (not a leaf in the reference's training,
        # dgl/training.py:192-209): its gradient is computed and written every step, never added to
        # the previous step's (which would time an extra N C H W accumulation per step)
        xr.grad = None
        if reducer is not None:
            reducer.arm()
        net(g, xr).backward(gy)
        if reducer is not None:
            reducer.synchronize()

    prev = mrp.compress.compress_path()
    product = prev  # the package default ("split": split-bf16 forward / data gradient)
    times = {(k, path): [] for k in ("fwd", "train") for path in (product, "library")}
    try:
        for _ in range(2):
            fwd()
            train()
        for _ in range(3):
            for path in (product, "library"):
                mrp.compress.set_compress_path(path)
                for k, fn in (("fwd", fwd), ("train", train)):
                    for _ in range(2):
                        fn()
                    times[(k, path)].append(timed(fn, args.config_steps, world, device, args.dist_backend))
    finally:
        mrp.compress.set_compress_path(prev)
    med = {k: sorted(v)[1] for k, v in times.items()}
    t, tt = med[("fwd", product)], med[("train", product)]
    rec["forward"] = {"value": world * elems / t if scaling == "weak" else None, "unit": "elems/s",
                      "ms_per_step": t * 1e3,
                      "compress": f"aggregate kernel + matrix-core compress kernels, path {product!r} (no cat buffer)",
                      "ms_per_step_library_compress": med[("fwd", "library")] * 1e3}
    if scaling == "strong":  # every rank holds a different part of one global batch
        tot = torch.tensor([float(elems)], dtype=torch.float64,
                           device=device if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tot)
        rec["forward"]["value"] = float(tot.item()) / t
    rec["train_step"] = {"value": rec["forward"]["value"] * t / tt, "unit": "elems/s", "ms_per_step": tt * 1e3,
                         "ms_per_step_library_compress": med[("train", "library")] * 1e3,
                         "allreduce": (f"{len(reducer.buckets)} bucket(s), {sum(p.numel() for p in net.parameters()) * 4 / 2**20:.1f} MiB"
                                       if reducer is not None else None)}
    if reducer is not None:
        reducer.remove()
    # kernel rooflines on rotating buffer sets (layer 1's aggregation: the kernels every layer runs)
    with torch.no_grad():
        z = net.gcn1.edge_encoder.logits(g.edata["pose"])
    mode = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
    plane = Nt * C * P * 4
    nf = rotating_sets(2 * plane + E * 2 * C * 4)
    sets = [(x if i == 0 else torch.randn_like(x), torch.empty_like(x)) for i in range(nf)]
    launches = [lambda xi=xi, oi=oi: mrp.film_mean_forward_into(xi, z, csr, mode, oi) for xi, oi in sets]
    tf = time_launches(launches, args.kernel_iters, device)
    kname = "film_fwd_regular" if knn else "film_fwd"
    rec["roofline_fwd"] = roofline(kname, alg_bytes_fwd(Nt, E, C, P), tf, rotating_sets=nf,
                                   footprint_mb=round(nf * (2 * plane) / 2**20))
    del sets, launches
    ceil = copy_ceiling(plane, device, args.kernel_iters)
    rec["copy_ceiling"] = ceil
    with_ceiling(rec["roofline_fwd"], ceil)
    # the backward as training runs it (FilmCompressFunction: x's compress gradient is the base that
    # the kernel adds into dx, the DXB instantiation), and without the base for comparison
    nb = rotating_sets(4 * plane + 2 * E * 2 * C * 4)
    bsets = [(torch.randn_like(x), x if i == 0 else torch.randn_like(x), torch.randn_like(x)) for i in range(nb)]

    def bwd(G, xi, base):
        return mrp.aggregate.film_mean_backward(G, xi, z, csr, mode, True, True, grad_x_base=base)

    # k-NN graphs of > 8 nodes: the matrix-core backward (whole 64-pixel groups), else the VALU kernels
    bname = (("film_bwd_mfma" if P % 64 == 0 else "film_bwd_regular") if knn and N > 8 else "film_bwd_fused")
    launches = [lambda G=G, xi=xi, bs=bs: bwd(G, xi, bs) for G, xi, bs in bsets]
    tb = time_launches(launches, args.kernel_iters, device)
    rec["roofline_bwd"] = with_ceiling(roofline(bname, alg_bytes_bwd(Nt, E, C, P, base=True), tb, rotating_sets=nb,
                                                footprint_mb=round(nb * (4 * plane) / 2**20),
                                                form="training: grad_x base added in-kernel (the DXB instantiation)"),
                                       ceil)
    launches = [lambda G=G, xi=xi: bwd(G, xi, None) for G, xi, _ in bsets]
    tb0 = time_launches(launches, args.kernel_iters, device)
    rec["roofline_bwd_no_base"] = with_ceiling(roofline(bname, alg_bytes_bwd(Nt, E, C, P), tb0, rotating_sets=nb,
                                                        footprint_mb=round(nb * (3 * plane) / 2**20)), ceil)
    del bsets, launches
    return rec


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(argv, gpus: int, port: int):
    """(argv, env) that start ``gpus`` ranks of this script, one process per GPU, with
    ``torch.distributed.run`` on 127.0.0.1 — the launch ``bench.py --gpus N`` performs by itself
    when it is not already running under a launcher (no WORLD_SIZE in the environment)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC: RCCL / tensor sharing across ranks
    env.pop("WORLD_SIZE", None)
    return cmd, env


def self_launch(argv) -> int:
    """``--gpus N > 1`` outside a launcher: start the N ranks as child processes and return their
    exit status (rank 0 prints the JSON line).  Runs before this process touches the GPU."""
    import subprocess
    gpus = int(parse_args(argv).gpus)
    cmd, env = launcher_command(argv, gpus, _free_port())
    return subprocess.call(cmd, env=env)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--graphs", type=int, default=32, help="graphs per rank (B)")
    ap.add_argument("--nodes", type=int, default=8, help="robots per graph (N)")
    ap.add_argument("--channels", type=int, default=512)
    ap.add_argument("--hw", type=int, default=32)
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--spinup-s", type=float, default=0.5,
                    help="untimed back-to-back steps before the warmup steps (GPU clock ramp from idle)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-train", action="store_true", help="skip the training-step measurement")
    ap.add_argument("--train-steps", type=int, default=20)
    ap.add_argument("--configs", default="0,1,2,3,4", help="BASELINE configs to measure ('' for none)")
    ap.add_argument("--config-steps", type=int, default=10)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) or gloo (control-flow tests)")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(sys.argv[1:]))

    rank, world, local = env_rank_world()
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    ndev = max(torch.cuda.device_count(), 1)
    device = torch.device("cuda", local % ndev)
    torch.cuda.set_device(device)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.dist_backend)

    B, N, C, H, W = args.graphs, args.nodes, args.channels, args.hw, args.hw
    P = H * W
    workload = f"gcn_film_mean_fwd_B{B}_N{N}_complete_C{C}_{H}x{W}_fp32"
    g = make_workload(B, N, C, H, W, seed=rank, device=device)
    opt = types.SimpleNamespace(feature_dim=C)
    torch.manual_seed(0)
    gcn = mrp.GCN(opt).to(device)
    x = g.ndata["image"]
    csr = g.csr(device)
    Nt, E = g.num_nodes(), g.num_edges()

    def step():
        return gcn(g, x)

    with torch.no_grad():
        # Clock / memory power-state ramp: from idle the first ~20-100 ms of back-to-back launches
        # run up to 1.9x slower (tools/exp_ramp.py: 348 -> 209 -> 188 -> 180 us per aggregation over
        # the first 60 ms; steps 294 -> 243 -> 226 -> 214 -> 207 us).  Run the step untimed for
        # --spinup-s seconds first so the K timed steps measure the steady state, not the ramp.
        spin_t0 = time.perf_counter()
        spin_steps = 0
        while time.perf_counter() - spin_t0 < args.spinup_s:
            for _ in range(20):
                step()
            torch.cuda.synchronize(device)
            spin_steps += 20
        for _ in range(args.warmup):
            step()
        elapsed = timed(step, args.steps, world, device, args.dist_backend) * args.steps

        # dominant kernel alone, for the roofline
        z = gcn.edge_encoder.logits(g.edata["pose"])  # what GCN.forward hands the kernel
        out = torch.empty_like(x)
        mode = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
        t_kernel = time_launches([lambda: mrp.film_mean_forward_into(x, z, csr, mode, out)], args.kernel_iters,
                                 device)
        del out
        ceil_h = copy_ceiling(Nt * C * P * 4, device, args.kernel_iters)

    train = None if args.no_train else train_step_time(gcn, g, x, world, device, args)
    configs = {}
    for cid in [int(c) for c in args.configs.split(",") if c.strip()]:
        if cid == 0:
            if world == 1:  # the reference's single-process CPU case: one rank, no sharding
                configs["configs[0]"] = config0_record(device, args)
        else:
            configs[f"configs[{cid}]"] = config_record(cid, world, rank, device, args)
        torch.cuda.empty_cache()
    gbuild = graph_build_time(B, N, device)

    elems_per_step = Nt * C * P
    value = world * elems_per_step * args.steps / elapsed
    bytes_launch = alg_bytes_fwd(Nt, E, C, P)
    traffic, traffic_src = pmc_traffic(workload)
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "elems/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "spinup": {"seconds": args.spinup_s, "steps": spin_steps,
                   "why": "untimed steps before the warmup so the timed steps see steady GPU clocks"},
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded complete 8-robot graphs, relative poses from random robot poses, randn features)",
        "config": {"workload": workload, "graphs_per_rank": B, "global_graphs": B * world, "robots": N,
                   "channels": C, "H": H, "W": W, "layers": 1, "parallelism": f"dp{world} (independent graphs)"},
        "roofline": with_ceiling(roofline("film_fwd", bytes_launch, t_kernel, traffic, traffic_src,
                                          read_frac=(bytes_launch - Nt * C * P * 4) / t_kernel / 1e9 / HBM_PEAK_GBS),
                                 ceil_h),
        "copy_ceiling": ceil_h,
    }
    if train is not None:
        t_train, reducer_buckets = train
        result["train_step"] = {
            "what": "GCN layer forward + backward (HIP fused dx/dgamma/dbeta kernel, encoder backward)"
                    + (" + bucketed gradient all-reduce" if world > 1 else ""),
            "value": world * elems_per_step / t_train, "unit": "elems/s", "ms_per_step": t_train * 1e3,
            "allreduce_buckets": reducer_buckets,
        }
    if configs:
        result["configs"] = configs
    result["graph_build"] = gbuild
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(B, N, C, H, W, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
