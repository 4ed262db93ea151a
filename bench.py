#!/usr/bin/env python3
"""Benchmark: aggregated node-features/sec through one GCN layer (BASELINE.json ``metric``).

Workload (SURVEY.md §8(d) north-star target): per rank B=32 per-frame graphs of N=8 robots
(complete directed graphs, the reference's ``dgl/dataloader.py:88-95``), node features
C=512 x 32 x 32 fp32 (ResNet18 width at H/8 x W/8 of a 256^2 image), synthetic and seeded, already
resident in HBM.  A *step* is one forward pass of the drop-in ``GCN`` layer over that batch:
edge encoder (9 -> C -> 2C Linear/ReLU/Linear/Sigmoid on the 1792 edge poses: HIP hidden-layer
kernel + library GEMM) + the HIP FiLM-mean aggregation (which applies the encoder's sigmoid).  value = elements (Nt*C*H*W) aggregated per second over all ranks.

Multi-GPU (``torch.distributed.run``, one process per GPU): graphs of a batch are independent, so
each rank runs its own B=32 graphs with no data-path collective ("scaling": "weak"); time is the
max over ranks of the barrier-bracketed K steps.

Extra JSON fields:
* ``roofline`` — the aggregation kernel alone, timed with HIP events on its stream over back-to-back
  launches; achieved = algorithmic bytes per launch / mean launch time (bytes: DESIGN.md §4).
  ``traffic`` is the PMC-measured HBM bytes per launch (rocprofv3 FETCH_SIZE/WRITE_SIZE, corrected
  per MI355X_MICROARCH.md) when ``profiles/pmc_traffic_*.json`` for this workload exists, else null.
* ``cpu_baseline`` — the CPU oracle (a torch restatement of the reference DGL UDF path, same op
  sequence) on a bounded sample of the same workload, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import mrp_gnn_amd as mrp  # noqa: E402
from mrp_gnn_amd.dist import env_rank_world  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "aggregated node-features/sec (N×C×H×W elems through GCN) at 1/2/4/8 MI355X"


def make_workload(B, N, C, H, W, seed, device):
    rng = np.random.RandomState(seed)
    graphs = []
    for _ in range(B):
        t = rng.uniform(-10, 10, size=(N, 3))
        q = rng.standard_normal((N, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        graphs.append(mrp.frame_graph(np.concatenate([t, q], 1).astype(np.float32)))
    g = mrp.batch(graphs)
    gen = torch.Generator().manual_seed(seed)
    g.ndata["image"] = torch.randn(B * N, C, H, W, generator=gen)
    return g.to(device)


def alg_bytes_fwd(Nt, E, C, P):
    """Algorithmic HBM bytes of one forward aggregation launch: every source plane read once,
    gamma/beta read once, every output plane written once."""
    return Nt * C * P * 4 + E * 2 * C * 4 + Nt * C * P * 4


def time_kernel(x, gb, csr, out, iters, device):
    """Mean duration of one aggregation launch, HIP events on the launch stream."""
    stream = torch.cuda.current_stream(device)
    mode = mrp._lib.MODE_FILM_MEAN | mrp._lib.GB_LOGITS
    for _ in range(3):
        mrp.film_mean_forward_into(x, gb, csr, mode, out)
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    start.record(stream)
    for _ in range(iters):
        mrp.film_mean_forward_into(x, gb, csr, mode, out)
    end.record(stream)
    end.synchronize()
    return start.elapsed_time(end) / iters * 1e-3  # seconds


def cpu_baseline(N, C, H, W, seconds, sample_graphs):
    """The reference op sequence on the host (oracle: edge encoder -> gather -> FiLM -> degree
    bucket -> mean), bounded to about ``seconds`` of CPU work."""
    import oracle
    threads = torch.get_num_threads()
    g = make_workload(sample_graphs, N, C, H, W, seed=1234, device="cpu")
    torch.manual_seed(0)
    enc = mrp.edge_encoder([C, C])
    params = dict(enc.named_parameters())
    src, dst = (t.numpy() for t in g.edges())
    x = g.ndata["image"]
    pose = g.edata["pose"]
    elems = x.numel()
    with torch.no_grad():
        oracle.gcn_forward(params, x, pose, src, dst)  # warm-up
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.gcn_forward(params, x, pose, src, dst)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    return {"value": elems * reps / el, "unit": "elems/s", "cores": threads, "kind": "port",
            "sample": f"{sample_graphs} graphs x N={N} x C={C} x {H}x{W}, {reps} forward passes in {el:.1f} s, "
                      f"torch CPU fp32, {threads} threads"}


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


def pmc_traffic(workload):
    """Per-launch HBM bytes from a committed rocprofv3 PMC summary for this workload, if any."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic_*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload and d.get("kernel") == "film_fwd":
            return d.get("hbm_bytes_per_launch"), os.path.basename(f)
    return None, None


def max_over_ranks(seconds, world, device, backend):
    if world == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def train_step_time(gcn, g, x, world, device, args):
    """One training step of the layer: forward, backward through the HIP kernels and the edge
    encoder, and (N > 1) the bucketed gradient all-reduce of the replicated parameters."""
    from mrp_gnn_amd.dist import GradAllReducer
    xr = x.detach().clone().requires_grad_(True)
    grad = torch.randn_like(x)
    reducer = GradAllReducer(gcn.parameters()) if world > 1 else None

    def step():
        for p in gcn.parameters():
            p.grad = None
        xr.grad = None
        gcn(g, xr).backward(grad)
        if reducer is not None:
            reducer.synchronize()

    for _ in range(3):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.train_steps):
        step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t = max_over_ranks((time.perf_counter() - t0) / args.train_steps, world, device, args.dist_backend)
    nb = len(reducer.buckets) if reducer is not None else 0
    if reducer is not None:
        reducer.remove()
    return t, nb


def block_step_time(world, device, args, rank):
    """BASELINE configs[1]: the 2-layer GCN of multi_view_dgl_model (compress_gcn + multi_gcn:
    gcn1 -> cat -> conv1 -> gcn2 -> cat -> conv2, dgl/model/models.py:180-189) on B=16 8-robot
    graphs, 512 x 32 x 32 features, forward.  Reported beside the north-star line, not as value."""
    B, N, C, H = 16, 8, 512, 32
    g = make_workload(B, N, C, H, H, seed=100 + rank, device=device)
    opt = type("opt", (), {"feature_dim": C, "compress_gcn": True, "multi_gcn": True})()
    torch.manual_seed(0)
    block = mrp.GCNBlock(opt).to(device)
    x = g.ndata["image"]
    with torch.no_grad():
        for _ in range(3):
            block(g, x)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(args.block_steps):
            block(g, x)
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
    t = max_over_ranks((time.perf_counter() - t0) / args.block_steps, world, device, args.dist_backend)
    elems = 2 * g.num_nodes() * C * H * H  # two GCN layers
    return {"config": "configs[1]: B=16/rank, N=8 complete, C=512, 32x32, 2 GCN layers with 1x1 compress "
                      "(gcn1-cat-conv1-gcn2-cat-conv2), forward",
            "value": world * elems / t, "unit": "elems/s", "ms_per_step": t * 1e3}


def main():
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
    ap.add_argument("--cpu-sample-graphs", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-train", action="store_true", help="skip the training-step measurement")
    ap.add_argument("--train-steps", type=int, default=20)
    ap.add_argument("--no-block", action="store_true", help="skip the configs[1] 2-layer block measurement")
    ap.add_argument("--block-steps", type=int, default=10)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) or gloo (control-flow tests)")
    args = ap.parse_args()

    rank, world, local = env_rank_world()
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
    opt = type("opt", (), {"feature_dim": C})()
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
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        elapsed = max_over_ranks(elapsed, world, device, args.dist_backend)

        # dominant kernel alone, for the roofline
        z = gcn.edge_encoder.logits(g.edata["pose"])  # what GCN.forward hands the kernel
        out = torch.empty_like(x)
        t_kernel = time_kernel(x, z, csr, out, args.kernel_iters, device)

    train = None
    if not args.no_train:
        train = train_step_time(gcn, g, x, world, device, args)
    block = None if args.no_block else block_step_time(world, device, args, rank)
    gbuild = graph_build_time(B, N, device)

    elems_per_step = Nt * C * P
    value = world * elems_per_step * args.steps / elapsed
    bytes_launch = alg_bytes_fwd(Nt, E, C, P)
    achieved = bytes_launch / t_kernel / 1e9
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
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "film_fwd",
                     "kernel_us": t_kernel * 1e6, "alg_bytes_per_launch": bytes_launch,
                     "read_frac": (bytes_launch - Nt * C * P * 4) / t_kernel / 1e9 / HBM_PEAK_GBS,
                     "traffic_source": traffic_src},
    }
    if train is not None:
        t_train, reducer_buckets = train
        result["train_step"] = {
            "what": "GCN layer forward + backward (HIP fused dx/dgamma/dbeta kernel, encoder backward)"
                    + (" + bucketed gradient all-reduce" if world > 1 else ""),
            "value": world * elems_per_step / t_train, "unit": "elems/s", "ms_per_step": t_train * 1e3,
            "allreduce_buckets": reducer_buckets,
        }
    if block is not None:
        result["block_step"] = block
    result["graph_build"] = gbuild
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(N, C, H, W, args.cpu_seconds, args.cpu_sample_graphs)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
