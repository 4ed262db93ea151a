#!/usr/bin/env python3
"""Experiment (not product code): does PyTorch TunableOp pick faster library GEMMs for the edge
encoder's shapes than the default heuristic?  Times forward z = addmm(b2, h, W2^T) and the two
backward GEMMs (dh = dz W2, dW2 = dz^T h) at E = 1792, C = 512 (the bench workload), default vs
tuned, and reports the BLAS backend (hipBLASLt vs rocBLAS) variants too.

    python tools/exp_tunableop.py            (on the GPU box)
"""
import os
import sys
import time

import torch


def bench(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    dev = torch.device("cuda:0")
    E, C = int(os.environ.get("E", 1792)), int(os.environ.get("C", 512))
    torch.manual_seed(0)
    h = torch.randn(E, C, device=dev)
    w2 = torch.randn(2 * C, C, device=dev)
    b2 = torch.randn(2 * C, device=dev)
    dz = torch.randn(E, 2 * C, device=dev)
    cases = {
        "fwd z=addmm(b2,h,W2^T)": lambda: torch.addmm(b2, h, w2.t()),
        "bwd dh=dz@W2": lambda: dz.mm(w2),
        "bwd dW2=dz^T@h": lambda: dz.t().mm(h),
    }
    flops = 2.0 * E * C * 2 * C
    for lib in ("default", "cublaslt", "cublas"):
        if lib != "default":
            try:
                torch.backends.cuda.preferred_blas_library(lib)
            except Exception as ex:  # noqa: BLE001
                print(f"{lib}: not selectable ({ex})")
                continue
        for name, fn in cases.items():
            us = bench(fn)
            print(f"{lib:9s} {name:26s} {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s", flush=True)
    torch.backends.cuda.preferred_blas_library("default")
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(os.path.join(os.environ.get("OUT", "gpurun_out"), "tunableop_results%d.csv"))
    t0 = time.time()
    for fn in cases.values():
        fn()
    torch.cuda.synchronize()
    print(f"tuning took {time.time() - t0:.1f} s", flush=True)
    tun.tuning_enable(False)
    for name, fn in cases.items():
        us = bench(fn)
        print(f"tunableop {name:26s} {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s", flush=True)
    tun.write_file()
    ref = torch.addmm(b2, h, w2.t())
    tun.enable(False)
    print("max |tuned - default| =", float((ref - torch.addmm(b2, h, w2.t())).abs().max()))


if __name__ == "__main__":
    sys.exit(main())
