"""In-tree build of the HIP library ``lib/libmrp_gnn.so`` for gfx950 (hipcc cross-compiles on
a GPU-less host).  ``python -m mrp_gnn_amd.build`` or ``__graft_entry__.build()``."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
SOURCES = [os.path.join(PKG_DIR, "csrc", f) for f in ("film_mean_fwd.hip", "film_mean_bwd.hip", "film_mean_bwd_1_8.hip",
                                                    "film_mean_bwd_9_12.hip", "film_mean_bwd_13_16.hip",
                                                    "edge_encoder.hip", "frame_graph.hip",
                                                    "compress_gemm.hip", "encoder_split.hip",
                                                    "compress_split.hip")]
OBJ_DIR = os.path.join(PKG_DIR, "build")
HEADERS = [os.path.join(REPO, "include", "mrp_gnn.h")] + [os.path.join(PKG_DIR, "csrc", h) for h in (
    "film_mean_kernels.hpp", "film_mean_bwd_launch.hpp", "fast_math.hpp", "tuning.hpp", "encoder_split.hpp")]
OUT = os.path.join(PKG_DIR, "lib", "libmrp_gnn.so")
ARCH = os.environ.get("MRP_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the HIP library)")


def _obj(src: str) -> str:
    return os.path.join(OBJ_DIR, os.path.basename(src) + ".o")


def _stale(src: str) -> bool:
    obj = _obj(src)
    return not os.path.exists(obj) or os.path.getmtime(obj) <= max(os.path.getmtime(d) for d in [src] + HEADERS)


def needs_build(out: str = OUT) -> bool:
    """The library is missing, an object is older than its source or a header, or the library is
    older than an object (freshness is judged per object, not against the library)."""
    if not os.path.exists(out) or any(_stale(s) for s in SOURCES):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(_obj(s)) > t for s in SOURCES)


FLAGS = ["-O3", "-std=c++17", "-fPIC", "-mcode-object-version=5", "-ffp-contract=off", "-Wno-pass-failed"]
# per-source extras: the compress GEMMs' only VALU beside the MFMAs is the bias-row sum of the
# weight gradient, where packed f32 ops (SLP-vectorised scalar adds) cost more than scalar ones
# (MI355X_MICROARCH.md, filler prices)
EXTRA_FLAGS = {"compress_gemm.hip": ["-fno-slp-vectorize"]}


def _compile(src: str, verbose: bool) -> str:
    obj = _obj(src)
    if not _stale(src):
        return obj
    cmd = [hipcc(), f"--offload-arch={ARCH}"] + FLAGS + EXTRA_FLAGS.get(os.path.basename(src), []) + [
        "-I", os.path.join(REPO, "include"), "-c", src,
                                                      "-o", obj + ".tmp"]
    if verbose:
        print("[mrp_gnn build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    """Compile every source to an object (in parallel, one hipcc per file) and link the library."""
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    os.makedirs(OBJ_DIR, exist_ok=True)
    if force:
        for src in SOURCES:
            obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
            if os.path.exists(obj):
                os.remove(obj)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(len(SOURCES), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), SOURCES))
    tmp = OUT + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print("[mrp_gnn build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
