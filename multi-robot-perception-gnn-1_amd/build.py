"""In-tree build of the HIP library ``lib/libmrp_gnn.so`` for gfx950 (hipcc cross-compiles on
a GPU-less host).  ``python -m mrp_gnn_amd.build`` or ``__graft_entry__.build()``."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
SOURCES = [os.path.join(PKG_DIR, "csrc", "film_mean.hip"), os.path.join(PKG_DIR, "csrc", "edge_encoder.hip")]
OUT = os.path.join(PKG_DIR, "lib", "libmrp_gnn.so")
ARCH = os.environ.get("MRP_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the HIP library)")


def needs_build(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = SOURCES + [os.path.join(REPO, "include", "mrp_gnn.h")]
    return any(os.path.getmtime(s) > t for s in deps)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = OUT + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC", "-mcode-object-version=5", "-ffp-contract=off",
           "-Wno-pass-failed", "-I", os.path.join(REPO, "include"), "-o", tmp] + SOURCES
    if verbose:
        print("[mrp_gnn build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
