#!/usr/bin/env python3
"""Kernel lab (not product code): build a variant of the HIP library from a copy of csrc/ with a text
patch applied, into tools/bin/<name>.so, for in-process A/B runs against the product library
(tools/ab_libs.py).  The patch is a list of (file, old, new) replacements in a Python file defining
PATCH.
usage: python tools/build_variant_lib.py <name> <patch.py>"""
import os
import runpy
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mrp_gnn_amd import build as b  # noqa: E402

name, patch = sys.argv[1], sys.argv[2]
edits = runpy.run_path(patch)["PATCH"]
tmp = tempfile.mkdtemp()
src = os.path.join(tmp, "csrc")
shutil.copytree(os.path.join(b.PKG_DIR, "csrc"), src)
for f, old, new in edits:
    p = os.path.join(src, f)
    s = open(p).read()
    assert old in s, (f, old[:60])
    open(p, "w").write(s.replace(old, new))
objs = []
procs = []
for s in b.SOURCES:
    o = os.path.join(tmp, os.path.basename(s) + ".o")
    # LAB_FLAGS_<file stem>="-f... -f...": extra flags for one source of the variant
    lab = os.environ.get("LAB_FLAGS_" + os.path.basename(s).split(".")[0], "").split()
    cmd = [b.hipcc(), f"--offload-arch={b.ARCH}"] + b.FLAGS + b.EXTRA_FLAGS.get(os.path.basename(s), []) + lab + [
        "-I", os.path.join(ROOT, "include"), "-c", os.path.join(src, os.path.basename(s)), "-o", o]
    procs.append(subprocess.Popen(cmd))
    objs.append(o)
assert all(p.wait() == 0 for p in procs)
out = os.path.join(ROOT, "tools", "bin", name + ".so")
subprocess.run([b.hipcc(), f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", out] + objs, check=True)
shutil.rmtree(tmp)
print(out)
