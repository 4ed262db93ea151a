#!/usr/bin/env python3
"""Per-shape durations and LDS counters of a tools/prof_kernels.py run (kernel lab helper, not product
code): prof_kernels runs, per shape (north_star, configs[1..4]), `iters` forward then `iters` backward
launches, so dispatches are assigned to shapes by order.
usage: python tools/trace_shapes.py <dir with trace/ and optionally pmc_SQ2/> [iters] [pmc_iters]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
it = int(sys.argv[2]) if len(sys.argv) > 2 else 20
pit = int(sys.argv[3]) if len(sys.argv) > 3 else 5
SHAPES = ["north_star", "cfg1", "cfg2", "cfg3", "cfg4"]
f = glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))[0]
rows = sorted((r for r in csv.DictReader(open(f)) if "film_" in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
pmc = glob.glob(os.path.join(d, "pmc_SQ2", "*counter_collection.csv"))
per, names = collections.defaultdict(dict), {}
if pmc:
    for r in csv.DictReader(open(pmc[0])):
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] = float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
ids = [k for k in sorted(per) if "film_" in names[k]]
i = j = 0
for s in SHAPES:
    for kind in ("fwd", "bwd"):
        seg = rows[i:i + it]
        i += it
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in seg]
        line = f"{s:10s} {kind} {seg[0]['Kernel_Name'][:48]:48s} {sum(ds) / len(ds):7.1f} us"
        if ids:
            c = collections.defaultdict(float)
            for k in ids[j:j + pit]:
                for n, v in per[k].items():
                    c[n] += v
            j += pit
            line += (f"  LDS conflicts {c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_LDS_IDX_ACTIVE'], 1):.3f}"
                     f"  LDS inst {c['SQ_INSTS_LDS'] / pit:9.0f}  VALU inst {c['SQ_INSTS_VALU'] / pit:10.0f}")
        print(line)
