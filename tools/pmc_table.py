"""Kernel lab (not product code): per-kernel averages of rocprofv3 --pmc CSVs (counter_collection.csv
files under the given directories), kernels matched by a name substring."""
import collections
import csv
import glob
import sys

pat = sys.argv[1]
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            if any(p in r["Kernel_Name"] for p in pat.split(",")):
                agg[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, dd in agg.items():
            print(d, k, {c: round(sum(v) / len(v)) for c, v in sorted(dd.items())})
