#!/usr/bin/env python3
"""Turn a ``tools/profile_round.sh`` output directory into the committed profile summaries.

    python tools/pmc_traffic.py gpurun_out/prof_r01 r01

Writes
  profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<round>_kernel_trace_film.csv  per-dispatch rows of our kernels (trimmed trace)
  profiles/pmc_traffic_<round>.json   per-launch HBM bytes of the aggregation kernels

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE (KiB) come from separate
PMC passes; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming read, so it
is doubled; WRITE_SIZE is exact for 16 B/lane stores.  bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import csv
import json
import os
import re
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return out


def main(src, rnd):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{rnd}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))
    film = [r for r in rows if "film_" in r["Kernel_Name"]]
    with open(os.path.join(prof, f"{rnd}_kernel_trace_film.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(film)
    durs = {}
    for r in film:
        durs.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    fetch = per_kernel(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    log = open(os.path.join(src, "bench_trace.log")).read()
    m = re.search(r'"workload": "([^"]+)"', log)
    workload = m.group(1) if m else None
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        fk = statistics.mean(fetch.get(name, [0.0]))
        wk = statistics.mean(write.get(name, [0.0]))
        kernels[name] = {
            "fetch_size_kib_raw": fk, "write_size_kib": wk,
            "hbm_read_bytes": 2 * fk * 1024, "hbm_write_bytes": wk * 1024,
            "hbm_bytes_per_launch": (2 * fk + wk) * 1024,
            "avg_duration_us_trace": statistics.mean(durs[name]) if name in durs else None,
            "dispatches": len(fetch.get(name, [])),
        }
    fwd = [k for k in kernels if "film_fwd" in k]
    summary = {
        "round": rnd, "workload": workload, "kernel": "film_fwd",
        "hbm_bytes_per_launch": kernels[fwd[0]]["hbm_bytes_per_launch"] if fwd else None,
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; FETCH_SIZE doubled (gfx950)",
        "kernels": kernels,
    }
    with open(os.path.join(prof, f"pmc_traffic_{rnd}.json"), "w") as f:
        json.dump(summary, f, indent=2)
    print(json.dumps(summary, indent=2))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
