#!/usr/bin/env python3
"""Summarise a ``tools/profile_round.sh`` output directory into committed profiles/ files.

    python tools/pmc_summary.py gpurun_out/prof_r04 r04

Writes
  profiles/<round>_bench_kernel_stats.csv  rocprofv3 --stats of the headline bench command
  profiles/<round>_kernel_stats.csv        rocprofv3 --stats of tools/prof_kernels.py (all configs)
  profiles/pmc_<round>.json                per (config shape, kernel): trace duration, HBM bytes per
                                           launch (FETCH_SIZE doubled + WRITE_SIZE, MI355X_MICROARCH.md
                                           §HBM), algorithmic bytes, and SQ counters per launch
  profiles/pmc_traffic_<round>.json        the headline kernel's record in bench.py's lookup format

tools/prof_kernels.py runs, per shape in SHAPES order, `iters` forward then `iters` backward launches;
dispatches of our kernels are assigned to shapes by that order.
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
SHAPES = [("north_star", (32, 8, 512, 32, None)), ("cfg1", (16, 8, 512, 32, None)), ("cfg2", (32, 8, 1280, 8, None)),
          ("cfg3", (8, 8, 2048, 8, None)), ("cfg4", (8, 16, 1024, 16, 4))]
WORKLOAD = "gcn_film_mean_fwd_B32_N8_complete_C512_32x32_fp32"


def alg_bytes(shape, kind):
    B, N, C, H, knn = shape
    Nt = B * N
    E = B * N * (knn if knn else N - 1)
    plane = Nt * C * H * H * 4
    gb = E * 2 * C * 4
    return 2 * plane + gb if kind == "fwd" else 3 * plane + 2 * gb


def ours(name):
    return "film_" in name


def dispatch_shapes(rows, iters, key="Dispatch_Id"):
    """Dispatch id -> (shape, fwd|bwd), from the launch order of prof_kernels.py.  A backward may be
    one kernel or two (film_bwd_dx + film_bwd_fused); the forward is always one."""
    rows = sorted(rows, key=lambda r: int(r[key]))
    out = {}
    i = 0
    for sname, _ in SHAPES:
        fwd = rows[i:i + iters]
        for r in fwd:
            out[int(r[key])] = (sname, "fwd")
        i += iters
        # backward launches: every following dispatch up to the next shape's forward kernel name
        first_bwd = rows[i]["Kernel_Name"] if i < len(rows) else None
        per = 1
        if i + 1 < len(rows) and rows[i + 1]["Kernel_Name"] != first_bwd:
            per = 2
        for r in rows[i:i + per * iters]:
            out[int(r[key])] = (sname, "bwd")
        i += per * iters
    return out


def counters(path):
    """{dispatch id: {counter: value}} and {dispatch id: kernel name}."""
    vals, names = {}, {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        vals.setdefault(d, {})[r["Counter_Name"]] = float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    return vals, names


def main(src, rnd, iters=20, pmc_iters=5):
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(src, "bench", "run_kernel_stats.csv"), os.path.join(prof, f"{rnd}_bench_kernel_stats.csv"))
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{rnd}_kernel_stats.csv"))
    trace = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))) if ours(r["Kernel_Name"])]
    tmap = dispatch_shapes(trace, iters)
    recs = {}
    for r in trace:
        sname, kind = tmap[int(r["Dispatch_Id"])]
        rec = recs.setdefault((sname, kind, r["Kernel_Name"]), {"durations_us": [], "vgpr": r.get("VGPR_Count"),
                                                               "lds": r.get("LDS_Block_Size"),
                                                               "grid": r.get("Grid_Size_X")})
        rec["durations_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for group in ("FETCH", "WRITE", "SQ1", "SQ2", "GRBM"):
        path = os.path.join(src, f"pmc_{group}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        vals, names = counters(path)
        rows = [{"Dispatch_Id": d, "Kernel_Name": n} for d, n in names.items()]
        pmap = dispatch_shapes(rows, pmc_iters)
        for d, cv in vals.items():
            sname, kind = pmap[d]
            rec = recs.setdefault((sname, kind, names[d]), {"durations_us": []})
            for k, v in cv.items():
                rec.setdefault("pmc", {}).setdefault(k, []).append(v)
    out = []
    shapes = dict(SHAPES)
    for (sname, kind, kname), rec in sorted(recs.items()):
        pmc = {k: statistics.mean(v) for k, v in rec.get("pmc", {}).items()}
        d = {"shape": sname, "dims": dict(zip(("B", "N", "C", "HW", "knn"), shapes[sname])), "pass": kind,
             "kernel": kname, "dispatches_traced": len(rec["durations_us"]),
             "avg_duration_us_trace": statistics.mean(rec["durations_us"]) if rec["durations_us"] else None,
             "vgpr_count_trace": rec.get("vgpr"), "grid": rec.get("grid")}
        if kind == "fwd" or "bwd_fused" in kname or "bwd_regular" in kname or "bwd_mfma" in kname:
            d["alg_bytes_per_launch"] = alg_bytes(shapes[sname], kind)
        if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
            d["hbm_bytes_per_launch"] = (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024
            if d.get("alg_bytes_per_launch"):
                d["traffic_over_alg"] = d["hbm_bytes_per_launch"] / d["alg_bytes_per_launch"]
        if d["avg_duration_us_trace"] and d.get("alg_bytes_per_launch"):
            d["achieved_gbs"] = d["alg_bytes_per_launch"] / d["avg_duration_us_trace"] / 1e3
            d["frac_of_8tbs"] = d["achieved_gbs"] / 8000.0
        wc = pmc.get("SQ_WAVE_CYCLES")
        if wc:
            d["valu_issue_frac"] = pmc.get("SQ_ACTIVE_INST_VALU", 0) / wc
            d["lds_issue_frac"] = pmc.get("SQ_ACTIVE_INST_LDS", 0) / wc
            d["wait_frac"] = pmc.get("SQ_WAIT_ANY", 0) / wc
        if pmc.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_frac"] = pmc.get("SQ_LDS_BANK_CONFLICT", 0) / pmc["SQ_LDS_IDX_ACTIVE"]
        d["pmc_per_launch"] = pmc
        out.append(d)
    with open(os.path.join(prof, f"pmc_{rnd}.json"), "w") as f:
        json.dump({"round": rnd, "method": "rocprofv3 --kernel-trace (durations) and separate --pmc passes "
                   "(FETCH_SIZE doubled per MI355X_MICROARCH.md, WRITE_SIZE exact for 16 B/lane stores); "
                   "tools/prof_kernels.py on rotating buffers > 512 MB", "records": out}, f, indent=1)
    head = [d for d in out if d["shape"] == "north_star" and d["pass"] == "fwd"]
    if head and head[0].get("hbm_bytes_per_launch"):
        with open(os.path.join(prof, f"pmc_traffic_{rnd}.json"), "w") as f:
            json.dump({"round": rnd, "workload": WORKLOAD, "kernel": "film_fwd",
                       "hbm_bytes_per_launch": head[0]["hbm_bytes_per_launch"],
                       "avg_duration_us_trace": head[0]["avg_duration_us_trace"],
                       "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; FETCH_SIZE doubled "
                                 "(gfx950)"}, f, indent=1)
    for d in out:
        print(f"{d['shape']:10s} {d['pass']} {d['kernel'][:55]:55s} {d['avg_duration_us_trace'] or 0:8.1f} us "
              f"frac {d.get('frac_of_8tbs', 0):.3f} traffic/alg {d.get('traffic_over_alg', 0):.3f} "
              f"valu {d.get('valu_issue_frac', 0):.3f} wait {d.get('wait_frac', 0):.3f} "
              f"ldsconf {d.get('lds_bank_conflict_frac', 0):.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
