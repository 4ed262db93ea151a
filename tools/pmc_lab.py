#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV directories of one kernel (lab tool, not product code): per kernel
name matching a substring, the median over dispatches of each counter, plus derived figures —
effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), MFMA-busy fraction of the 1024 SIMDs at that
clock and at 2.4 GHz, and the SQ wait shares (SQ_* wave counters are quad-cycles).

    python tools/pmc_lab.py <kernel substring> <dir> [<dir> ...]"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def load(dirs, sub):
    per = defaultdict(lambda: defaultdict(list))  # dispatch -> counter -> values
    dur = {}
    for d in dirs:
        with open(f"{d}/p_counter_collection.csv") as f:
            for r in csv.DictReader(f):
                if sub not in r["Kernel_Name"]:
                    continue
                key = (d, int(r["Dispatch_Id"]))
                per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return per, dur


def main():
    sub, dirs = sys.argv[1], sys.argv[2:]
    per, dur = load(dirs, sub)
    byname = defaultdict(list)
    for key, cs in per.items():
        for name, vals in cs.items():
            byname[name].append(sum(vals))
    med = {k: statistics.median(v) for k, v in byname.items()}
    t = statistics.median(dur.values())
    out = {"kernel": sub, "dispatches": len(per), "duration_us": t * 1e6, "counters": med}
    if "GRBM_GUI_ACTIVE" in med:
        clk = med["GRBM_GUI_ACTIVE"] / 8 / t
        out["clock_ghz"] = clk / 1e9
        if "SQ_VALU_MFMA_BUSY_CYCLES" in med:
            busy = med["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024
            out["mfma_busy_at_clock"] = busy / (clk * t)
            out["mfma_busy_at_2p4GHz"] = busy / (2.4e9 * t)
    if "SQ_WAVE_CYCLES" in med:
        wc = med["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in med:
                out[k.lower() + "_frac"] = med[k] / wc
    if "SQ_LDS_BANK_CONFLICT" in med and "SQ_LDS_IDX_ACTIVE" in med:
        out["lds_conflict_frac"] = med["SQ_LDS_BANK_CONFLICT"] / max(med["SQ_LDS_IDX_ACTIVE"], 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
