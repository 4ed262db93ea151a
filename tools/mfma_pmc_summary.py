#!/usr/bin/env python3
"""Summarise the matrix-core PMC passes of ``tools/profile_round.sh`` (split-bf16 compress GEMMs at the
configs[3] layer shape, the edge encoder at the headline shape) into profiles/<round>_matrix_core_pmc.json.

    python tools/mfma_pmc_summary.py gpurun_out/prof_r04 r04

SQ_VALU_MFMA_BUSY_CYCLES = 32 x the v_mfma_f32_32x32x16_bf16 issued, 16 x the v_mfma_f32_16x16x32_bf16
(the same count for the same products on either shape: 402653184 for both forms of each configs[3]
GEMM in round 4's passes); normalised by 1024 SIMDs x the
profiled duration at the 2.4 GHz peak clock, and at the clock the pass ran at (SQ_BUSY_CYCLES over 32
shader engines x the duration).  The first dispatch of each pass is dropped (cold caches, clock ramp)."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WHAT = {
    "gemm_fwd": "split-bf16 compress forward, configs[3] layer shape (64 nodes, C=2048, 8x8): M=2048 N=4096 K=4096",
    "gemm_dgrad": "split-bf16 compress data gradient, same shape: M=4096 N=4096 K=2048",
    "gemm_wgrad": "split-bf16 compress weight gradient, same shape: M=2048 N=4096 K=4096, the default form at "
                  "C >= 1024: dy split once (split_rows, not counted) + gemm_nt_psa",
    "gemm_wgrad3": "split-bf16 compress weight gradient, same shape, both operands split in the kernel "
                   "(gemm_nt_split_w4_mf16, the round-4 default)",
    "encoder": "split-bf16 edge encoder forward (shared-hidden form), headline shape E=1792 C=512",
}


def load(path, regex):
    per = collections.defaultdict(dict)
    span = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if regex not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] = float(r["Counter_Value"])
            span[d] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
    return per, span


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    out = {"round": rnd, "method": __doc__.split("\n\n", 2)[2].strip(), "records": {}}
    for name, regex in (("gemm_fwd", "gemm_n"), ("gemm_dgrad", "gemm_n"), ("gemm_wgrad", "gemm_n"),
                        ("gemm_wgrad3", "gemm_n"), ("encoder", "encoder")):
        path = os.path.join(src, "pmc_" + name, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        per, span = load(path, regex)
        ids = sorted(per)[1:] or sorted(per)
        if name.startswith("gemm_wgrad"):  # the split-K sum kernel does not match "gemm_n"; only the product
            ids = [d for d in ids if "gemm_nt" in span[d][2]] or ids
        n = len(ids)
        c = {k: sum(per[d].get(k, 0.0) for d in ids) / n for k in per[ids[0]]}
        dur = sum((span[d][1] - span[d][0]) for d in ids) / n / 1e3  # us
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        clock = c.get("SQ_BUSY_CYCLES", 0.0) / 32 / (dur * 1e-6) if dur > 0 else 0.0
        rec = {
            "what": WHAT[name],
            "kernel": span[ids[0]][2],
            "dispatches_averaged": n,
            "avg_duration_us_profiled": dur,
            "clock_ghz_from_sq_busy": clock / 1e9,
            "mfma_busy_over_1024_simds_x_duration_at_2p4GHz": busy / (1024 * dur * 1e-6 * 2.4e9) if dur else None,
            "mfma_busy_over_1024_simds_x_duration_at_run_clock": busy / (1024 * dur * 1e-6 * clock) if clock else None,
            "wait_any_over_wave_cycles": c.get("SQ_WAIT_ANY", 0.0) / max(c.get("SQ_WAVE_CYCLES", 1.0), 1.0),
            "valu_inst_over_wave_cycles": c.get("SQ_ACTIVE_INST_VALU", 0.0) / max(c.get("SQ_WAVE_CYCLES", 1.0), 1.0),
            "counters": c,
        }
        out["records"][name] = rec
        print(f"{name:10s} {rec['kernel'][:40]:40s} {dur:8.1f} us  clock {clock / 1e9:4.2f} GHz  "
              f"MFMA busy {rec['mfma_busy_over_1024_simds_x_duration_at_2p4GHz']:.3f} @2.4 GHz, "
              f"{rec['mfma_busy_over_1024_simds_x_duration_at_run_clock'] or 0:.3f} @run clock")
    with open(os.path.join(ROOT, "profiles", f"{rnd}_matrix_core_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
