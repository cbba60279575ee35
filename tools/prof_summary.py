#!/usr/bin/env python3
"""Summarise a rocprofv3 profile directory of bench.py runs (developer tool).

Reads <dir>/kt/*_kernel_stats.csv and every <dir>/*/*_counter_collection.csv,
averages each counter over the verify path's dispatches (split form: the
sv_prep_kernel<0> + sv_main_kernel pair, summed per verify launch; fused form:
sv_verify_lat_kernel<0>) and prints a
JSON summary with per-launch HBM traffic (FETCH_SIZE doubled per
MI355X_MICROARCH.md §HBM for 16-B streaming reads is NOT applied here: our
reads are 16-B per-lane gathers, so both the raw and the doubled value are
reported), VALU instruction counts per signature and issue efficiency.

Usage: python tools/prof_summary.py gpurun_out/prof2 [--batch 1048576]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    batch = 1 << 20
    if "--batch" in sys.argv:
        batch = int(sys.argv[sys.argv.index("--batch") + 1])
    out = {"profile_dir": d, "batch": batch}
    # (round 3: the kernels are instantiated with and without per-key tables,
    # sv_prep_kernel<0, false> / sv_main_kernel<false>; the headline runs without)
    pat = re.compile(r"sv_verify(_lat)?_kernel<0>|sv_prep_kernel<0(, false){0,2}>|sv_main_kernel(<false>)?\(")
    # the throughput path may cut one launch into several equal chunks
    # (sv_plan_chunk): chunk size = the prep kernel's grid (one lane per
    # signature), and a launch's value = per-dispatch value x chunks
    chunks = 1
    for f in glob.glob(os.path.join(d, "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if re.search(r"sv_prep_kernel<0(, false){0,2}>", r["Kernel_Name"]) and int(r["Grid_Size"]) >= 1024:
                chunks = max(1, batch // int(r["Grid_Size"]))
                break
        if chunks > 1:
            break
    out["chunks_per_launch"] = chunks
    ks = glob.glob(os.path.join(d, "kt", "*_kernel_stats.csv"))
    if ks:
        per = {}
        for r in csv.DictReader(open(ks[0])):
            if pat.search(r["Name"]):
                per[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                  "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
        if per:
            out["kernel"] = " + ".join(sorted(per))
            out["kernels"] = per
            out["calls"] = min(v["calls"] for v in per.values()) // chunks
            # one verify launch = `chunks` dispatches of each kernel of the path
            for k in ("avg_ns", "min_ns", "max_ns"):
                out[k] = chunks * sum(v[k] for v in per.values())
    # per kernel: counter -> list over dispatches; a launch's value = sum over the path's kernels
    vals = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(d, "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if not pat.search(r["Kernel_Name"]):
                continue
            if int(r["Grid_Size"]) < 1024:
                continue
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[r["Kernel_Name"]] = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size",
                                                        "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")}
    avg = defaultdict(float)
    per_kernel = {}
    for kn, cv in vals.items():
        per_kernel[kn] = {c: chunks * sum(v) / len(v) for c, v in cv.items()}
        for c, a in per_kernel[kn].items():
            avg[c] += a
    avg = dict(avg)
    out["dispatch"] = meta
    out["counters_avg_per_launch_by_kernel"] = per_kernel
    out["counters_avg_per_launch"] = avg
    if "FETCH_SIZE" in avg:
        out["fetch_bytes_per_launch_raw"] = avg["FETCH_SIZE"] * 1024
        out["fetch_bytes_per_launch_x2"] = avg["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in avg:
        out["write_bytes_per_launch"] = avg["WRITE_SIZE"] * 1024
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        out["hbm_bytes_per_launch"] = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        out["hbm_bytes_per_verify"] = out["hbm_bytes_per_launch"] / batch
        out["algorithmic_bytes_per_verify"] = 32 + 64 + 32 + 1
    if "SQ_INSTS_VALU" in avg:
        # SQ_INSTS_* count wave-instructions
        out["valu_inst_per_verify"] = avg["SQ_INSTS_VALU"] * 64 / batch
        for k in ("SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS",
                  "SQ_INSTS_SMEM"):
            if k in avg:
                out[k.lower() + "_per_verify"] = avg[k] * 64 / batch
    if "avg_ns" in out and "SQ_INSTS_VALU" in avg:
        t = out["avg_ns"] * 1e-9
        out["valu_lane_inst_per_s"] = avg["SQ_INSTS_VALU"] * 64 / t
    if "GRBM_GUI_ACTIVE" in avg and "avg_ns" in out:
        out["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / (out["avg_ns"])
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
        out["valu_active_frac_of_wave_cycles"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
    if "SQ_BUSY_CYCLES" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        out["note"] = "SQ_* cycle counters are in quad-cycles (MI355X_MICROARCH.md)"
    if "SQ_INSTS_VALU" in avg and "avg_ns" in out:
        # each wave64 VALU instruction occupies its SIMD for 4 cycles (1024 SIMDs)
        ghz = out.get("effective_clock_ghz", 2.4)
        out["valu_issue_util"] = avg["SQ_INSTS_VALU"] * 4 / (1024 * out["avg_ns"] * ghz)
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        out["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import importlib
    os.environ.setdefault("SV_NO_TORCH", "1")
    out["kernel_source_sha256"] = importlib.import_module("stellar-core_amd").kernel_source_digest()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
