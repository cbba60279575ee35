#!/usr/bin/env python3
"""Copy a tools/profile_run.sh result into profiles/ (developer tool).

  python tools/save_profile.py gpurun_out/r1b/prof profiles/r01/<name>

Copies the kernel-stats and counter CSVs plus summary.json, and rewrites
profiles/<round>_traffic.json (the file bench.py reads roofline.traffic from,
keyed by the verify kernel's source digest) from the summary.
"""
import glob
import json
import os
import shutil
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "*", "*_kernel_stats.csv")) + \
            glob.glob(os.path.join(src, "*", "*_counter_collection.csv")):
        shutil.copy(f, os.path.join(dst, os.path.basename(f)))
    s = json.load(open(os.path.join(src, "summary.json")))
    s["profile_dir"] = dst
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(s, f, indent=1)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    t = {
        "batch": s["batch"],
        "hbm_bytes_per_launch": s["hbm_bytes_per_launch"],
        "fetch_size_raw_bytes": s["fetch_bytes_per_launch_raw"],
        "write_size_bytes": s["write_bytes_per_launch"],
        "kernel_avg_ns": s["avg_ns"],
        "valu_inst_per_verify": s["valu_inst_per_verify"],
        "valu_issue_util": s["valu_issue_util"],
        "l2_hit_rate": s["l2_hit_rate"],
        # the clock the chip held over the profiled kernels (GRBM_GUI_ACTIVE /
        # wall): bench.py's roofline.mad_issue_frac_at_profiled_clock
        "effective_clock_ghz": s.get("effective_clock_ghz"),
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes (tools/profile_run.sh), "
                  "%s/{fetch,write}_counter_collection.csv; FETCH_SIZE not doubled (per-lane 16-B gathers, "
                  "not a wide streaming read: MI355X_MICROARCH.md HBM note)" % os.path.relpath(dst, repo),
        "kernel": s["kernel"],
        "kernel_source_sha256": s["kernel_source_sha256"],
    }
    # profiles/<round>_traffic.json, the round taken from the destination
    # (profiles/r04/... -> r04); bench.py takes the newest one whose kernel
    # digest matches the sources it runs
    rnd = os.path.relpath(os.path.abspath(dst), os.path.join(repo, "profiles")).split(os.sep)[0]
    with open(os.path.join(repo, "profiles", "%s_traffic.json" % rnd), "w") as f:
        json.dump(t, f, indent=1)
    print(json.dumps(t, indent=1))


if __name__ == "__main__":
    main()
