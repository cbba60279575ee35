#!/usr/bin/env python3
"""Developer tool: lines up tools/host_call_probe.py calls (its stderr, PROBE
lines) with a rocprofv3 kernel trace of the same run: per call, each kernel
and copy as [start..end] microseconds after the call began.
  python tools/host_call_timeline.py probe.err kt_kernel_trace.csv"""
import csv
import re
import sys


def main():
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0])
          for r in csv.DictReader(open(sys.argv[2]))]
    for line in open(sys.argv[1]):
        m = re.match(r"PROBE n=(\d+) start_ns=(\d+) ms=([\d.]+)", line)
        if not m:
            continue
        n, s, ms = int(m[1]), int(m[2]), float(m[3])
        e = s + ms * 1e6
        kk = [(a, b, nm) for a, b, nm in ks if a >= s and b <= e + 1e5]
        print(n, "%.3f" % ms, " ".join("%s[%.0f..%.0f]" % (nm[-16:], (a - s) / 1e3, (b - s) / 1e3) for a, b, nm in kk))


if __name__ == "__main__":
    main()
