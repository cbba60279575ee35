#!/usr/bin/env python3
"""Prints host_api_ms per size of tools/size_sweep.py JSON files side by side.
  python tools/sweep_ab.py [--path auto] file.json ..."""
import json
import sys

args = sys.argv[1:]
path = "auto"
if args and args[0] == "--path":
    path, args = args[1], args[2:]
for f in args:
    d = json.load(open(f))
    rows = d["paths"][path]
    print(f.split("/")[-1], " ".join("%s:%.3f%s" % (n, r["host_api_ms"], "" if r["verdicts_ok"] else "!BAD")
                                     for n, r in rows.items()))
