#!/usr/bin/env python3
"""Developer tool: latency-path verdicts of one library build against the golden
fixtures under every debug mode.  Usage: python tools/diag_lat.py [lib.so]"""
import os
os.environ.setdefault("SV_TEST_KNOBS", "1")  # (sv_set_debug_flags PREP_ONLY / FAIL)
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: F401,E402

sv = importlib.import_module("stellar-core_amd")
if len(sys.argv) > 1:
    sv.load_library(sys.argv[1])
modes = {"normal": 0, "trivial": sv.DBG_TRIVIAL_PAIR, "maxw": sv.DBG_MAX_WINDOWS,
         "both": sv.DBG_TRIVIAL_PAIR | sv.DBG_MAX_WINDOWS}
for mname, f in modes.items():
    sv.set_debug_flags(f)
    for name in ("intree", "adversarial", "lattice_edge", "msglen"):
        d = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))
        for path in ("latency", "throughput"):
            out = sv.verify_batch(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"], device=0, path=path)
            bad = np.nonzero(out != d["verdict"])[0]
            print("%-8s %-13s %-10s rows %5d bad %3d %s" % (mname, name, path, len(out), len(bad), list(bad[:8])),
                  flush=True)
sv.set_debug_flags(0)
