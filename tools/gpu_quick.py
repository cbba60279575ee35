#!/usr/bin/env python3
"""First-light GPU check (developer tool): fixtures through the host API,
GPU signer vs the libsodium-generated valid set, and a 1M timing probe."""
import hashlib
import importlib
import os
import struct
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SV_NO_TORCH", "1")
sv = importlib.import_module("stellar-core_amd")

print("version", sv.version(), "devices", sv.device_count(), flush=True)
G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
for name in ["intree", "valid", "msglen", "adversarial"]:
    d = np.load(os.path.join(G, name + ".npz"))
    t = time.time()
    out = sv.verify_batch(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"])
    dt = time.time() - t
    bad = np.nonzero(out != d["verdict"])[0]
    print("%-12s n=%5d mismatches=%d  %.3fs" % (name, len(out), len(bad), dt), flush=True)
    if len(bad):
        print("   first bad", [(int(i), str(d["class_names"][d["cls"][i]]), int(d["verdict"][i])) for i in bad[:10]])

# fixed path on the valid set
d = np.load(os.path.join(G, "valid.npz"))
sel = d["msg_len"] == 32
msgs = np.stack([d["msg"][o:o + 32] for o in d["msg_off"][sel]])
out = sv.verify_fixed(d["pk"][sel], d["sig"][sel], msgs)
print("fixed32 valid all ok:", bool(out.all()), flush=True)

# 1M timing with host API (data replicated from the valid set)
n = 1 << 20
reps = n // int(sel.sum()) + 1
pk = np.tile(d["pk"][sel], (reps, 1))[:n]
sig = np.tile(d["sig"][sel], (reps, 1))[:n]
mm = np.tile(msgs, (reps, 1))[:n]
sv.verify_fixed(pk[:65536], sig[:65536], mm[:65536])
sv.timing_enable(True)
t = time.time()
out = sv.verify_fixed(pk, sig, mm)
dt = time.time() - t
ms, la, sg = sv.kernel_time(0)
print("1M fixed: all ok=%s wall=%.3fs -> %.3e verifies/s ; kernel %.2f ms -> %.3e verifies/s" % (
    bool(out.all()), dt, n / dt, ms, n / (ms * 1e-3)), flush=True)
