#!/usr/bin/env python3
"""Developer tool: single-signature latency of the engine's CPU path
(sv_ed25519_verify_cpu: what a single PubKeyUtils::verifySig miss runs) next
to libsodium 1.0.18 crypto_sign_verify_detached, same signatures, one thread."""
import ctypes
import importlib
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sv = importlib.import_module("stellar-core_amd")
lib = sv.load_library()
d = np.load(os.path.join(REPO, "tests", "golden", "valid.npz"))
n = min(400, len(d["verdict"]))
rows = [(d["pk"][i].tobytes(), d["sig"][i].tobytes(),
         d["msg"][int(d["msg_off"][i]):int(d["msg_off"][i]) + int(d["msg_len"][i])].tobytes()) for i in range(n)]
lib.sv_ed25519_verify_cpu.restype = ctypes.c_int
fns = [("engine CPU path", lambda p, s, m: lib.sv_ed25519_verify_cpu(p, s, m, ctypes.c_size_t(len(m))) == 1)]
for path in ("/opt/conda/lib/libsodium.so.23", "libsodium.so.23"):
    try:
        so = ctypes.CDLL(path)
        so.sodium_init()
        so.sodium_version_string.restype = ctypes.c_char_p
        fns.append(("libsodium " + so.sodium_version_string().decode(),
                    lambda p, s, m: so.crypto_sign_verify_detached(s, m, ctypes.c_ulonglong(len(m)), p) == 0))
        break
    except OSError:
        pass
for name, f in fns:
    assert all(f(*r) for r in rows[:50])
    best = 1e9
    for _ in range(5):
        t = time.perf_counter()
        for r in rows:
            f(*r)
        best = min(best, (time.perf_counter() - t) / n)
    print("%-18s %.1f us per verify (best of 5 passes over %d signatures, 1 thread)" % (name, best * 1e6, n))
