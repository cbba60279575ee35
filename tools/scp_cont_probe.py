#!/usr/bin/env python3
"""Developer tool (CPU, no GPU): what the continuations of a micro-batcher
batch cost in svh_scp_run (config 4's harness) -- submit -> continuation
(verdict) minus submit -> batch verified (ready) -- with a stand-in batch
verifier that accepts everything (svh_set_test_verifier), over random
distinct envelopes in paced bursts.  One JSON line per repeat.

  python tools/scp_cont_probe.py [n] [burst] [interval_us] [repeats]"""
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

VERIFY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12000
    burst = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    interval = int(sys.argv[3]) if len(sys.argv) > 3 else 5000
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    sv = importlib.import_module("stellar-core_amd")
    host = ctypes.CDLL(sv.HOSTLIB_PATH)
    host.svh_set_test_verifier.argtypes = [ctypes.c_void_p]
    host.svh_last_error_string.restype = ctypes.c_char_p

    def fn(pk, sig, msg, off, ln, k, out):
        ctypes.memset(out, 1, k)
        t = time.perf_counter() + 60e-6  # (about a warm lane call's GPU time)
        while time.perf_counter() < t:
            pass
        return 0

    cfn = VERIFY_FN(fn)
    host.svh_set_test_verifier(ctypes.cast(cfn, ctypes.c_void_p))
    rng = np.random.default_rng(5)
    pk = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    sig = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    ln = rng.integers(128, 385, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    msg = rng.integers(0, 256, int(ln.sum()), dtype=np.uint8)
    vp = ctypes.c_void_p
    for rep in range(reps):
        host.svh_cache_clear()
        out = np.zeros(n, np.uint8)
        p = bench.ScpParams(ctypes.sizeof(bench.ScpParams), 4, burst, interval, 8192, 2000, 2, 0, 0, 1, 0, 200)
        r = bench.ScpResult()
        rc = host.svh_scp_run(vp(pk.ctypes.data), vp(sig.ctypes.data), vp(msg.ctypes.data), vp(off.ctypes.data),
                              vp(ln.ctypes.data), ctypes.c_size_t(n), ctypes.byref(p), vp(out.ctypes.data),
                              ctypes.byref(r))
        assert rc == 0, host.svh_last_error_string()
        print(json.dumps({"rep": rep, "verdict_p50_us": r.verdict_p50_us, "ready_p50_us": r.ready_p50_us,
                          "gap_p50_us": r.verdict_p50_us - r.ready_p50_us, "verdict_p99_us": r.verdict_p99_us,
                          "main_p50_us": r.main_p50_us, "batches": r.batches, "mean_batch": r.mean_batch,
                          "hits": r.main_hits, "misses": r.main_misses}), flush=True)
    host.svh_set_test_verifier(None)


if __name__ == "__main__":
    main()
