#!/usr/bin/env python3
"""Developer tool: config 4 through the integration path (svh_scp_run, the
bench's config4_integrated) over a grid of micro-batcher settings, one JSON
line per setting: submit -> batch verified (ready), -> continuation
(verdict) and -> main-thread verifySig latencies, batch counts.

  python tools/scp_probe.py [n] [settings]
    settings: "burst:interval:linger:inflight:workers:producers[:quiet:maxlinger],..." (quiet default 0: off)
With SV_HOST_TRACE=1 / SV_LAT_TRACE=1 in the environment the engine prints
its per-batch host stages to stderr."""
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401  (one HIP runtime)
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12000
    grid = sys.argv[2] if len(sys.argv) > 2 else "1000:5000:0:1:2:4,1000:5000:100:1:2:4,1000:5000:0:2:2:4"
    sv = importlib.import_module("stellar-core_amd")
    sodium = bench.load_libsodium()
    pk, sig, buf, off, lens, expect = bench.scp_envelope_set(sodium, n, seed=77)
    host = ctypes.CDLL(sv.HOSTLIB_PATH)
    host.svh_last_error_string.restype = ctypes.c_char_p
    host.svh_scp_run.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_void_p]
    for k, spec in enumerate(["1000:5000:0:1:2:4"] + grid.split(",")):
        v = [int(x) for x in spec.split(":")] + [0, 200][len(spec.split(":")) - 6:]
        burst, interval, linger, inflight, workers, producers, quiet, maxl = v[:8]
        p = bench.ScpParams(ctypes.sizeof(bench.ScpParams), producers, burst, interval, 8192, 2000, workers, 0, linger,
                            inflight, quiet, maxl)
        r = bench.ScpResult()
        out = np.full(n, 7, np.uint8)
        host.svh_cache_clear()
        t0 = time.perf_counter()
        rc = host.svh_scp_run(pk.ctypes.data, sig.ctypes.data, buf.ctypes.data, off.ctypes.data, lens.ctypes.data, n,
                              ctypes.byref(p), out.ctypes.data, ctypes.byref(r))
        assert rc == 0, host.svh_last_error_string()
        d = {f: getattr(r, f) for f, _ in bench.ScpResult._fields_}
        d.update({"spec": spec, "ok": bool((out == expect).all()), "wall": time.perf_counter() - t0})
        if k > 0:  # (the first is a warm-up)
            print(json.dumps(d), flush=True)
        if k == 0:
            sv.key_cache_wait(0)


if __name__ == "__main__":
    main()
