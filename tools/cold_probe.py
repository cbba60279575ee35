#!/usr/bin/env python3
"""Developer tool: cold-key latency-lane batches (key cache off: the octet
kernel), the bench's SCP set at several sizes, timed at the C-ABI call as the
bench's latency_1k_cold_keys block does.  One JSON line: p50 / p99 ms per size
and whether every verdict matched libsodium.  Run once per library / setting
(SV_OCT_HI_MAX) and interleave the runs for an A/B.

  python tools/cold_probe.py [iters] [sizes,comma,separated]"""
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
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    sizes = tuple(int(x) for x in sys.argv[2].split(",")) if len(sys.argv) > 2 else (1000, 2048, 4096)
    sv = importlib.import_module("stellar-core_amd")
    sodium = bench.load_libsodium()
    clib = sv.load_library()
    sv.set_key_cache(0)
    res = {"iters": iters, "lib": os.environ.get("SV_PROBE_LIB_NAME", "tree"),
           "oct_hi_max": os.environ.get("SV_OCT_HI_MAX", "default"), "sizes": {}}
    for n in sizes:
        pks, sigs, lmsgs, expect = bench.scp_latency_set(sodium, n=n, seed=4242 + n)
        pk_a = np.ascontiguousarray(np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 32))
        sg_a = np.ascontiguousarray(np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 64))
        m_len = np.array([len(m) for m in lmsgs], np.uint32)
        m_off = np.zeros(n, np.uint64)
        m_off[1:] = np.cumsum(m_len[:-1], dtype=np.uint64)
        m_buf = np.frombuffer(b"".join(lmsgs), np.uint8)
        out = np.zeros(n, np.uint8)
        args = [ctypes.c_void_p(a.ctypes.data) for a in (pk_a, sg_a, m_buf, m_off, m_len)]
        c_out = ctypes.c_void_p(out.ctypes.data)
        opts = ctypes.byref(sv.sv_opts(ctypes.sizeof(sv.sv_opts), 0, 0, 0))
        lat = []
        ok = True
        for it in range(iters + 20):
            t = time.perf_counter()
            rc = clib.sv_ed25519_verify_batch(args[0], args[1], args[2], args[3], args[4], ctypes.c_size_t(n), c_out,
                                              opts)
            dt = (time.perf_counter() - t) * 1e3
            assert rc == 0, rc
            ok = ok and bool(np.array_equal(out, expect))
            if it >= 20:
                lat.append(dt)
        res["sizes"][str(n)] = {"p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
                                "verdicts_match_libsodium": ok}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
