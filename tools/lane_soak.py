#!/usr/bin/env python3
"""Developer tool: soak of the latency lane with its image read in place.
Cycles 8 different libsodium-signed SCP-shaped sets (bench.scp_latency_set,
distinct seeds and sizes) in a random order through sv_ed25519_verify_batch,
warm and cold, and checks every batch's verdicts: a kernel that read a stale
image (an earlier batch's bytes) would give another set's verdicts.
Usage: python tools/lane_soak.py [iterations]"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: F401,E402
import bench  # noqa: E402
from ab_lat_capi import Opts  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    sodium = bench.load_libsodium()
    assert sodium is not None
    sets = []
    for k, n in enumerate([1000, 1000, 999, 640, 1500, 333, 2048, 1000]):
        pks, sigs, msgs, expect = bench.scp_latency_set(sodium, n=n, seed=1000 + k)
        arrs = (np.ascontiguousarray(np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 32)),
                np.ascontiguousarray(np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 64)),
                np.frombuffer(b"".join(msgs), np.uint8), None, None)
        ln = np.array([len(m) for m in msgs], np.uint32)
        off = np.zeros(len(msgs), np.uint64)
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
        arrs = (arrs[0], arrs[1], arrs[2], off, ln)
        sets.append((arrs, [ctypes.c_void_p(a.ctypes.data) for a in arrs], expect))
    lib = ctypes.CDLL(os.path.join(REPO, "stellar-core_amd", "libstellar_sigverify.so"))
    lib.sv_set_key_cache.argtypes = [ctypes.c_size_t]
    assert lib.sv_init() == 0
    opts = ctypes.byref(Opts(ctypes.sizeof(Opts), 0, 0, 0))
    rng = np.random.default_rng(7)
    bad = 0
    t0 = time.perf_counter()
    for mode in ("warm", "cold"):
        assert lib.sv_set_key_cache(1024 if mode == "warm" else 0) == 0
        for it in range(iters // 2):
            _, args, expect = sets[int(rng.integers(0, len(sets)))]
            out = np.zeros(len(expect), np.uint8)
            assert lib.sv_ed25519_verify_batch(*args, ctypes.c_size_t(len(expect)), ctypes.c_void_p(out.ctypes.data),
                                               opts) == 0
            if not np.array_equal(out, expect):
                bad += 1
            if it % 5000 == 0:
                print("%s %d batches, %d with wrong verdicts, %.1f s" % (mode, it, bad, time.perf_counter() - t0),
                      flush=True)
    print("done: %d batches over %d sets, %d with wrong verdicts" % (iters, len(sets), bad), flush=True)
    assert bad == 0


if __name__ == "__main__":
    main()
