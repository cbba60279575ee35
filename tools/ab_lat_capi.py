#!/usr/bin/env python3
"""Developer tool: interleaved A/B of the 1k-batch latency through the C-ABI
(sv_ed25519_verify_batch, as bench.py's latency_1k) for whole-library
variants.  Usage: python tools/ab_lat_capi.py libA.so libB.so [...]

Every library gets the same libsodium-signed SCP-sized set (bench.py
scp_latency_set: 100 validators, 128-384 B messages, 10 % adversarial); warm
= key cache on (the comb kernel after the first batch), cold = key cache off
(the octet kernel).  Rounds alternate between the libraries; reports the
median over rounds of each round's p50 and the per-library verdict check.
AB_SIZES=1000,4096,...: the same SCP shape at other batch sizes."""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: F401,E402  (torch's HIP runtime first)
import bench  # noqa: E402

ROUNDS = int(os.environ.get("AB_ROUNDS", "8"))
ITERS = int(os.environ.get("AB_ITERS", "300"))
MODES = os.environ.get("AB_MODES", "warm,cold").split(",")
SIZES = [int(x) for x in os.environ.get("AB_SIZES", "1000").split(",")]


class Opts(ctypes.Structure):  # (sv_opts, include/stellar_sigverify.h)
    _fields_ = [("struct_size", ctypes.c_uint32), ("device", ctypes.c_int32), ("max_devices", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


def main():
    paths = sys.argv[1:]
    sodium = bench.load_libsodium()
    assert sodium is not None, "libsodium needed for the SCP set"
    sets = {}
    for size in SIZES:
        pks, sigs, lmsgs, expect = bench.scp_latency_set(sodium, n=size)
        pk_a = np.ascontiguousarray(np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 32))
        sg_a = np.ascontiguousarray(np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 64))
        m_len = np.array([len(m) for m in lmsgs], np.uint32)
        m_off = np.zeros(len(lmsgs), np.uint64)
        m_off[1:] = np.cumsum(m_len[:-1], dtype=np.uint64)
        m_buf = np.frombuffer(b"".join(lmsgs), np.uint8)
        arrs = (pk_a, sg_a, m_buf, m_off, m_len)
        sets[size] = (arrs, [ctypes.c_void_p(a.ctypes.data) for a in arrs], expect)
    libs = {}
    for p in paths:
        lib = ctypes.CDLL(p, mode=os.RTLD_LOCAL)
        lib.sv_set_key_cache.argtypes = [ctypes.c_size_t]
        assert lib.sv_init() == 0
        libs[os.path.basename(p)] = lib
    opts = ctypes.byref(Opts(ctypes.sizeof(Opts), 0, 0, 0))
    keys = ["%s%s" % (m, "" if len(SIZES) == 1 else "@%d" % z) for z in SIZES for m in MODES]
    res = {k: {c: [] for c in keys} for k in libs}
    for rnd in range(ROUNDS):
        for name, lib in libs.items():
            for size in SIZES:
                _, args, expect = sets[size]
                n = len(expect)
                out = np.zeros(n, np.uint8)
                outp = ctypes.c_void_p(out.ctypes.data)
                for mode in MODES:
                    assert lib.sv_set_key_cache(1024 if mode == "warm" else 0) == 0
                    for it in range(20):  # (warm-up; the second sighting builds the keys)
                        assert lib.sv_ed25519_verify_batch(*args, ctypes.c_size_t(n), outp, opts) == 0
                        if it == 1:
                            assert lib.sv_key_cache_wait(0) == 0
                    lat = []
                    for _ in range(ITERS):
                        t0 = time.perf_counter()
                        rc = lib.sv_ed25519_verify_batch(*args, ctypes.c_size_t(n), outp, opts)
                        lat.append((time.perf_counter() - t0) * 1e3)
                        assert rc == 0
                    if "diag" not in name:  # (diagnostic builds: wrong verdicts by design)
                        assert np.array_equal(out, expect), "%s %s: verdicts differ from libsodium" % (name, mode)
                    k = "%s%s" % (mode, "" if len(SIZES) == 1 else "@%d" % size)
                    res[name][k].append(float(np.percentile(lat, 50)))
        print("round %d: %s" % (rnd, "  ".join("%s %s" % (k, " ".join("%s %.4f" % (c, v[c][-1]) for c in keys))
                                                for k, v in res.items())), flush=True)
    for name, v in res.items():
        print("%-30s p50 %s  (median of %d rounds x %d iterations; %s)"
              % (name, "  ".join("%s %.4f ms" % (c, float(np.median(v[c]))) for c in keys), ROUNDS, ITERS,
                 "diagnostic build, verdicts not checked" if "diag" in name else "verdicts = libsodium"), flush=True)


if __name__ == "__main__":
    main()
