"""Latency-path probe (developer tool): p50 host-API latency and kernel time
of SCP-shaped batches (100 validator keys, 128-384 B messages) at several
sizes, warm key cache (comb kernel) and cold (octet kernel).

    python tools/lat_probe.py [--sizes 1000,2048,4096] [--iters 50] [--out file.json]

Kernel time: HIP events around each launch on the latency lane's stream
(sv_timing_enable).  Signing uses the build's oracle restatement (no
libsodium needed on the GPU box).
"""
import argparse
import ctypes
import hashlib
import importlib
import json
import os
import struct
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def scp_set(n, seed=5):
    o = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    o.oracle_ed25519_seed_keypair.argtypes = [ctypes.c_char_p] * 3
    o.oracle_ed25519_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    keys = []
    for v in range(100):
        pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
        o.oracle_ed25519_seed_keypair(pk, sk, hashlib.sha256(b"SVVAL" + struct.pack("<Q", v)).digest())
        keys.append((pk.raw, sk.raw))
    rng = np.random.default_rng(seed)
    pks, sigs, msgs = [], [], []
    for i in range(n):
        pk, sk = keys[i % 100]
        m = rng.integers(0, 256, int(rng.integers(128, 385)), dtype=np.uint8).tobytes()
        s = ctypes.create_string_buffer(64)
        o.oracle_ed25519_sign(s, m, len(m), sk)
        pks.append(pk)
        sigs.append(s.raw)
        msgs.append(m)
    ln = np.array([len(m) for m in msgs], np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    return (np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 32), np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 64),
            np.frombuffer(b"".join(msgs), np.uint8), off, ln)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1000,2048,4096")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--out", default=None)
    ap.add_argument("--cold", type=int, default=1)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    sv = importlib.import_module("stellar-core_amd")
    rows = []
    for n in [int(x) for x in args.sizes.split(",")]:
        pk, sig, msg, off, ln = scp_set(n)
        for mode in (["warm", "cold"] if args.cold else ["warm"]):
            sv.set_key_cache(1024 if mode == "warm" else 0)
            for _ in range(3):
                out = sv.verify_batch(pk, sig, msg, off, ln, device=0)
            sv.key_cache_wait(0)
            for _ in range(3):
                out = sv.verify_batch(pk, sig, msg, off, ln, device=0)
            assert out.all(), "all rows are valid"
            st0 = sv.key_cache_stats(0)
            sv.kernel_time_reset()
            sv.timing_enable(True)
            lat = []
            for _ in range(args.iters):
                t = time.perf_counter()
                sv.verify_batch(pk, sig, msg, off, ln, device=0)
                lat.append((time.perf_counter() - t) * 1e3)
            sv.timing_enable(False)
            ms, la, _ = sv.kernel_time(0)
            st1 = sv.key_cache_stats(0)
            r = {"n": n, "mode": mode, "p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
                 "kernel_ms": ms / max(1, la), "warm_batches": st1["warm_batches"] - st0["warm_batches"],
                 "iters": args.iters}
            rows.append(r)
            print("n=%6d %-4s p50 %.3f ms p99 %.3f ms kernel %.3f ms (warm %d/%d)" % (
                n, mode, r["p50_ms"], r["p99_ms"], r["kernel_ms"], r["warm_batches"], args.iters), flush=True)
    sv.set_key_cache(1024)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
