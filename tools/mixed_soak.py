#!/usr/bin/env python3
"""Developer tool: mixed-workload soak of every entry point at once.

Threads run for SECONDS, each checking every verdict it gets:
  bulk      host-API batches of random size (20k..300k: quad, one-lane, the
            multi-chunk staging pipeline), fixed 32-byte messages
  lane      latency-lane batches (1..4096) over 100 validator keys (warm comb
            kernel) and over fresh keys (cold octet kernel), variable lengths
  keyed     sv_ed25519_verify_batch_keyed: verdicts and BLAKE2b-256 cache keys
            (checked against hashlib)
  device    sv_ed25519_verify_device on its own torch stream, with the bitmap
  cpu       the engine's CPU path on small batches
  txset     the C++ mirror's tx-set check with the pipelined pre-pass
            (svh_check_txset use_prefetch 4), outcomes against the same
            set's one-batch outcomes taken before the soak
  scp       the SCP harness (svh_scp_run: micro-batcher, batched main-thread
            post, main-thread verifySig), verdicts and cache hits
Rows come from the engine's GPU signer (valid) with one random bit flipped in
R, S, A or the message on a random third of them (rejected), so the expected
verdicts are known without libsodium.  Prints one JSON line: per-thread call
and signature counts, mismatches (must be 0) and errors.
Usage: python tools/mixed_soak.py [SECONDS]
"""
import hashlib
import importlib
import json
import os
import struct
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402  (one HIP runtime, shared with the engine)

sv = importlib.import_module("stellar-core_amd")

POOL = 1 << 19


def signed_pool(dev, n, base):
    s, m = bytearray(), bytearray()
    for i in range(base, base + n):
        p = struct.pack("<Q", i)
        s += hashlib.sha256(b"SOAKSEED" + p).digest()
        m += hashlib.sha256(b"SOAKMSG" + p).digest()
    ts = torch.from_numpy(np.frombuffer(bytes(s), np.uint8).reshape(n, 32).copy()).to(dev)
    tm = torch.from_numpy(np.frombuffer(bytes(m), np.uint8).reshape(n, 32).copy()).to(dev)
    tpk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    tsig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    sv.sign_device(0, ts.data_ptr(), tm.data_ptr(), n, tpk.data_ptr(), tsig.data_ptr(),
                   torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    return tpk.cpu().numpy(), tsig.cpu().numpy(), tm.cpu().numpy()


def corrupt(rng, pk, sig, msg, keys_too=True):
    """Copies with a random bit flipped in R, S, A or the message on ~1/3 of rows
    (keys_too=False: never A, so a validator batch keeps its known keys)."""
    pk, sig, msg = pk.copy(), sig.copy(), msg.copy()
    n = pk.shape[0]
    bad = rng.random(n) < 1 / 3
    rows = np.nonzero(bad)[0]
    where = rng.integers(0, 4, len(rows))
    if not keys_too:
        where[where == 2] = 3
    bit = (1 << rng.integers(0, 8, len(rows))).astype(np.uint8)
    for r, w, b in zip(rows, where, bit):
        if w == 0:
            sig[r, rng.integers(0, 32)] ^= b
        elif w == 1:
            sig[r, 32 + rng.integers(0, 31)] ^= b
        elif w == 2:
            pk[r, rng.integers(0, 32)] ^= b
        else:
            msg[r, rng.integers(0, 32)] ^= b
    return pk, sig, msg, (~bad).astype(np.uint8)


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    dev = torch.device("cuda", 0)
    pk, sig, msg = signed_pool(dev, POOL, 0)
    # 100 validator keys x 64 messages for the warm lane (keys repeat)
    vs, vm = bytearray(), bytearray()
    for i in range(6400):
        vs += hashlib.sha256(b"SOAKVAL" + struct.pack("<Q", i // 64)).digest()
        vm += hashlib.sha256(b"SOAKVMSG" + struct.pack("<Q", i)).digest()
    ts = torch.from_numpy(np.frombuffer(bytes(vs), np.uint8).reshape(-1, 32).copy()).to(dev)
    tm = torch.from_numpy(np.frombuffer(bytes(vm), np.uint8).reshape(-1, 32).copy()).to(dev)
    vpk_t = torch.empty((6400, 32), dtype=torch.uint8, device=dev)
    vsig_t = torch.empty((6400, 64), dtype=torch.uint8, device=dev)
    sv.sign_device(0, ts.data_ptr(), tm.data_ptr(), 6400, vpk_t.data_ptr(), vsig_t.data_ptr(),
                   torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    vpk, vsig, vmsg = vpk_t.cpu().numpy(), vsig_t.cpu().numpy(), tm.cpu().numpy()

    stop = time.time() + seconds
    stats = {}
    lock = threading.Lock()

    def record(name, calls, sigs, bad, err=None):
        with lock:
            s = stats.setdefault(name, {"calls": 0, "signatures": 0, "mismatches": 0, "errors": []})
            s["calls"] += calls
            s["signatures"] += sigs
            s["mismatches"] += bad
            if err and len(s["errors"]) < 5:
                s["errors"].append(err)

    def pick(rng, n):
        lo = int(rng.integers(0, POOL - n + 1))
        return corrupt(rng, pk[lo:lo + n], sig[lo:lo + n], msg[lo:lo + n])

    def bulk(seed):
        rng = np.random.default_rng(seed)
        while time.time() < stop:
            n = int(rng.integers(20_000, 300_000))
            p, s, m, want = pick(rng, n)
            try:
                got = sv.verify_fixed(p, s, m, 32, device=0)
                record("bulk", 1, n, int((got != want).sum()))
            except Exception as e:  # an error is reported, never counted as verdicts
                record("bulk", 1, 0, 0, repr(e))

    def lane(seed):
        rng = np.random.default_rng(seed)
        while time.time() < stop:
            n = int(rng.integers(1, 4097))
            if rng.random() < 0.75:  # validator keys (warm once their tables are built)
                rows = rng.integers(0, 6400, n)
                p, s, m, want = corrupt(rng, vpk[rows], vsig[rows], vmsg[rows], keys_too=False)
            else:
                p, s, m, want = pick(rng, n)
            off = np.arange(n, dtype=np.uint64) * 32
            try:
                got = sv.verify_batch(p, s, m.reshape(-1), off, np.full(n, 32, np.uint32), device=0,
                                      path="latency")
                record("lane", 1, n, int((got != want).sum()))
            except Exception as e:
                record("lane", 1, 0, 0, repr(e))

    def keyed(seed):
        rng = np.random.default_rng(seed)
        while time.time() < stop:
            n = int(rng.integers(256, 20_000))
            p, s, m, want = pick(rng, n)
            off = np.arange(n, dtype=np.uint64) * 32
            try:
                got, keys = sv.verify_batch_keyed(p, s, m.reshape(-1), off, np.full(n, 32, np.uint32), device=0)
                bad = int((got != want).sum())
                for i in rng.integers(0, n, 16):
                    k = hashlib.blake2b(p[i].tobytes() + s[i].tobytes() + m[i].tobytes(), digest_size=32).digest()
                    bad += k != keys[i].tobytes()
                record("keyed", 1, n, bad)
            except Exception as e:
                record("keyed", 1, 0, 0, repr(e))

    def device(seed):
        rng = np.random.default_rng(seed)
        st = torch.cuda.Stream(dev)
        while time.time() < stop:
            n = int(rng.integers(1, 200_000))
            p, s, m, want = pick(rng, n)
            with torch.cuda.stream(st):
                tp, tsg, tmm = (torch.from_numpy(x).to(dev, non_blocking=False) for x in (p, s, m))
                tv = torch.zeros(n, dtype=torch.uint8, device=dev)
                tb = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
            try:
                sv.verify_device(0, tp.data_ptr(), tsg.data_ptr(), tmm.data_ptr(), n, tv.data_ptr(), tb.data_ptr(),
                                 st.cuda_stream)
                st.synchronize()
                got = tv.cpu().numpy()
                bits = np.unpackbits(tb.cpu().numpy().view(np.uint8), bitorder="little")[:n]
                record("device", 1, n, int((got != want).sum()) + int((bits != want).sum()))
            except Exception as e:
                record("device", 1, 0, 0, repr(e))

    def cpu(seed):
        rng = np.random.default_rng(seed)
        while time.time() < stop:
            n = int(rng.integers(1, 64))
            p, s, m, want = pick(rng, n)
            got = sv.verify_batch_cpu(p, s, m.reshape(-1), np.arange(n, dtype=np.uint64) * 32,
                                      np.full(n, 32, np.uint32), threads=1)
            record("cpu", 1, n, int((got != want).sum()))

    # the host-integration workers (libstellar_host): a 3000-tx set and SCP-shaped bursts
    import ctypes
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import txset_gen as tg

    host = ctypes.CDLL(sv.HOSTLIB_PATH)
    host.svh_last_error_string.restype = ctypes.c_char_p
    host.svh_set_test_verifier.argtypes = [ctypes.c_void_p]
    host.svh_set_test_verifier(None)
    def sign_fn(reqs):  # the engine's RFC 8032 signer over the generator's (seed, message) requests
        n = len(reqs)
        ts = torch.from_numpy(np.frombuffer(b"".join(r[0] for r in reqs), np.uint8).reshape(n, 32).copy()).to(dev)
        tmm = torch.from_numpy(np.frombuffer(b"".join(r[1] for r in reqs), np.uint8).reshape(n, 32).copy()).to(dev)
        tp = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        tsg = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        sv.sign_device(0, ts.data_ptr(), tmm.data_ptr(), n, tp.data_ptr(), tsg.data_ptr(),
                       torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        a, b = tp.cpu().numpy(), tsg.cpu().numpy()
        return [(a[i].tobytes(), b[i].tobytes()) for i in range(n)]

    # (outcomes are compared with the same set's one-batch outcomes, taken before the soak)
    txs = tg.generate(3000, sign_fn, seed=31)
    T, S, G = tg.to_ctypes(txs)
    nt = len(txs)

    def check_txset(mode):
        ok = np.zeros(nt, np.uint8)
        used = np.zeros(nt, np.uint8)
        rc = host.svh_check_txset(T, ctypes.c_size_t(nt), S, G, mode, ok.ctypes.data_as(ctypes.c_void_p),
                                  used.ctypes.data_as(ctypes.c_void_p), None)
        if rc != 0:
            raise RuntimeError(host.svh_last_error_string())
        return ok, used

    want_ok, want_used = check_txset(1)

    def txset(seed):
        while time.time() < stop:
            try:
                ok, used = check_txset(4)
                record("txset", 1, nt, int((ok != want_ok).sum() + (used != want_used).sum()))
            except Exception as e:
                record("txset", 1, 0, 0, repr(e))

    class Prm(ctypes.Structure):
        _fields_ = [(k, ctypes.c_uint32) for k in ("struct_size", "producers", "burst", "interval_us", "max_batch",
                    "max_delay_us", "workers", "policy", "linger_us", "idle_in_flight", "quiet_us",
                    "max_linger_us", "batch_post")]

    def scp(seed):
        rng = np.random.default_rng(seed)
        res = (ctypes.c_char * 4096)()
        while time.time() < stop:
            n = 2000
            rows = rng.integers(0, 6400, n)
            p, s, m, want = corrupt(rng, vpk[rows], vsig[rows], vmsg[rows], keys_too=False)
            # distinct envelopes (a duplicate in flight in two batches reads as a miss, as for concurrent calls)
            _, first = np.unique(np.concatenate([p, s, m], axis=1), axis=0, return_index=True)
            first = np.sort(first)
            p, s, m, want = (np.ascontiguousarray(x[first]) for x in (p, s, m, want))
            n = len(first)
            off = np.arange(n, dtype=np.uint64) * 32
            ln = np.full(n, 32, np.uint32)
            out = np.full(n, 7, np.uint8)
            prm = Prm(ctypes.sizeof(Prm), 2, 500, 2000, 8192, 2000, 2, 0, 0, 1, 0, 200, 1)
            host.svh_cache_clear()
            P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
            rc = host.svh_scp_run(P(p), P(s), P(m.reshape(-1)), P(off), P(ln), ctypes.c_size_t(n), ctypes.byref(prm),
                                  P(out), res)
            if rc != 0:
                record("scp", 1, 0, 0, host.svh_last_error_string().decode())
                continue
            record("scp", 1, n, int((out != want).sum()))

    workers = [bulk, bulk, lane, lane, keyed, device, cpu, txset, scp]
    th = [threading.Thread(target=f, args=(100 + k,)) for k, f in enumerate(workers)]
    t0 = time.time()
    last = t0
    for t in th:
        t.start()
    while any(t.is_alive() for t in th):
        time.sleep(5)
        if time.time() - last > 50:  # progress for a watchdog that needs output
            last = time.time()
            with lock:
                print("progress %.0fs %s" % (last - t0, {k: v["calls"] for k, v in stats.items()}),
                      file=sys.stderr, flush=True)
    for t in th:
        t.join()
    out = {"seconds": time.time() - t0, "threads": [f.__name__ for f in workers], "per_kind": stats,
           "key_cache": sv.key_cache_stats(0),
           "ok": all(v["mismatches"] == 0 and not v["errors"] for v in stats.values())}
    print(json.dumps(out), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
