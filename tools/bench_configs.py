#!/usr/bin/env python3
"""Secondary BASELINE.json configs on one MI355X (developer/report tool; the
headline line is bench.py = config 2).  Prints one JSON object.

  config1  100k random signatures over 32-byte hashes, and the reference's own
           benchmark shape (10k keys x 256-byte messages, SecretKey.cpp:182-234):
           GPU via the host API (PCIe-inclusive) and device API (kernel only),
           libsodium raw on 1 and all host threads, and the verifySig-equivalent
           path (C++ PubKeyUtils mirror: BLAKE2b key + cache + mutex) with
           libsodium behind it.
  config3  synthetic 5000-tx ledger, 1-20 ED25519 signers per tx (+ HASH_X,
           PRE_AUTH_TX, signed-payload signers, wrong-key colliding hints):
           C++ SignatureChecker mirror with the one-batch GPU pre-pass vs the
           same checker with per-signature libsodium (the reference's path);
           outcomes compared with an independent Python replay.
  configmb SCP/overlay flood through the VerifyMicroBatcher:
           8 producer threads submit 200k envelope-sized (~180 B) messages;
           GPU engine behind verifySigBatch vs libsodium behind it; throughput
           and submit->verdict latency p50/p99.
  config5  catchup scale: 64 x 2^20 signatures (the libsodium-pinned 1M set
           tiled 64x, cache bypassed) in one device-resident batch.
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
sys.path.insert(0, os.path.join(REPO, "tests"))

SODIUM = "/opt/conda/lib/libsodium.so.23"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def threads():
    return max(1, min(64, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)))


class Env:
    def __init__(self):
        import torch
        self.torch = torch
        self.sv = importlib.import_module("stellar-core_amd")
        self.dev = torch.device("cuda", 0)
        self.stream = torch.cuda.current_stream(self.dev).cuda_stream
        self.base = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
        self.base.cpubase_run.restype = ctypes.c_double
        self.base.cpubase_run.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_uint32, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        self.have_sodium = os.path.exists(SODIUM)
        self.sodium = ctypes.CDLL(SODIUM) if self.have_sodium else None
        if self.sodium is not None:
            assert self.sodium.sodium_init() >= 0
        self.host = ctypes.CDLL(self.sv.HOSTLIB_PATH)
        self.host.svh_last_error_string.restype = ctypes.c_char_p
        self.host.svh_set_test_verifier.argtypes = [ctypes.c_void_p]
        env_host_mb = self.host.svh_mb_run
        env_host_mb.restype = ctypes.c_int

    def gpu_sign(self, seeds, msgs):
        t = self.torch
        n = seeds.shape[0]
        ts = t.from_numpy(np.array(seeds, copy=True)).to(self.dev)
        tm = t.from_numpy(np.array(msgs, copy=True)).to(self.dev)
        pk = t.empty((n, 32), dtype=t.uint8, device=self.dev)
        sg = t.empty((n, 64), dtype=t.uint8, device=self.dev)
        self.sv.sign_device(0, ts.data_ptr(), tm.data_ptr(), n, pk.data_ptr(), sg.data_ptr(), self.stream)
        t.cuda.synchronize(self.dev)
        return pk, sg, tm

    def sodium_sign(self, seed, msg):
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        self.sodium.crypto_sign_seed_keypair(pk, sk, seed)
        s = ctypes.create_string_buffer(64)
        self.sodium.crypto_sign_detached(s, None, msg, ctypes.c_ulonglong(len(msg)), sk)
        return pk.raw, s.raw

    def cpu_rate(self, pk, sig, msg, mlen, nthreads):
        n = pk.shape[0]
        out = np.zeros(n, np.uint8)
        pk, sig, msg = (np.ascontiguousarray(x) for x in (pk, sig, msg))
        dt = self.base.cpubase_run(SODIUM.encode() if self.have_sodium else None, pk.ctypes.data, sig.ctypes.data,
                                   msg.ctypes.data, mlen, n, nthreads, out.ctypes.data)
        return n / dt, out


def host_api_rate(env, pk, sig, msg, mlen, reps=3):
    sv = env.sv
    sv.verify_fixed(pk[:1024], sig[:1024], msg.reshape(-1)[:1024 * mlen], mlen)
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        out = sv.verify_fixed(pk, sig, msg.reshape(-1), mlen)
        best = min(best, time.perf_counter() - t0)
    return pk.shape[0] / best, out


def device_rate(env, tpk, tsig, tmsg, n, mlen, reps=5):
    t, sv = env.torch, env.sv
    tv = t.zeros(n, dtype=t.uint8, device=env.dev)
    sv.verify_device(0, tpk.data_ptr(), tsig.data_ptr(), tmsg.data_ptr(), n, tv.data_ptr(), 0, env.stream,
                     fixed_msg_len=mlen)
    t.cuda.synchronize(env.dev)
    sv.kernel_time_reset()
    sv.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        sv.verify_device(0, tpk.data_ptr(), tsig.data_ptr(), tmsg.data_ptr(), n, tv.data_ptr(), 0, env.stream,
                         fixed_msg_len=mlen)
    sv.synchronize(0)
    t.cuda.synchronize(env.dev)
    wall = (time.perf_counter() - t0) / reps
    sv.timing_enable(False)
    ms, la, _ = sv.kernel_time(0)
    return n / wall, n / (ms / la * 1e-3), tv.cpu().numpy()


def verifysig_equivalent_rate(env, pk, sig, msg, mlen, nthreads):
    """C++ PubKeyUtils mirror (BLAKE2b key, cache, mutex) with libsodium behind it."""
    if not env.have_sodium:
        return None
    base = env.base
    base.cpubase_set_sodium.argtypes = [ctypes.c_char_p, ctypes.c_int]
    assert base.cpubase_set_sodium(SODIUM.encode(), nthreads) == 0
    env.host.svh_set_test_verifier(ctypes.cast(base.cpubase_sodium_batch, ctypes.c_void_p))
    env.host.svh_cache_clear()
    n = pk.shape[0]
    off = (np.arange(n, dtype=np.uint64) * mlen)
    ln = np.full(n, mlen, np.uint32)
    out = np.zeros(n, np.uint8)
    pk, sig, msg = (np.ascontiguousarray(x) for x in (pk, sig, msg))
    t0 = time.perf_counter()
    rc = env.host.svh_verify_sig_batch(ctypes.c_void_p(pk.ctypes.data), ctypes.c_void_p(sig.ctypes.data), None,
                                       ctypes.c_void_p(msg.ctypes.data), ctypes.c_void_p(off.ctypes.data),
                                       ctypes.c_void_p(ln.ctypes.data), ctypes.c_size_t(n),
                                       ctypes.c_void_p(out.ctypes.data))
    dt = time.perf_counter() - t0
    env.host.svh_set_test_verifier(None)
    env.host.svh_cache_clear()
    assert rc == 0
    return n / dt


def verifysig_batch_gpu_rate(env, pk, sig, msg, mlen, keyed):
    """C++ PubKeyUtils::verifySigBatch mirror on the GPU engine, cache cleared:
    keyed (f4: engine returns the BLAKE2b cache keys) or host-hashed."""
    h = env.host
    h.svh_set_keyed_threshold.argtypes = [ctypes.c_size_t]
    h.svh_set_test_verifier(None)
    h.svh_set_keyed_threshold(1 if keyed else 0)
    n = pk.shape[0]
    off = (np.arange(n, dtype=np.uint64) * mlen)
    ln = np.full(n, mlen, np.uint32)
    pk, sig, msg = (np.ascontiguousarray(x) for x in (pk, sig, msg))
    best = 1e9
    for _ in range(3):
        h.svh_cache_clear()
        out = np.zeros(n, np.uint8)
        t0 = time.perf_counter()
        rc = h.svh_verify_sig_batch(ctypes.c_void_p(pk.ctypes.data), ctypes.c_void_p(sig.ctypes.data), None,
                                    ctypes.c_void_p(msg.ctypes.data), ctypes.c_void_p(off.ctypes.data),
                                    ctypes.c_void_p(ln.ctypes.data), ctypes.c_size_t(n),
                                    ctypes.c_void_p(out.ctypes.data))
        best = min(best, time.perf_counter() - t0)
        assert rc == 0, h.svh_last_error_string()
    h.svh_set_keyed_threshold(4096)
    h.svh_cache_clear()
    return n / best, bool(out.all())


def config1(env):
    res = {}
    T = threads()
    rng = np.random.default_rng(1)
    n = 100_000
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    tpk, tsig, tm = env.gpu_sign(seeds, msgs)
    pk, sig = tpk.cpu().numpy(), tsig.cpu().numpy()
    host_rate, out_h = host_api_rate(env, pk, sig, msgs, 32)
    wall_rate, kern_rate, out_d = device_rate(env, tpk, tsig, tm, n, 32)
    cpu1, o1 = env.cpu_rate(pk[:10000], sig[:10000], msgs[:10000], 32, 1)
    cpuT, oT = env.cpu_rate(pk, sig, msgs, 32, T)
    vse1 = verifysig_equivalent_rate(env, pk[:10000], sig[:10000], msgs[:10000], 32, 1)
    vsg_h, ok_h = verifysig_batch_gpu_rate(env, pk, sig, msgs, 32, keyed=False)
    vsg_k, ok_k = verifysig_batch_gpu_rate(env, pk, sig, msgs, 32, keyed=True)
    # the engine's CPU path (host build of the same algorithm), one thread, and
    # single verifySig calls that miss the cache (one item -> the CPU path)
    k1 = 2000
    t0 = time.perf_counter()
    oc = env.sv.verify_batch_cpu(pk[:k1], sig[:k1], msgs[:k1].reshape(-1), np.arange(k1, dtype=np.uint64) * 32,
                                 np.full(k1, 32, np.uint32), threads=1)
    cpu_path1 = k1 / (time.perf_counter() - t0)
    h = env.host
    h.svh_verify_sig.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
    h.svh_cache_clear()
    lat = []
    single_ok = True
    for i in range(k1):
        a_, b_, c_ = pk[i].tobytes(), sig[i].tobytes(), msgs[i].tobytes()
        t0 = time.perf_counter()
        r = h.svh_verify_sig(a_, b_, 64, c_, 32)
        lat.append(time.perf_counter() - t0)
        single_ok = single_ok and r == 1
    h.svh_cache_clear()
    res["single_verifysig"] = {
        "cpu_path_1thread_verifies_per_s": cpu_path1, "cpu_path_all_valid": bool(oc.all()),
        "verifysig_miss_p50_us": float(np.percentile(lat, 50) * 1e6),
        "verifysig_miss_p99_us": float(np.percentile(lat, 99) * 1e6),
        "verifysig_all_valid": single_ok,
        "path": "svh_verify_sig (C++ PubKeyUtils::verifySig mirror): cache miss, one item -> engine CPU path",
    }
    res["100k_x_32B"] = {
        "gpu_verifysig_batch_host_hashed_per_s": vsg_h, "gpu_verifysig_batch_keyed_per_s": vsg_k,
        "verifysig_batch_all_valid": ok_h and ok_k,
        "gpu_host_api_verifies_per_s": host_rate, "gpu_device_api_verifies_per_s": wall_rate,
        "gpu_kernel_verifies_per_s": kern_rate, "cpu_libsodium_1thread": cpu1,
        "cpu_libsodium_threads": cpuT, "cpu_threads": T, "cpu_verifysig_equivalent_1thread": vse1,
        "all_valid": bool(out_h.all() and out_d.all() and o1.all() and oT.all()),
    }
    if env.have_sodium:
        k = 10_000
        pks, sigs, ms = [], [], []
        for i in range(k):
            m = hashlib.shake_256(b"REF256" + struct.pack("<Q", i)).digest(256)
            p, s = env.sodium_sign(hashlib.sha256(b"REFKEY" + struct.pack("<Q", i)).digest(), m)
            pks.append(p); sigs.append(s); ms.append(m)
        pk2 = np.frombuffer(b"".join(pks), np.uint8).reshape(k, 32)
        sg2 = np.frombuffer(b"".join(sigs), np.uint8).reshape(k, 64)
        m2 = np.frombuffer(b"".join(ms), np.uint8).reshape(k, 256)
        hr, oh = host_api_rate(env, pk2, sg2, m2, 256)
        c1, oc1 = env.cpu_rate(pk2, sg2, m2, 256, 1)
        cT, ocT = env.cpu_rate(pk2, sg2, m2, 256, T)
        v1 = verifysig_equivalent_rate(env, pk2, sg2, m2, 256, 1)
        res["ref_shape_10k_x_256B"] = {
            "gpu_host_api_verifies_per_s": hr, "cpu_libsodium_1thread": c1, "cpu_libsodium_threads": cT,
            "cpu_threads": T, "cpu_verifysig_equivalent_1thread": v1,
            "all_valid": bool(oh.all() and oc1.all() and ocT.all()),
        }
    return res


def config3(env, n_tx=5000, sets=5):
    """BASELINE config 3.  A node checks each ledger's tx set once, so the
    headline is over `sets` DISTINCT sets (different accounts, keys and
    signatures), each checked once after a first set that warms the process
    (thread pools, staging, workspaces): median and max, plus the process's
    first call.  Host comparators on set 0: the same checkers with libsodium
    per signature on one thread (the reference's path), and the same batch
    pre-pass with libsodium on all of the job's host threads."""
    import txset_gen as tg

    def gpu_sign_fn(reqs):
        seeds = np.frombuffer(b"".join(r[0] for r in reqs), np.uint8).reshape(-1, 32)
        msgs = np.frombuffer(b"".join(r[1] for r in reqs), np.uint8).reshape(-1, 32)
        tpk, tsig, _ = env.gpu_sign(seeds, msgs)
        pk, sg = tpk.cpu().numpy(), tsig.cpu().numpy()
        return [(pk[i].tobytes(), sg[i].tobytes()) for i in range(len(reqs))]

    def var_sign_fn(reqs):
        return [env.sodium_sign(s, m) for s, m in reqs]

    def make(seed):
        txs = tg.generate(n_tx, gpu_sign_fn, seed=seed)
        if env.have_sodium:
            tg.add_payload_signatures(txs, var_sign_fn)
        return txs, tg.to_ctypes(txs)

    def run(cts, prefetch):
        T, S, G = cts
        ok = np.zeros(n_tx, np.uint8)
        used = np.zeros(n_tx, np.uint8)
        pairs = ctypes.c_uint64()
        env.host.svh_cache_clear()
        t1 = time.perf_counter()
        rc = env.host.svh_check_txset(T, ctypes.c_size_t(n_tx), S, G, prefetch, ok.ctypes.data_as(ctypes.c_void_p),
                                      used.ctypes.data_as(ctypes.c_void_p), ctypes.byref(pairs))
        dt = time.perf_counter() - t1
        assert rc == 0, env.host.svh_last_error_string()
        ph = (ctypes.c_double * 4)()
        env.host.svh_txset_last_phases(ph)
        phases.append(list(ph))
        return ok, used, dt, pairs.value

    phases = []
    t0 = time.perf_counter()
    built = [make(2025 + k) for k in range(sets + 1)]
    gen_s = (time.perf_counter() - t0) / (sets + 1)
    txs, cts = built[0]
    nsig = sum(len(t["sigs"]) for t in txs)
    # the headline runs the pipelined pre-pass (svh_check_txset use_prefetch 4: two halves, the engine on one
    # beside the host work of the other); the one-batch pre-pass (use_prefetch 1) is timed beside it
    ok_g, used_g, dt_first, pairs = run(cts, 4)
    run(cts, 1)
    del phases[:]
    outs = [run(b[1], 4) for b in built[1:]]  # each distinct set once
    dts = [o[2] for o in outs]
    ph = np.array(phases)  # the distinct sets' phases, in ms
    outs1 = [run(b[1], 1) for b in built[1:]]
    dts1 = [o[2] for o in outs1]
    ph1 = np.array(phases[len(outs):])
    same_as_one_batch = all((a[0] == b[0]).all() and (a[1] == b[1]).all() for a, b in zip(outs, outs1))
    phase_split = {k: float(np.median(ph[:, j])) for j, k in enumerate(
        ("marshal_ms", "half0_pair_enumeration_ms", "overlapped_engine_and_host_ms", "half1_checkers_ms"))}
    phase_split["per_set"] = [[round(float(x), 3) for x in row] for row in ph]
    phase_split["what"] = ("svh_txset_last_phases medians over the distinct sets, pipelined pre-pass: the mirror "
                           "objects' allocation; half 0's marshal + pair enumeration (SignatureBatchPrefetch::"
                           "addBatch); engine on half 0 beside half 1's enumeration, then engine on half 1 beside "
                           "half 0's checkers; half 1's checkers")
    phase_split_one_batch = {k: float(np.median(ph1[:, j])) for j, k in enumerate(
        ("marshal_ms", "pair_enumeration_ms", "engine_prepass_ms", "checkers_ms"))}
    dt_rep = min(run(cts, 4)[2] for _ in range(3))  # the first set again (warm per-key state): not the headline
    out = {"txs": n_tx, "decorated_signatures": nsig, "prefetched_pairs": pairs, "generate_s": gen_s,
           "distinct_sets": sets,
           "gpu_prepass_checker_s": float(np.median(dts)), "gpu_prepass_checker_max_s": float(max(dts)),
           "gpu_prepass_checker_first_call_s": dt_first, "gpu_prepass_same_set_repeat_min_s": dt_rep,
           "gpu_prepass_txs_per_s": n_tx / float(np.median(dts)),
           "prepass_mode": "pipelined (svh_check_txset use_prefetch 4)",
           "phase_split": phase_split,
           "one_batch_prepass": {"median_s": float(np.median(dts1)), "max_s": float(max(dts1)),
                                 "phase_split": phase_split_one_batch,
                                 "outcomes_equal_pipelined": bool(same_as_one_batch),
                                 "what": "the same sets through the one-batch pre-pass (use_prefetch 1)"},
           "timing": "median / max over %d distinct sets, each checked once after a first (warm-up) set; "
                     "first_call = the process's first set" % sets}
    if env.have_sodium:
        base = env.base
        base.cpubase_set_sodium.argtypes = [ctypes.c_char_p, ctypes.c_int]
        assert base.cpubase_set_sodium(SODIUM.encode(), 1) == 0
        env.host.svh_set_test_verifier(ctypes.cast(base.cpubase_sodium_batch, ctypes.c_void_p))
        ok_c, used_c, dt_c, _ = run(cts, 0)  # reference path: per-signature libsodium, one thread
        T = threads()
        assert base.cpubase_set_sodium(SODIUM.encode(), T) == 0
        ok_t, used_t, dt_t, _ = run(cts, 1)  # the same pre-pass, libsodium on every host thread
        env.host.svh_set_test_verifier(None)
        env.host.svh_cache_clear()
        so = env.sodium

        def verify(pk, sig, msg):
            return so.crypto_sign_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0

        match = True
        for (tx_k, _), o in zip(built, [(ok_g, used_g)] + [(x[0], x[1]) for x in outs]):
            want_ok, want_used = tg.replay(tx_k, verify)
            match = match and bool((o[0] == want_ok).all() and (o[1] == want_used).all())
            if tx_k is txs:
                match = match and bool((ok_c == want_ok).all() and (used_c == want_used).all()
                                       and (ok_t == want_ok).all() and (used_t == want_used).all())
                n_ok, n_used = int(want_ok.sum()), int(want_used.sum())
        out.update({
            "cpu_reference_checker_s": dt_c, "cpu_reference_txs_per_s": n_tx / dt_c,
            "cpu_libsodium_prepass_threads_s": dt_t, "cpu_prepass_threads": T,
            "speedup_vs_reference_1thread": dt_c / out["gpu_prepass_checker_s"],
            "speedup_vs_libsodium_prepass_all_threads": dt_t / out["gpu_prepass_checker_s"],
            "outcomes_match_python_replay": match,
            "txs_ok": n_ok, "txs_all_sigs_used": n_used,
        })
    return out


class MbStats(ctypes.Structure):
    _fields_ = [("items", ctypes.c_uint64), ("batches", ctypes.c_uint64), ("flushed_by_size", ctypes.c_uint64),
                ("flushed_by_deadline", ctypes.c_uint64), ("max_batch", ctypes.c_uint64),
                ("lat_p50_us", ctypes.c_double), ("lat_p99_us", ctypes.c_double)]


def configmb(env, n=200_000, producers=8):
    rng = np.random.default_rng(9)
    lens = rng.integers(120, 240, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    msg = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    nk = 64  # validator-set sized key population
    pks, sks = [], []
    for i in range(nk):
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        if env.have_sodium:
            env.sodium.crypto_sign_seed_keypair(pk, sk, hashlib.sha256(b"VAL" + struct.pack("<Q", i)).digest())
        pks.append(pk.raw); sks.append(sk.raw)
    if not env.have_sodium:
        return {"skipped": "libsodium absent"}
    kid = rng.integers(0, nk, n)
    sig = np.zeros((n, 64), np.uint8)
    s = ctypes.create_string_buffer(64)
    for i in range(n):
        o = int(off[i])
        env.sodium.crypto_sign_detached(s, None, msg[o:o + int(lens[i])].tobytes(), ctypes.c_ulonglong(int(lens[i])),
                                        sks[kid[i]])
        sig[i] = np.frombuffer(s.raw, np.uint8)
    sig[::97, 5] ^= 1  # some forgeries
    pk = np.ascontiguousarray(np.frombuffer(b"".join(pks), np.uint8).reshape(nk, 32)[kid])
    want = np.ones(n, np.uint8)
    want[::97] = 0
    vp = ctypes.c_void_p

    def run(max_batch, max_delay_us, workers=1):
        out = np.zeros(n, np.uint8)
        st = MbStats()
        env.host.svh_cache_clear()
        t0 = time.perf_counter()
        rc = env.host.svh_mb_run_workers(vp(pk.ctypes.data), vp(sig.ctypes.data), vp(msg.ctypes.data),
                                         vp(off.ctypes.data), vp(lens.ctypes.data), ctypes.c_size_t(n), producers,
                                         workers, ctypes.c_uint32(max_batch), ctypes.c_uint32(max_delay_us),
                                         ctypes.c_uint32(0), vp(out.ctypes.data), ctypes.byref(st))
        dt = time.perf_counter() - t0
        assert rc == 0, env.host.svh_last_error_string()
        return {"verifies_per_s": n / dt, "batches": st.batches, "flushed_by_size": st.flushed_by_size,
                "flushed_by_deadline": st.flushed_by_deadline, "max_batch_seen": st.max_batch,
                "lat_p50_us": st.lat_p50_us, "lat_p99_us": st.lat_p99_us,
                "verdicts_match": bool((out == want).all())}

    res = {"messages": n, "producers": producers, "gpu": {}}
    for mbatch in (1024, 8192, 65536):
        res["gpu"]["max_batch_%d" % mbatch] = run(mbatch, 2000)
    for workers in (2, 4, 8):  # several flush workers: batches in flight at once
        for mbatch in (1024, 8192):
            res["gpu"]["max_batch_%d_workers_%d" % (mbatch, workers)] = run(mbatch, 2000, workers)
    base = env.base
    base.cpubase_set_sodium.argtypes = [ctypes.c_char_p, ctypes.c_int]
    assert base.cpubase_set_sodium(SODIUM.encode(), 1) == 0
    env.host.svh_set_test_verifier(ctypes.cast(base.cpubase_sodium_batch, ctypes.c_void_p))
    res["cpu_libsodium_1thread_batch_1024"] = run(1024, 2000)
    env.host.svh_set_test_verifier(None)
    env.host.svh_cache_clear()
    return res


def config5(env, tiles=64):
    t = env.torch
    n1 = 1 << 20
    s = bytearray()
    m = bytearray()
    for i in range(n1):
        p = struct.pack("<Q", i)
        s += hashlib.sha256(b"SVSEED" + p).digest()
        m += hashlib.sha256(b"SVMSG" + p).digest()
    seeds = np.frombuffer(bytes(s), np.uint8).reshape(n1, 32)
    msgs = np.frombuffer(bytes(m), np.uint8).reshape(n1, 32)
    tpk, tsig, tm = env.gpu_sign(seeds, msgs)
    n = n1 * tiles
    bpk = tpk.repeat(tiles, 1)
    bsig = tsig.repeat(tiles, 1)
    bmsg = tm.repeat(tiles, 1)
    wall, kern, out = device_rate(env, bpk, bsig, bmsg, n, 32, reps=2)
    return {"signatures": n, "construction": "libsodium-pinned 2^20 dataset tiled %dx on device" % tiles,
            "device_api_verifies_per_s": wall, "kernel_verifies_per_s": kern, "all_valid": bool(out.all()),
            "seconds_per_batch": n / wall}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,3,mb,5")
    ap.add_argument("--txs", type=int, default=5000)
    args = ap.parse_args()
    env = Env()
    res = {"device": "MI355X", "cpu_threads": threads()}
    for c in args.configs.split(","):
        t0 = time.perf_counter()
        res["config" + c] = {"1": lambda: config1(env), "3": lambda: config3(env, args.txs),
                             "5": lambda: config5(env), "mb": lambda: configmb(env)}[c]()
        log("config %s done in %.1fs" % (c, time.perf_counter() - t0))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
