#!/usr/bin/env python3
"""Headline benchmark: ed25519 verifies/sec @1M batch per GPU + p50 latency @1k batch.

Metric and configs: BASELINE.json.  One "step" = one pass of the hot path
(sv_ed25519_verify_device) over one batch of 2^20 signatures per GPU, inputs
already resident in HBM.  N GPUs run as N processes (torchrun), each verifying
its own contiguous slice of the global index space (weak scaling, no data-path
collective; the only collectives are the barrier and the max-over-ranks of the
timed region, over gloo).

Dataset: seed_i = SHA-256("SVSEED"||u64le i), msg_i =
SHA-256("SVMSG"||u64le i); keypairs and signatures are generated ON THE GPU
by the engine's RFC 8032 signer, and on rank 0 the SHA-256 of the
pk||sig||msg stream is compared with the libsodium-generated digest in
tests/golden/digests.json, so the bench verifies the exact dataset libsodium
would produce.

Printed by rank 0: one JSON line (contract in the task statement) with
  roofline      VALU-integer roofline of the verify kernel (kernel time from
                HIP events on the engine's stream over the timed region)
  cpu_baseline  libsodium crypto_sign_verify_detached (the function
                PubKeyUtils::verifySig calls), multithreaded on this host's
                cores over a bounded sample of the same dataset
  latency_1k    p50/p99 end-to-end latency of 1000-signature SCP-sized batches
                through the host API (H2D + kernel + D2H)
"""
import argparse
import ctypes
import hashlib
import importlib
import json
import os
import struct
import sys
import threading
import time
import traceback

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "ed25519 verifies/sec @1M batch (1/8 GPU) + p50 latency @1k batch"
# Algorithmic work per verify: ~1524 field squarings x 44 +
# ~1488 multiplications x 72 32x32->64 multiply-adds of the 8x32-bit-limb
# schoolbook formulation of libsodium's op count.
W_MAD_PER_VERIFY = 174192
# Peak of the instruction the field arithmetic is built from: v_mad_u64_u32
# (32x32->64 multiply-add) issues at 4 cycles per wave64 instruction per
# SIMD-32 = 64 lane-ops/clk/CU (measured 60.6 at 8 waves/SIMD, 53.2 at the
# verify kernels' 2; the same harness reads v_fma_f32 at 112 of the 128 the
# CDNA4 guide states: profiles/r02/ubench_valu_rates.txt) x 256 CUs x 2.4 GHz.
MAD_LANE_OPS_PER_CLK_CU = 64
PEAK_CLOCK_HZ = 2.4e9
PEAK_SOURCE = ("v_mad_u64_u32 64 lane-ops/clk/CU (4 cyc per wave64 instruction per SIMD-32) x CUs x 2.4 GHz; "
               "harness profiles/r02/ubench_valu_rates.txt measures 60.6 (95 %) at 8 waves/SIMD")
NOMINAL_PEAK_SURVEY = 9.83e12  # SURVEY.md §8 d7 assumption (quarter-rate); measured rate is 3.5x higher


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def leg_failed(result, key, exc):
    """An optional leg of rank 0 (everything but the timed region and config
    5's collective) that raised: the error goes into the line under `key`
    instead of costing the line (an 8-GPU node runs the in-process leg over
    real devices for the first time)."""
    log("leg %s failed:" % key)
    traceback.print_exc()
    result[key] = {"error": "%s: %s" % (type(exc).__name__, exc)}


def seeds_and_msgs(lo, hi):
    seeds = bytearray()
    msgs = bytearray()
    for i in range(lo, hi):
        p = struct.pack("<Q", i)
        seeds += hashlib.sha256(b"SVSEED" + p).digest()
        msgs += hashlib.sha256(b"SVMSG" + p).digest()
    return np.frombuffer(bytes(seeds), np.uint8), np.frombuffer(bytes(msgs), np.uint8)


def load_libsodium():
    for name in ("libsodium.so.23", "libsodium.so", "/opt/conda/lib/libsodium.so.23"):
        try:
            lib = ctypes.CDLL(name)
            if lib.sodium_init() < 0:
                continue
            lib.sodium_version_string.restype = ctypes.c_char_p
            return lib
        except OSError:
            continue
    return None


def cpu_verify_rate(pk, sig, msg, mlen, threads, sodium_path):
    """Native pthread harness (oracle/cpu_baseline.c): libsodium when
    sodium_path is given ("reference"), else the oracle restatement ("port")."""
    base = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    base.cpubase_run.restype = ctypes.c_double
    base.cpubase_run.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_uint32, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    n = pk.shape[0]
    pk = np.ascontiguousarray(pk)
    sig = np.ascontiguousarray(sig)
    msg = np.ascontiguousarray(msg)
    out = np.zeros(n, np.uint8)
    dt = base.cpubase_run(sodium_path.encode() if sodium_path else None, pk.ctypes.data, sig.ctypes.data,
                          msg.ctypes.data, mlen, n, threads, out.ctypes.data)
    if dt <= 0:
        raise RuntimeError("cpu baseline harness failed (%s)" % dt)
    return n / dt, dt, out


def host_cpus():
    """Threads for the CPU baseline: every CPU this process may run on
    (sched_getaffinity), limited by the cgroup CPU quota when one is set (a
    quota below the affinity count means only that many run at once)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        quota = None
    threads = aff if quota is None else max(1, min(aff, int(quota + 1e-9)))
    threads = min(threads, 256)  # (oracle/cpu_baseline.c thread table)
    return threads, {"sched_getaffinity": aff, "os_cpu_count": os.cpu_count(), "cgroup_quota_cpus": quota,
                     "threads_used": threads}


def cpu_batch_latency(spath, pk, sig, buf, off, ln, threads, iters):
    """p50 wall time of one libsodium batch (one crypto_sign_verify_detached per
    signature on `threads` pthreads, oracle/cpu_baseline.c cpubase_sodium_batch)."""
    base = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    base.cpubase_set_sodium.argtypes = [ctypes.c_char_p, ctypes.c_int]
    if base.cpubase_set_sodium(spath.encode(), threads) != 0:
        raise RuntimeError("libsodium setup failed")
    base.cpubase_sodium_batch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_void_p]
    out = np.zeros(len(ln), np.uint8)
    ts = []
    for _ in range(iters):
        t1 = time.perf_counter()
        rc = base.cpubase_sodium_batch(pk.ctypes.data, sig.ctypes.data, buf.ctypes.data, off.ctypes.data,
                                       ln.ctypes.data, len(ln), out.ctypes.data)
        ts.append((time.perf_counter() - t1) * 1e3)
        if rc != 0:
            raise RuntimeError("cpubase_sodium_batch failed")
    return float(np.percentile(ts, 50)), out


def sodium_path():
    for p in ("/opt/conda/lib/libsodium.so.23", "libsodium.so.23", "libsodium.so"):
        try:
            ctypes.CDLL(p)
            return p
        except OSError:
            continue
    return None


def verifysig_equivalent_rate(sv, spath, pk, sig, msg, mlen, threads):
    """The reference's PubKeyUtils::verifySig on `threads` threads: the C++
    mirror (BLAKE2b cache key, 0xffff-entry cache behind its mutex) with one
    libsodium call per miss behind it (SecretKey.cpp:435-468), cache cleared
    first.  Native harness oracle/cpu_baseline.c cpubase_verifysig_threads."""
    base = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    host = ctypes.CDLL(sv.HOSTLIB_PATH)
    base.cpubase_set_sodium.argtypes = [ctypes.c_char_p, ctypes.c_int]
    if base.cpubase_set_sodium(spath.encode(), 1) != 0:
        raise RuntimeError("libsodium setup failed")
    base.cpubase_verifysig_threads.restype = ctypes.c_double
    base.cpubase_verifysig_threads.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    host.svh_set_test_verifier.argtypes = [ctypes.c_void_p]
    n = pk.shape[0]
    pk, sig, msg = (np.ascontiguousarray(x) for x in (pk, sig, msg))
    off = np.arange(n, dtype=np.uint64) * mlen
    ln = np.full(n, mlen, np.uint32)
    out = np.zeros(n, np.uint8)
    host.svh_set_test_verifier(ctypes.cast(base.cpubase_sodium_batch, ctypes.c_void_p))
    host.svh_cache_clear()
    try:
        dt = base.cpubase_verifysig_threads(ctypes.cast(host.svh_verify_sig, ctypes.c_void_p), pk.ctypes.data,
                                            sig.ctypes.data, msg.ctypes.data, off.ctypes.data, ln.ctypes.data, n,
                                            threads, out.ctypes.data)
    finally:
        host.svh_set_test_verifier(None)
        host.svh_cache_clear()
    if dt <= 0:
        raise RuntimeError("verifySig harness failed (%s)" % dt)
    return n / dt, out


def config1(sv, sodium, spath, pk_h, sig_h, msgs, threads, device):
    """BASELINE config 1 / SURVEY.md §8 d2, both shapes: 100k x 32-byte hashes
    (BASELINE.json; the bench dataset's first 100k) and the reference's own
    benchmark shape, 10k keypairs x 256-byte messages (SecretKey.cpp:182-234,
    CryptoTests.cpp:299-306; libsodium-signed here).  Raw libsodium and the
    verifySig equivalent, 1 thread and all cores, beside the GPU host API."""
    out = {}
    k = min(100_000, pk_h.shape[0])
    shapes = [("100k_x_32B", pk_h[:k], sig_h[:k], msgs[:32 * k].reshape(k, 32), 32, 16384)]
    pks, sgs, ms = [], [], []
    for i in range(10_000):
        m = hashlib.shake_256(b"REF256" + struct.pack("<Q", i)).digest(256)
        pkb = ctypes.create_string_buffer(32)
        skb = ctypes.create_string_buffer(64)
        sodium.crypto_sign_seed_keypair(pkb, skb, hashlib.sha256(b"REFKEY" + struct.pack("<Q", i)).digest())
        sb = ctypes.create_string_buffer(64)
        sodium.crypto_sign_detached(sb, None, m, ctypes.c_ulonglong(256), skb)
        pks.append(pkb.raw); sgs.append(sb.raw); ms.append(m)
    shapes.append(("ref_shape_10k_x_256B", np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 32),
                   np.frombuffer(b"".join(sgs), np.uint8).reshape(-1, 64),
                   np.frombuffer(b"".join(ms), np.uint8).reshape(-1, 256), 256, 10_000))
    for name, pk, sg, m, mlen, st in shapes:
        sv.verify_fixed(pk[:1024], sg[:1024], m[:1024], mlen, device=device)
        best, g_ok = None, True
        for _ in range(3):
            t1 = time.perf_counter()
            o = sv.verify_fixed(pk, sg, m, mlen, device=device)
            dt = time.perf_counter() - t1
            g_ok = g_ok and bool(o.all())
            best = dt if best is None else min(best, dt)
        c_t, _, o1 = cpu_verify_rate(pk, sg, m.reshape(-1), mlen, threads, spath)
        c_1, _, o2 = cpu_verify_rate(pk[:st], sg[:st], m[:st].reshape(-1), mlen, 1, spath)
        v_1, o3 = verifysig_equivalent_rate(sv, spath, pk[:st], sg[:st], m[:st], mlen, 1)
        v_t, o4 = verifysig_equivalent_rate(sv, spath, pk, sg, m, mlen, threads)
        out[name] = {
            "signatures": int(pk.shape[0]), "msg_len": mlen,
            "gpu_host_api_verifies_per_s": pk.shape[0] / best,
            "cpu_libsodium_threads": c_t, "cpu_libsodium_1thread": c_1,
            "cpu_verifysig_equivalent_threads": v_t, "cpu_verifysig_equivalent_1thread": v_1,
            "cpu_threads": threads, "single_thread_sample": st,
            "all_valid": bool(g_ok and o1.all() and o2.all() and o3.all() and o4.all()),
        }
    # verify-hit benchmarking (CryptoTests.cpp:308-316: benchmarkOpsPerSecond
    # with 10 passes, the last 9 timed, every call a cache hit): the mirror's
    # PubKeyUtils::verifySig on the 10k x 256 B cases, 1 thread and 3 threads
    # contending for the cache (native loop, include/stellar_host.h)
    host = ctypes.CDLL(sv.HOSTLIB_PATH)
    host.svh_bench_verify_hits.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                                                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    _, pk, sg, m, mlen, _ = shapes[1]
    pk, sg, m = (np.ascontiguousarray(x) for x in (pk, sg, m))
    hit = {"cases": int(pk.shape[0]), "msg_len": mlen, "passes": 10,
           "what": "PubKeyUtils::verifySig mirror (BLAKE2b-256 key, 0xffff-entry random-eviction cache behind its "
                   "mutex); pass 0 fills the cache (CPU-path verifies), passes 1-9 timed, all hits"}
    for th in (1, 3):
        host.svh_cache_clear()
        rate, fill = ctypes.c_double(), ctypes.c_double()
        rc = host.svh_bench_verify_hits(pk.ctypes.data, sg.ctypes.data, m.ctypes.data, mlen, pk.shape[0], 10, th,
                                        ctypes.byref(rate), ctypes.byref(fill))
        hit["hits_per_s_%dthread%s" % (th, "" if th == 1 else "s")] = rate.value
        hit["fill_pass_s_%d" % th] = fill.value
        hit["ok_%d" % th] = rc == 0
    host.svh_cache_clear()
    # the same loop over the reference's own hit path (oracle/refcache.cpp:
    # libsodium BLAKE2b key, exists() + get() on a std::unordered_map hashed
    # by SipHash under shortHash's mutex, all behind gVerifySigCacheMutex)
    ref = ctypes.CDLL(os.path.join(REPO, "oracle", "librefcache.so"))
    ref.refcache_bench_hits.argtypes = [ctypes.c_char_p] + [ctypes.c_void_p] * 3 + [
        ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    for th in (1, 3):
        rate, fill = ctypes.c_double(), ctypes.c_double()
        rc = ref.refcache_bench_hits(spath.encode(), pk.ctypes.data, sg.ctypes.data, m.ctypes.data, mlen,
                                     pk.shape[0], 10, th, ctypes.byref(rate), ctypes.byref(fill))
        hit["reference_shape_hits_per_s_%dthread%s" % (th, "" if th == 1 else "s")] = rate.value if rc == 0 else None
    hit["reference_shape"] = ("oracle/refcache.cpp: SecretKey.cpp:446-456 as written -- libsodium "
                              "crypto_generichash key, exists() then get() on RandomEvictionCache's unordered_map, "
                              "std::hash<uint256> = crypto_shorthash under shortHash's mutex (HashOfHash.cpp, "
                              "ShortHash.cpp)")
    out["hit_path"] = hit
    return out


def in_process_multi_gpu(sv, pk, sig, msg, reps=3):
    """sv_ed25519_verify_batch_fixed(device = -1, max_devices = G) over a
    G x 2^20 host batch (the bench dataset tiled G times, tile g with rows
    g, g + 97, ... corrupted) for G = 1, 2, 4, 8 up to the slot count; best of
    `reps` calls, verdicts checked against the corruption pattern, and the
    SHA-256 of the verdict bytes."""
    slots = sv.device_count()
    n = pk.shape[0]
    out = {"slots": slots, "device_map": os.environ.get("SV_DEVICE_MAP"),
           "what": "one process, sv_ed25519_verify_batch_fixed(device=-1, max_devices=G) from pageable host arrays: "
                   "G contiguous slices on G device slots, each driven and packed by the slot's own staging workers "
                   "(pinned to the GPU's NUMA node), verdicts gathered into the caller's buffer; host_feed: the same "
                   "host side without kernels (sv_host_feed_probe)", "per_G": {}}
    G = 1
    while G <= min(8, slots):
        N = G * n
        P = np.tile(pk, (G, 1))
        S = np.tile(sig, (G, 1))
        M = np.tile(msg, (G, 1))
        want = np.ones(N, np.uint8)
        for g in range(G):
            rows = np.arange(g * n + g, (g + 1) * n, 97)
            S[rows, 40] ^= 0x04
            want[rows] = 0
        sv.verify_fixed(P[:4096], S[:4096], M[:4096], 32, device=-1, max_devices=G)
        best, ok = None, True
        for _ in range(reps):
            t1 = time.perf_counter()
            o = sv.verify_fixed(P, S, M, 32, device=-1, max_devices=G)
            dt = time.perf_counter() - t1
            ok = ok and bool(np.array_equal(o, want))
            best = dt if best is None else min(best, dt)
        row = {"signatures": N, "ms": best * 1e3, "verifies_per_s": N / best,
               "verdicts_ok": ok, "verdict_sha256": hashlib.sha256(o.tobytes()).hexdigest()}
        # the host side alone (sv_host_feed_probe: slices, each slot's staging
        # workers, pack into pinned staging, H2D; no kernels): what G slots'
        # host feed delivers against what G GPUs verify
        feed = {}
        for upload in (False, True):
            fb, fs = None, None
            for _ in range(2):
                r = sv.host_feed_probe(P, S, M, 32, max_devices=G, upload=upload)
                if fb is None or r["seconds"] < fb:
                    fb, fs = r["seconds"], r
            feed["pack_and_h2d" if upload else "pack_only"] = {"sigs_per_s": N / fb, "GBps": N * 128 / fb / 1e9}
        feed.update({k: fs[k] for k in ("threads_per_slot", "usable_cpus", "gpu_numa", "staging_numa",
                                        "pinned_cpus")})
        row["host_feed"] = feed
        out["per_G"][str(G)] = row
        log("in-process G=%d: %.3e verifies/s; host feed %.1f GB/s pack, %.1f GB/s pack+H2D" % (
            G, N / best, feed["pack_only"]["GBps"], feed["pack_and_h2d"]["GBps"]))
        del P, S, M
        G *= 2
    base = out["per_G"]["1"]["verifies_per_s"]
    for v in out["per_G"].values():
        v["speedup_vs_1_slot"] = v["verifies_per_s"] / base
    return out


def config5(sv, torch, dev, stream, device, d_pk, d_sig, d_msg, n, world, rank, barrier, dist, tiles=64):
    """BASELINE config 5 (catchup scale): 64 x 2^20 signatures sharded as
    contiguous slices over the job's ranks (one GPU each; 1/2/4/8 GPUs as the
    driver launches bench.py), each rank verifying its 64/N tiles of its own
    libsodium-pinned 2^20 dataset in ONE device batch (every signature is
    verified in full: the engine has no cache).  Barrier-bracketed, max over
    ranks; a gathered digest of the per-rank verdict digests."""
    per = tiles // world if tiles % world == 0 else max(1, tiles // world)
    N = n * per
    bpk = d_pk.view(n, 32).repeat(per, 1)
    bsig = d_sig.view(n, 64).repeat(per, 1)
    bmsg = d_msg.view(n, 32).repeat(per, 1)
    out = torch.zeros(N, dtype=torch.uint8, device=dev)
    bm = torch.zeros((N + 63) // 64, dtype=torch.int64, device=dev)
    sv.verify_device(device, bpk.data_ptr(), bsig.data_ptr(), bmsg.data_ptr(), N, out.data_ptr(), bm.data_ptr(),
                     stream)  # (warm-up: workspace sized for the chunk)
    torch.cuda.synchronize(dev)
    walls = []
    sv.kernel_time_reset()
    sv.timing_enable(True)
    for _ in range(2):
        out.zero_()
        torch.cuda.synchronize(dev)
        barrier()
        t0 = time.perf_counter()
        sv.verify_device(device, bpk.data_ptr(), bsig.data_ptr(), bmsg.data_ptr(), N, out.data_ptr(),
                         bm.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        barrier()
        walls.append(time.perf_counter() - t0)
    sv.timing_enable(False)
    ms, _, sigs = sv.kernel_time(device)
    ok = bool(out.all().item()) and bool((bm == -1).all().item())
    bits = bm.cpu()
    wall = min(walls)
    if world > 1:
        t = torch.tensor([wall, 0.0 if ok else 1.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, ok = float(t[0]), float(t[1]) == 0.0
        parts = [torch.zeros_like(bits) for _ in range(world)]
        dist.all_gather(parts, bits)  # (equal slices: 64 % world == 0)
        bits = torch.cat(parts)
    # the whole batch's verdict bitmap, gathered in global row order
    digest = hashlib.sha256(bits.numpy().tobytes()).hexdigest()
    del bpk, bsig, bmsg, out, bm
    torch.cuda.empty_cache()
    total = N * world
    return {"signatures": total, "n_gpus": world, "signatures_per_gpu": N,
            "construction": "each rank's libsodium-pinned 2^20 bench slice tiled %dx in HBM, one "
                            "sv_ed25519_verify_device call per rank (contiguous global slices)" % per,
            "verifies_per_s": total / wall, "seconds_per_batch": wall,
            "rank0_kernel_verifies_per_s": sigs / (ms * 1e-3) if ms > 0 else None,
            "all_valid_and_bitmap_full": ok,
            "gathered_bitmap_sha256": digest,
            "expected_bitmap_sha256": hashlib.sha256(b"\xff" * (total // 8)).hexdigest()}


def config3(n_tx=5000):
    """BASELINE config 3: a synthetic 5000-transaction set (1-20 ED25519
    signers, HASH_X, pre-auth and signed-payload signers, fee bumps; tests/
    txset_gen.py) through the SignatureChecker mirror with the GPU batch
    pre-pass, against the same checkers calling libsodium per signature on one
    thread; outcomes checked against the Python replay of the reference logic
    (tools/bench_configs.py config3)."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import bench_configs as bc
    return bc.config3(bc.Env(), n_tx)


def scp_latency_set(sodium, n=1000, adversarial=0.1, seed=20250211):
    """Config 4: 100 validators, 1000 signatures over 128-384 B messages, 10% adversarial."""
    rng = np.random.default_rng(seed)
    vals = []
    for v in range(100):
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        sodium.crypto_sign_seed_keypair(pk, sk, hashlib.sha256(b"SVVAL" + struct.pack("<Q", v)).digest())
        vals.append((pk.raw, sk.raw))
    pks, sigs, msgs, expect = [], [], [], []
    n_adv = int(n * adversarial)
    adv_rows = set(rng.choice(n, n_adv, replace=False).tolist())
    L = 2**252 + 27742317777372353535851937790883648493
    for i in range(n):
        pk, sk = vals[i % 100]
        m = rng.integers(0, 256, int(rng.integers(128, 385)), dtype=np.uint8).tobytes()
        s = ctypes.create_string_buffer(64)
        sodium.crypto_sign_detached(s, None, m, ctypes.c_ulonglong(len(m)), sk)
        sig = bytearray(s.raw)
        pkb = bytearray(pk)
        if i in adv_rows:
            kind = i % 5
            if kind == 0:      # non-canonical S (S + L)
                S = int.from_bytes(sig[32:], "little") + L
                sig[32:] = S.to_bytes(32, "little")
            elif kind == 1:    # small-order R
                sig[:32] = bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a")
            elif kind == 2:    # small-order A
                pkb[:] = bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05")
            elif kind == 3:    # non-canonical A (y = p)
                pkb[:] = ((2**255 - 19)).to_bytes(32, "little")
            else:              # flipped R bit
                sig[3] ^= 0x10
        ok = sodium.crypto_sign_verify_detached(bytes(sig), m, ctypes.c_ulonglong(len(m)), bytes(pkb)) == 0
        pks.append(bytes(pkb)); sigs.append(bytes(sig)); msgs.append(m); expect.append(1 if ok else 0)
    return pks, sigs, msgs, np.array(expect, np.uint8)


class ScpParams(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint32) for k in ("struct_size", "producers", "burst", "interval_us", "max_batch",
                                               "max_delay_us", "workers", "policy", "linger_us", "idle_in_flight",
                                               "quiet_us", "max_linger_us", "batch_post")]


class ScpResult(ctypes.Structure):
    _fields_ = ([(k, ctypes.c_double) for k in ("verdict_p50_us", "verdict_p90_us", "verdict_p99_us",
                                                "verdict_max_us", "verdict_mean_us", "main_p50_us", "main_p99_us",
                                                "main_call_p50_us")]
                + [(k, ctypes.c_uint64) for k in ("main_hits", "main_misses", "main_mismatches", "batches",
                                                  "flushed_by_size", "flushed_by_deadline", "flushed_idle",
                                                  "max_batch")]
                + [("mean_batch", ctypes.c_double)]
                + [(k, ctypes.c_uint64) for k in ("gpu_batches", "gpu_signatures", "cpu_signatures", "fallbacks")]
                + [(k, ctypes.c_double) for k in ("wall_s", "ready_p50_us", "ready_p99_us")]
                + [("burst_waits", ctypes.c_uint64)]
                + [("main_busy_s", ctypes.c_double), ("main_call_mean_us", ctypes.c_double)])


def scp_envelope_set(sodium, n, seed, adversarial=0.1, validators=100):
    """n distinct SCP-envelope-sized signatures (128-384 B statements) by
    `validators` keys, `adversarial` of them non-canonical S / small-order R /
    small-order A / non-canonical A / flipped R bit (the config-4 classes of
    scp_latency_set); libsodium-signed and libsodium-verified on a thread pool
    (ctypes releases the GIL inside the calls)."""
    from concurrent.futures import ThreadPoolExecutor
    rng = np.random.default_rng(seed)
    vals = []
    for v in range(validators):
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        sodium.crypto_sign_seed_keypair(pk, sk, hashlib.sha256(b"SVVAL" + struct.pack("<Q", v)).digest())
        vals.append((pk.raw, sk.raw))
    lens = rng.integers(128, 385, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    who = rng.integers(0, validators, n)
    pk = np.frombuffer(b"".join(vals[w][0] for w in who), np.uint8).reshape(n, 32).copy()
    sig = np.zeros((n, 64), np.uint8)
    L = 2**252 + 27742317777372353535851937790883648493
    adv = rng.random(n) < adversarial
    kind = rng.integers(0, 5, n)

    def sign(lo, hi):
        s = ctypes.create_string_buffer(64)
        for i in range(lo, hi):
            m = buf[int(off[i]):int(off[i]) + int(lens[i])].tobytes()
            sodium.crypto_sign_detached(s, None, m, ctypes.c_ulonglong(len(m)), vals[who[i]][1])
            sig[i] = np.frombuffer(s.raw, np.uint8)

    parts = 16
    with ThreadPoolExecutor(parts) as ex:
        list(ex.map(lambda t: sign(n * t // parts, n * (t + 1) // parts), range(parts)))
    for i in np.nonzero(adv)[0]:
        k = kind[i]
        if k == 0:
            S = int.from_bytes(sig[i, 32:].tobytes(), "little") + L
            sig[i, 32:] = np.frombuffer(S.to_bytes(32, "little"), np.uint8)
        elif k == 1:
            sig[i, :32] = np.frombuffer(bytes.fromhex(
                "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"), np.uint8)
        elif k == 2:
            pk[i] = np.frombuffer(bytes.fromhex(
                "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"), np.uint8)
        elif k == 3:
            pk[i] = np.frombuffer((2**255 - 19).to_bytes(32, "little"), np.uint8)
        else:
            sig[i, 3] ^= 0x10
    expect = np.zeros(n, np.uint8)

    def verify(lo, hi):
        for i in range(lo, hi):
            m = buf[int(off[i]):int(off[i]) + int(lens[i])].tobytes()
            expect[i] = sodium.crypto_sign_verify_detached(sig[i].tobytes(), m, ctypes.c_ulonglong(len(m)),
                                                           pk[i].tobytes()) == 0

    with ThreadPoolExecutor(parts) as ex:
        list(ex.map(lambda t: verify(n * t // parts, n * (t + 1) // parts), range(parts)))
    return pk, sig, buf, off, lens, expect


def config4_integrated(sv, sodium, n=48000):
    """BASELINE config 4 as stellar-core would run it (VERDICT r4 missing #1):
    overlay threads submit SCP envelopes into ONE VerifyMicroBatcher
    (Peer.cpp:963-970), whose flush workers run keyed verifySigBatch calls
    (GPU BLAKE2b keys, cache walk, the slot's latency lane with the warm-key
    comb kernel); each verdict's continuation posts the envelope to a main
    thread that calls verifySig as HerderImpl::verifyEnvelope does
    (HerderImpl.cpp:2414-2432).  100 validator keys, 128-384 B statements,
    10 % adversarial, every envelope distinct (the verify cache starts empty
    for each mode; the device key cache is warm after the first batch).
    Reported: submit -> verdict and submit -> main-thread verifySig latency,
    the main thread's cache hit count, verdicts vs libsodium."""
    host = ctypes.CDLL(sv.HOSTLIB_PATH)
    host.svh_last_error_string.restype = ctypes.c_char_p
    host.svh_scp_run.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_void_p]
    t0 = time.perf_counter()
    pk, sig, buf, off, lens, expect = scp_envelope_set(sodium, n, seed=4242)
    gen_s = time.perf_counter() - t0

    def run(sl, producers, burst, interval_us, workers=2, policy=0, linger_us=0, max_batch=8192,
            max_delay_us=2000, quiet_us=0, max_linger_us=200, batch_post=1):
        a, b = sl
        m = b - a
        p = ScpParams(ctypes.sizeof(ScpParams), producers, burst, interval_us, max_batch, max_delay_us, workers,
                      policy, linger_us, 1, quiet_us, max_linger_us, batch_post)
        r = ScpResult()
        out = np.full(m, 7, np.uint8)
        o0 = int(off[a])
        offs = np.ascontiguousarray(off[a:b] - off[a])
        host.svh_cache_clear()
        rc = host.svh_scp_run(pk[a:b].ctypes.data, sig[a:b].ctypes.data, buf[o0:].ctypes.data, offs.ctypes.data,
                              np.ascontiguousarray(lens[a:b]).ctypes.data, m, ctypes.byref(p), out.ctypes.data,
                              ctypes.byref(r))
        if rc != 0:
            raise RuntimeError("svh_scp_run: %s" % host.svh_last_error_string())
        d = {k: getattr(r, k) for k, _ in ScpResult._fields_}
        for k in list(d):
            if k.endswith("_us"):
                d[k.replace("_us", "_ms")] = d.pop(k) / 1e3
        d.update({"envelopes": m, "producers": producers, "burst": burst, "interval_us": interval_us,
                  "workers": workers, "policy": "deadline" if policy else "when_idle", "linger_us": linger_us,
                  "quiet_us": quiet_us, "max_linger_us": max_linger_us,
                  "main_thread_post": "one task per verified batch" if batch_post else "one task per envelope",
                  "max_batch_setting": max_batch, "max_delay_us": max_delay_us,
                  "offered_per_s": (burst * 1e6 / interval_us) if interval_us else None,
                  "achieved_per_s": m / d["wall_s"] if d["wall_s"] > 0 else None,
                  "main_hit_ratio": d["main_hits"] / max(1, d["main_hits"] + d["main_misses"]),
                  # the main thread's verifySig ceiling over the run (calls / time inside them):
                  # an offered rate above it queues on the main thread whatever the engine does
                  "main_thread_verifysig_per_s": m / d["main_busy_s"] if d["main_busy_s"] > 0 else None,
                  "verdicts_match_libsodium": bool((out == expect[a:b]).all())})
        return d

    res = {"set": "%d distinct envelopes, 100 validator keys, 128-384 B statements, 10%% adversarial "
                  "(libsodium-signed and -verified)" % n, "generate_s": gen_s}
    run((0, 2000), 4, 1000, 5000)  # warm-up: lane, staging and the validators' device key tables
    sv.key_cache_wait(0)
    # the overlay posts one main-thread task per verified batch (VerifyMicroBatcher::submitTagged +
    # Options::onBatch; VERDICT r5 next #7: postOnMainThread batching); the *_per_envelope_post shapes keep
    # the round-5 harness (one continuation and one post per envelope) beside them
    res["paced_1k_every_5ms"] = run((2000, 32000), 4, 1000, 5000)
    res["paced_1k_every_5ms_per_envelope_post"] = run((2000, 32000), 4, 1000, 5000, batch_post=0)
    res["paced_1k_every_5ms_burst_wait_20us"] = run((2000, 32000), 4, 1000, 5000, quiet_us=20, max_linger_us=300)
    res["trickle_4_every_200us"] = run((32000, 36000), 4, 4, 200)
    res["flood"] = run((0, n), 4, 0, 0, workers=4)
    res["flood_per_envelope_post"] = run((0, n), 4, 0, 0, workers=4, batch_post=0)
    res["paced_1k_every_5ms_deadline_policy"] = run((36000, 46000), 4, 1000, 5000, policy=1)
    return res


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 20, help="signatures per GPU per step")
    ap.add_argument("--latency-iters", type=int, default=1000)
    ap.add_argument("--cpu-sample", type=int, default=524288)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-host-api", action="store_true")
    ap.add_argument("--no-config1", action="store_true", help="skip the config-1 CPU/host-API block")
    ap.add_argument("--no-config4i", action="store_true", help="skip config 4 through the micro-batcher")
    ap.add_argument("--no-config35", action="store_true",
                    help="skip the config-3 (5000-tx set) and config-5 (64M signatures) blocks")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))

    import torch  # device memory + streams; imported before the engine so both share one HIP runtime
    import torch.distributed as dist

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    sv = importlib.import_module("stellar-core_amd")
    # one process per GPU: rank -> device LOCAL_RANK.  SV_BENCH_SHARE_GPUS=1
    # (rehearsal only) maps ranks onto the visible devices modulo their count.
    if os.environ.get("SV_BENCH_SHARE_GPUS") == "1":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def barrier():
        if world > 1:
            dist.barrier()

    def sync():
        sv.synchronize(local)
        torch.cuda.synchronize(dev)

    n = args.batch
    lo = rank * n
    t_gen = time.perf_counter()
    seeds, msgs = seeds_and_msgs(lo, lo + n)
    d_seed = torch.from_numpy(seeds.copy()).to(dev)
    d_msg = torch.from_numpy(msgs.copy()).to(dev)
    d_pk = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_sig = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    d_verdict = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_bitmap = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    sv.sign_device(local, d_seed.data_ptr(), d_msg.data_ptr(), n, d_pk.data_ptr(), d_sig.data_ptr(), stream)
    sync()
    log("rank %d: dataset [%d, %d) generated on device in %.2fs" % (rank, lo, lo + n, time.perf_counter() - t_gen))

    digest_ok = None
    pk_h = sig_h = None
    if rank == 0:
        pk_h = d_pk.cpu().numpy().reshape(n, 32)
        sig_h = d_sig.cpu().numpy().reshape(n, 64)
        with open(os.path.join(REPO, "tests", "golden", "digests.json")) as f:
            want = json.load(f)
        if str(n) in want:
            stream_bytes = np.concatenate([pk_h, sig_h, msgs.reshape(n, 32)], axis=1).tobytes()
            digest_ok = hashlib.sha256(stream_bytes).hexdigest() == want[str(n)]
            log("dataset digest vs libsodium (%d sigs): %s" % (n, "MATCH" if digest_ok else "MISMATCH"))

    def step():
        sv.verify_device(local, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), n, d_verdict.data_ptr(),
                         d_bitmap.data_ptr(), stream)

    for _ in range(args.warmup):
        step()
    sync()
    barrier()
    sv.kernel_time_reset()
    sv.timing_enable(True)
    sync()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    sv.timing_enable(False)
    k_ms, k_launches, k_sigs = sv.kernel_time(local)
    # every signature of the dataset is valid: all verdict bytes 1 and every
    # full ballot word of the bitmap all-ones
    verdict_count = int(d_verdict.sum(dtype=torch.int64).item())
    full = n // 64
    bitmap_ok = bool((d_bitmap[:full] == -1).all().item())
    verdicts_ok = verdict_count == n and bitmap_ok

    global_digest = None
    if world > 1:
        t = torch.tensor([elapsed, 0.0 if verdicts_ok else 1.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, bad = float(t[0]), float(t[1])
        verdicts_ok = bad == 0.0
        # host gather of every rank's verdict slice (outside the timed region)
        sh = importlib.import_module("stellar-core_amd.sharding")
        full = sh.gather_verdicts(d_verdict.cpu().numpy(), n * world, world, rank)
        global_digest = sh.verdict_digest(full)
    total = n * world * args.steps
    value = total / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    kernel_ms = k_ms / max(1, k_launches)
    kernel_rate = n / (kernel_ms * 1e-3) if kernel_ms > 0 else 0.0

    # host-buffer API over the same 2^20 signatures (rank 0): pinned staging,
    # H2D, kernels and D2H pipelined in 2^18-signature chunks -- what a host
    # caller gets; reported beside the HBM-resident `value`, never as it
    host_api = None
    if rank == 0 and not args.no_host_api:
        msg_h = msgs.reshape(n, 32)
        sv.verify_fixed(pk_h[:4096], sig_h[:4096], msg_h[:4096], 32, device=local)  # warm the staging
        best, ok_all = None, True
        for _ in range(3):
            t1 = time.perf_counter()
            out_h = sv.verify_fixed(pk_h, sig_h, msg_h, 32, device=local)
            dt = time.perf_counter() - t1
            ok_all = ok_all and bool(out_h.all())
            best = dt if best is None else min(best, dt)
        host_api = {"verifies_per_s": n / best, "ms": best * 1e3, "batch": n, "verdicts_ok": ok_all,
                    "path": "sv_ed25519_verify_batch_fixed from pageable host arrays (parallel pack into 2 pinned "
                            "chunk slots, H2D / kernels / D2H on 3 streams)"}

    # single-process multi-GPU (VERDICT r4 missing #2): a stellar-core node is
    # ONE process (ApplicationImpl.cpp:157-190), so production multi-GPU is the
    # engine's own device = -1 sharding (contiguous slices over the device
    # slots, one host thread each, a host gather).  One process (N = 1) that
    # sees G > 1 slots (an 8-GPU node, or SV_DEVICE_MAP rehearsing slots on one
    # card) times a G x 2^20 host batch on 1, 2, 4, 8 slots.
    inproc = None
    if rank == 0 and world == 1 and not args.no_host_api and n == 1 << 20:
        try:
            inproc = in_process_multi_gpu(sv, pk_h, sig_h, msgs.reshape(n, 32))
        except Exception as e:
            holder = {}
            leg_failed(holder, "in_process_multi_gpu", e)
            inproc = holder["in_process_multi_gpu"]

    result = None
    if rank == 0:
        props = torch.cuda.get_device_properties(dev)
        cus = props.multi_processor_count
        peak_mad_per_s = MAD_LANE_OPS_PER_CLK_CU * cus * PEAK_CLOCK_HZ
        achieved = kernel_rate * W_MAD_PER_VERIFY / 1e12
        traffic = None
        prof = {}
        tf = None
        rounds = sorted((f[:-len("_traffic.json")] for f in os.listdir(os.path.join(REPO, "profiles"))
                         if f.endswith("_traffic.json")), reverse=True)
        for rnd in rounds:  # the newest profile measured on this kernel source wins
            cand = os.path.join(REPO, "profiles", rnd + "_traffic.json")
            if os.path.exists(cand):
                try:
                    with open(cand) as f:
                        if json.load(f).get("kernel_source_sha256") == sv.kernel_source_digest():
                            tf = cand
                            break
                except Exception:
                    pass
        tf = tf or os.path.join(REPO, "profiles", "r03_traffic.json")
        if os.path.exists(tf):
            try:
                with open(tf) as f:
                    tj = json.load(f)
                # only when measured on this very kernel source and batch size
                if int(tj.get("batch", -1)) == n and tj.get("kernel_source_sha256") == sv.kernel_source_digest():
                    traffic = tj.get("hbm_bytes_per_launch")
                    prof = {k: tj[k] for k in ("valu_inst_per_verify", "valu_issue_util", "l2_hit_rate",
                                               "kernel_avg_ns", "effective_clock_ghz") if k in tj}
                    prof["source"] = "profiles/%s (rocprofv3 PMC, tools/profile_run.sh)" % os.path.basename(tf)
            except Exception:
                traffic = None
        # hardware multiply-adds the SIMDs issue per verify (tools/madcount.py,
        # SV_MADCOUNT build), when measured on this kernel source
        hw_mads, hw_src = None, None
        mfs = sorted((os.path.join(REPO, "profiles", d, "madcount.json") for d in os.listdir(os.path.join(REPO, "profiles"))
                      if os.path.exists(os.path.join(REPO, "profiles", d, "madcount.json"))), reverse=True)
        for mf in mfs:  # the newest count measured on this kernel source
            try:
                with open(mf) as f:
                    mj = json.load(f)
                if mj.get("kernel_source_sha256") == sv.kernel_source_digest():
                    hw_mads = float(mj["hw_mads_per_verify"])
                    hw_src = ("%s (tools/madcount.py: prep %.0f + main %.0f per verify)"
                              % (os.path.relpath(mf, REPO), mj["prep_mads_per_verify"], mj["main_mads_per_verify"]))
                    break
            except Exception:
                hw_mads = None
        result = {
            "metric": METRIC,
            "value": value,
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: RFC 8032 keypairs/signatures generated on-device from SHA-256 seeds "
                    "(digest-checked against libsodium 1.0.18), 32-byte messages",
            "config": {
                "workload": "BASELINE config 2: 2^20 uniform random valid ed25519 signatures, one batch per GPU "
                            "(N GPUs: contiguous index slices of one global dataset)",
                "batch_per_gpu": n,
                "global_batch": n * world,
                "msg_len": 32,
                "parallelism": "shard%d (contiguous slices, no collective)" % world,
            },
            "verdicts_ok": verdicts_ok,
            "dataset_digest_ok": digest_ok,
            "gathered_verdict_digest": global_digest,
            "kernel": {"ms_per_launch": kernel_ms, "launches": k_launches, "verifies_per_s": kernel_rate},
            "roofline": {
                "bound": "valu-int",
                "achieved": achieved,
                "peak": peak_mad_per_s / 1e12,
                "unit": "T mad32/s",
                "frac": achieved / (peak_mad_per_s / 1e12),
                "traffic": traffic,
                "algorithmic_per_verify": W_MAD_PER_VERIFY,
                # the same peak against the mads the kernels actually issue
                "hw_mads_per_verify": hw_mads,
                "mad_issue_frac": (kernel_rate * hw_mads / peak_mad_per_s) if hw_mads else None,
                "hw_mads_source": hw_src,
                "peak_source": PEAK_SOURCE,
                "frac_vs_survey_nominal_peak": kernel_rate * W_MAD_PER_VERIFY / NOMINAL_PEAK_SURVEY,
                "traffic_unit": "bytes per launch (FETCH_SIZE + WRITE_SIZE)",
                "profiled": prof or None,
                # the same mads against the peak at the clock the chip holds under
                # this load (GRBM_GUI_ACTIVE / 8 / wall in the profile; DVFS)
                "mad_issue_frac_at_profiled_clock": (
                    kernel_rate * hw_mads / (MAD_LANE_OPS_PER_CLK_CU * cus * prof["effective_clock_ghz"] * 1e9)
                    if hw_mads and prof.get("effective_clock_ghz") else None),
            },
        }
        if host_api is not None:
            host_api["frac_of_device_api"] = host_api["verifies_per_s"] / value
            result["host_api"] = host_api
        if inproc is not None:
            result["in_process_multi_gpu"] = inproc

    # ---- latency @1k batch (config 4), rank 0 only
    sodium = load_libsodium() if rank == 0 else None
    if rank == 0 and not args.no_latency:
        try:
            if sodium is not None:
                pks, sigs, lmsgs, expect = scp_latency_set(sodium)
                src = "SCP-sized 128-384 B messages, 100 validators, 10% adversarial (libsodium-signed, libsodium verdicts)"
            else:
                k = 1000
                pks = [pk_h[i].tobytes() for i in range(k)]
                sigs = [sig_h[i].tobytes() for i in range(k)]
                lmsgs = [msgs[32 * i:32 * i + 32].tobytes() for i in range(k)]
                expect = np.ones(k, np.uint8)
                src = "first 1000 of the device dataset (32 B messages; libsodium unavailable for SCP-sized set)"
            pk_a = np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 32)
            sg_a = np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 64)
            # the caller's batch in C-ABI form (message bytes + offsets + lengths),
            # built once: the timed call is what a C++ caller pays per batch
            m_len = np.array([len(m) for m in lmsgs], np.uint32)
            m_off = np.zeros(len(lmsgs), np.uint64)
            m_off[1:] = np.cumsum(m_len[:-1], dtype=np.uint64)
            m_buf = np.frombuffer(b"".join(lmsgs), np.uint8)
            # the timed call is the C-ABI entry point itself, as a C++ caller
            # (Peer.cpp / HerderImpl) makes it: argument pointers prepared once,
            # no Python-binding conversions inside the timed region (those are
            # timed separately as python_binding_p50_ms)
            clib = sv.load_library()
            pk_a, sg_a = np.ascontiguousarray(pk_a), np.ascontiguousarray(sg_a)
            v_out = np.zeros(len(m_len), np.uint8)
            c_args = [ctypes.c_void_p(a.ctypes.data) for a in (pk_a, sg_a, m_buf, m_off, m_len)]
            c_out = ctypes.c_void_p(v_out.ctypes.data)
            c_n = ctypes.c_size_t(len(m_len))
            c_opts = ctypes.byref(sv.sv_opts(ctypes.sizeof(sv.sv_opts), local, 0, 0))

            def timed(iters, traces=None):
                lat = []
                for _ in range(iters):
                    t1 = time.perf_counter()
                    rc = clib.sv_ed25519_verify_batch(c_args[0], c_args[1], c_args[2], c_args[3], c_args[4], c_n, c_out,
                                                      c_opts)
                    lat.append((time.perf_counter() - t1) * 1e3)
                    if rc != 0:
                        raise RuntimeError("sv_ed25519_verify_batch: %d" % rc)
                    if traces is not None:
                        traces.append(sv.lat_last_trace())
                return np.array(lat), v_out.copy()

            def timed_py(iters):
                lat = []
                for _ in range(iters):
                    t1 = time.perf_counter()
                    sv.verify_batch(pk_a, sg_a, m_buf, m_off, m_len, device=local)
                    lat.append((time.perf_counter() - t1) * 1e3)
                return np.array(lat)

            def slow_iterations(lat, traces):
                # every iteration above 2x p50 with the engine's host-side stages
                # (sv_lat_last_trace): which stage the time went to
                p50 = float(np.percentile(lat, 50))
                slow = [i for i in range(len(lat)) if lat[i] > 2 * p50]
                med = {k: float(np.median([t[k] for t in traces])) for k in sv.LAT_TRACE_FIELDS}
                return {"count": len(slow), "of": len(lat), "median_stages_us": med,
                        "iterations": [dict(index=i, ms=float(lat[i]), **{k: round(v, 1) for k, v in traces[i].items()})
                                       for i in slow[:20]]}

            # steady state of an SCP flood: the validators' key tables are built
            # (low-priority stream) after the first batch, then every batch runs
            # the warm-key comb kernel
            for _ in range(3):
                sv.verify_batch(pk_a, sg_a, m_buf, m_off, m_len, device=local)
            sv.key_cache_wait(local)
            timed(5)
            st0 = sv.key_cache_stats(local)
            tr_w = []
            lat, out = timed(args.latency_iters, tr_w)
            st1 = sv.key_cache_stats(local)
            lat_py = timed_py(200)
            warm = st1["warm_batches"] - st0["warm_batches"]
            # cold keys: key cache off (every batch on the octet kernel, no per-key state)
            cap0 = st1["capacity"]
            sv.set_key_cache(0)
            timed(5)
            tr_c = []
            lat_c, out_c = timed(args.latency_iters, tr_c)
            sv.set_key_cache(cap0)
            result["latency_1k"] = {
                "batch": len(pks),
                "p50_ms": float(np.percentile(lat, 50)),
                "p99_ms": float(np.percentile(lat, 99)),
                "iters": args.latency_iters,
                "key_cache": "warm: %d of %d timed batches ran the comb kernel (100 validator keys cached after the "
                             "first batch; csrc/comb.h)" % (warm, args.latency_iters),
                "path": "C-ABI sv_ed25519_verify_batch called directly (ctypes, pointers prepared once), one call per "
                        "batch on the slot's latency lane (pack into pinned staging + H2D + kernel writing verdicts into "
                        "mapped pinned memory + sync)",
                "python_binding_p50_ms": float(np.percentile(lat_py, 50)),
                "set": src,
                "verdicts_match_libsodium": bool((out == expect).all()),
                "slow_iterations": slow_iterations(lat, tr_w),
            }
            result["latency_1k_cold_keys"] = {
                "p50_ms": float(np.percentile(lat_c, 50)),
                "p99_ms": float(np.percentile(lat_c, 99)),
                "iters": args.latency_iters,
                "key_cache": "off (sv_set_key_cache(0)): the octet kernel, no per-key state -- what a batch of "
                             "never-seen keys gets",
                "verdicts_match_libsodium": bool((out_c == expect).all()),
                "slow_iterations": slow_iterations(lat_c, tr_c),
            }
            spath_l = sodium_path() if sodium is not None else None
            if spath_l is not None and not args.no_cpu:
                thr, _ = host_cpus()
                one, o1 = cpu_batch_latency(spath_l, pk_a, sg_a, m_buf, m_off, m_len, 1, 5)
                allc, o2 = cpu_batch_latency(spath_l, pk_a, sg_a, m_buf, m_off, m_len, thr, 21)
                result["latency_1k"]["cpu_libsodium"] = {
                    "p50_ms_1thread": one, "p50_ms_all_cores": allc, "threads": thr,
                    "verdicts_match": bool((o1 == expect).all() and (o2 == expect).all()),
                    "what": "the same 1000-signature set, one libsodium crypto_sign_verify_detached per signature "
                            "(oracle/cpu_baseline.c cpubase_sodium_batch, static partition over pthreads)"}

            if sodium is not None and not args.no_config4i:
                t_c = time.perf_counter()
                result["config4_integrated"] = config4_integrated(sv, sodium)
                log("config 4 through the micro-batcher in %.1fs" % (time.perf_counter() - t_c))

            # the bulk configurations below run outside the latency lane's
            # shared-mode window (SV_LAT_SHARE_MS, csrc/sv_api.cpp share_now)
            time.sleep(1.1)
        except Exception as e:  # (rank 0's optional legs: recorded, never the whole line)
            leg_failed(result, 'latency_1k', e)

    # ---- CPU baseline (rank 0, every N: after the timed region and its final
    # barrier, on the host cores of this job; the other ranks wait at the next
    # collective)
    if rank == 0 and not args.no_cpu:
        try:
            threads, cpu_info = host_cpus()
            spath = sodium_path() if sodium is not None else None
            if spath is not None:
                kind = "reference"
                sample = min(args.cpu_sample, n)
                st_sample = min(16384, n)
                desc = "libsodium %s crypto_sign_verify_detached (dlopen %s), first %d signatures of the bench dataset" % (
                    sodium.sodium_version_string().decode(), spath, sample)
            else:
                kind = "port"
                sample = min(8192, n)
                st_sample = min(1024, n)
                desc = "oracle/ C restatement (libsodium unavailable), first %d signatures" % sample
            rate, dt, out = cpu_verify_rate(pk_h[:sample], sig_h[:sample], msgs[:32 * sample], 32, threads, spath)
            rate1, dt1, out1 = cpu_verify_rate(pk_h[:st_sample], sig_h[:st_sample], msgs[:32 * st_sample], 32, 1, spath)
            result["cpu_baseline"] = {
                "value": rate,
                "unit": "verifies/s",
                "cores": threads,
                "kind": kind,
                "sample": desc + " (%.2f s wall on %d pthreads, static contiguous partition; native harness "
                                 "oracle/cpu_baseline.c)" % (dt, threads),
                "single_thread_value": rate1,
                "host_cpus": cpu_info,
                "cpu_verdicts_all_valid": bool(out.all() and out1.all()),
                "gpu_over_cpu": value / rate if rate > 0 else None,
            }
            if spath is not None and not args.no_config1:
                t_c1 = time.perf_counter()
                result["config1"] = config1(sv, sodium, spath, pk_h, sig_h, msgs, threads, local)
                log("config 1 (both shapes) in %.1fs" % (time.perf_counter() - t_c1))
        except Exception as e:  # (rank 0's optional legs: recorded, never the whole line)
            leg_failed(result, 'cpu_baseline', e)
    if not args.no_config35 and n == 1 << 20 and 64 % world == 0:
        t_c = time.perf_counter()
        c5 = config5(sv, torch, dev, stream, local, d_pk, d_sig, d_msg, n, world, rank, barrier, dist)
        if rank == 0:
            result["config5"] = c5
            log("config 5 (64M signatures on %d GPU(s)) in %.1fs" % (world, time.perf_counter() - t_c))
    if rank == 0 and not args.no_config35 and n == 1 << 20:
        t_c = time.perf_counter()
        try:
            result["config3"] = config3()
        except Exception as e:
            leg_failed(result, "config3", e)
        log("config 3 (5000-tx set) in %.1fs" % (time.perf_counter() - t_c))

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
