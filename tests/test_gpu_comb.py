"""GPU parity of the warm-key latency path (csrc/sv_comb.hip, csrc/comb.h).

A latency-path host batch whose public keys are all in the device's key cache
runs the comb kernel; every other batch runs the octet kernel and queues its
keys for a table build.  Both must give libsodium's verdict on every row:
  * every golden fixture class (reference in-tree vectors, libsodium-signed
    valid rows, message lengths 0..512, every adversarial class including
    small-order / non-canonical / off-curve keys, which the cache records as
    rejecting keys), first cold, then warm;
  * an SCP-shaped set (100 validator keys, 0..400-byte messages, mutated rows)
    at sizes that select each kernel geometry (1, 2 and 4 signatures per
    chain wave), against the oracle;
  * eviction: a cache smaller than the key set still gives exact verdicts;
  * batches from several threads at once (two run side by side on the lane),
    with eviction churn and warm;
  * the staged-copy lane (SV_LAT_ZC_IN=0 / SV_LAT_ZERO_COPY=0: one H2D of the
    image, one D2H of the verdicts) gives the same verdicts as the default
    (kernels read the image and write the verdicts in mapped memory);
  * the same staged fallbacks for keyed lane batches (keys D2H instead of
    written in mapped memory) and for one-chunk bulk batches (SV_BULK_ZC_IN=0:
    staged H2D instead of the image read in place), keyed, unkeyed and through
    the pieced progress path, verdicts and BLAKE2b keys exact.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from scp_sets import scp_set as _scp_set

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(sv):
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    return 0


@pytest.fixture
def cache(sv, gpu):
    sv.set_key_cache(8192)
    yield sv
    sv.set_key_cache(1024)


def _run(sv, d, rows=None):
    pk, sig, off, ln = d["pk"], d["sig"], d["msg_off"], d["msg_len"]
    if rows is not None:
        pk, sig, off, ln = pk[rows], sig[rows], off[rows], ln[rows]
    return sv.verify_batch(pk, sig, d["msg"], off, ln, device=0, path="latency")


def _warm_up(sv, d, want, rounds=16):
    """Runs the batch until it is served warm; every run must be exact."""
    for r in range(rounds):
        w0 = sv.key_cache_stats(0)["warm_batches"]
        out = _run(sv, d)
        assert (out == want).all(), "round %d: %s" % (r, np.nonzero(out != want)[0][:10])
        if sv.key_cache_stats(0)["warm_batches"] == w0 + 1:
            return r
        sv.key_cache_wait(0)
    raise AssertionError("batch never ran warm: %s" % sv.key_cache_stats(0))


@pytest.mark.parametrize("name", ["intree", "valid", "msglen", "adversarial", "lattice_edge"])
def test_golden_fixtures_warm(sv, cache, golden, name):
    d = golden[name]
    r = _warm_up(sv, d, d["verdict"])
    assert r >= 1  # (the first run is cold: its keys were unknown)
    out = _run(sv, d)  # warm again
    bad = np.nonzero(out != d["verdict"])[0]
    assert len(bad) == 0, [(int(i), str(d["class_names"][d["cls"][i]])) for i in bad[:10]]


@pytest.mark.parametrize("n", [1, 7, 500, 1200, 3000])
def test_scp_set_geometries(sv, cache, oracle, n):
    """n = 1..768 runs 1 signature per chain wave, up to 1536 two, above four
    (sv_comb_spw); tails of the last workgroup are exercised by odd n."""
    d = _scp_set(oracle, n, seed=n)
    assert 0 < int(d["verdict"].sum()) <= n
    _warm_up(sv, d, d["verdict"])
    out = _run(sv, d)
    assert (out == d["verdict"]).all()


def test_fixed32_messages_warm(sv, cache, golden):
    """The fixed-length entry point (32-byte tx hashes, MODE 0) on the comb kernel."""
    d = golden["valid"]
    rows = np.nonzero(d["msg_len"] == 32)[0]
    assert len(rows) > 100
    msg = np.stack([d["msg"][int(d["msg_off"][i]):int(d["msg_off"][i]) + 32] for i in rows])
    pk, sig = d["pk"][rows], d["sig"][rows]
    for _ in range(8):
        w0 = sv.key_cache_stats(0)["warm_batches"]
        out = sv.verify_fixed(pk, sig, msg, 32, device=0, path="latency")
        assert out.all()
        if sv.key_cache_stats(0)["warm_batches"] == w0 + 1:
            break
        sv.key_cache_wait(0)
    else:
        raise AssertionError("never warm")
    sig2 = sig.copy()
    sig2[::3, 40] ^= 4
    out = sv.verify_fixed(pk, sig2, msg, 32, device=0, path="latency")
    want = np.ones(len(rows), np.uint8)
    want[::3] = 0
    assert (out == want).all()


@pytest.mark.parametrize("mlen", [1, 100, 497, 600])
def test_fixed_other_length_messages_warm(sv, cache, oracle, mlen):
    """Fixed-length messages other than 32 bytes (MODE 2) on the comb kernel:
    windows starting at several alignments (100: multiples of 4 mod 16; 497:
    every alignment, filling up to all 32 quads of the 512-byte window), 1
    and 600 (no window: hashed from memory)."""
    import ctypes
    rng = np.random.default_rng(mlen)
    keys = []
    for _ in range(20):
        pkb, skb = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
        oracle.oracle_ed25519_seed_keypair(pkb, skb, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        keys.append((pkb.raw, skb.raw))
    n = 240
    pk = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    msg = rng.integers(0, 256, (n, mlen), dtype=np.uint8)
    for i in range(n):
        pkb, skb = keys[i % 20]
        sb = ctypes.create_string_buffer(64)
        oracle.oracle_ed25519_sign(sb, msg[i].tobytes(), mlen, skb)
        pk[i] = np.frombuffer(pkb, np.uint8)
        sig[i] = np.frombuffer(sb.raw, np.uint8)
    want = np.ones(n, np.uint8)
    sig[::7, 33] ^= 0x10  # S bit
    want[::7] = 0
    msg[3::11, mlen - 1] ^= 0x01  # last message byte
    want[3::11] = 0
    for _ in range(8):
        w0 = sv.key_cache_stats(0)["warm_batches"]
        out = sv.verify_fixed(pk, sig, msg, mlen, device=0, path="latency")
        assert (out == want).all(), np.nonzero(out != want)[0][:10]
        if sv.key_cache_stats(0)["warm_batches"] == w0 + 1:
            break
        sv.key_cache_wait(0)
    else:
        raise AssertionError("never warm")


def test_small_cache_evicts_exactly(sv, gpu, oracle):
    """A 64-key cache under a 100-key workload keeps evicting; verdicts stay
    exact whichever kernel serves each batch."""
    sv.set_key_cache(64)
    try:
        for seed in range(6):
            d = _scp_set(oracle, 300, seed=1000 + seed)
            for _ in range(2):
                out = _run(sv, d)
                assert (out == d["verdict"]).all()
                sv.key_cache_wait(0)
        st = sv.key_cache_stats(0)
        assert st["capacity"] == 64 and st["keys"] <= 64
        assert st["evictions"] > 0
    finally:
        sv.set_key_cache(1024)


@pytest.mark.parametrize("cap", [64, 8192])
def test_concurrent_lane_batches(sv, gpu, oracle, cap):
    """Batches from several host threads at once: the lane plans and launches
    them one at a time but runs up to two side by side (sv_api.cpp LatCtx).
    With a 64-key cache under a 600-key workload every batch evicts and queues
    table builds while the other context's comb kernel reads the tables; with a
    large one the same sets run warm side by side.  Every verdict exact."""
    import threading
    sets = [_scp_set(oracle, 200 + 37 * k, seed=2000 + k) for k in range(6)]
    sv.set_key_cache(cap)
    errors = []
    try:
        def worker(t):
            try:
                for it in range(10):
                    d = sets[(t * 5 + it) % len(sets)]
                    out = _run(sv, d)
                    bad = np.nonzero(out != d["verdict"])[0]
                    if len(bad):
                        errors.append((t, it, bad[:5].tolist()))
            except Exception as e:  # (reported below, not swallowed)
                errors.append((t, repr(e)))
        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:5]
        st = sv.key_cache_stats(0)
        assert st["warm_batches"] + st["cold_batches"] >= 40
        if cap == 64:
            assert st["evictions"] > 0
    finally:
        sv.set_key_cache(1024)


def test_device_and_host_lane_batches_concurrent(sv, gpu, oracle):
    """Device-API lane batches (queued on a free context, not waited for) from
    one thread while host lane batches run on the contexts from two others:
    stream order keeps each context's work apart, every verdict exact."""
    import threading
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    n = 3000
    rng = np.random.default_rng(77)
    seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(dev)
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), n, pk.data_ptr(), sig.data_ptr(), st)
    torch.cuda.synchronize(dev)
    sig[::5, 40] ^= 0x08
    want_d = np.ones(n, np.uint8)
    want_d[::5] = 0
    sets = [_scp_set(oracle, 400 + 50 * k, seed=3000 + k) for k in range(3)]
    errors = []

    def device_worker():
        try:
            s = torch.cuda.Stream(dev)
            out = torch.zeros(n, dtype=torch.uint8, device=dev)
            for it in range(12):
                with torch.cuda.stream(s):
                    out.zero_()
                    sv.verify_device(0, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), n, out.data_ptr(), 0,
                                     s.cuda_stream)
                s.synchronize()
                got = out.cpu().numpy()
                if not np.array_equal(got, want_d):
                    errors.append(("device", it, np.nonzero(got != want_d)[0][:5].tolist()))
        except Exception as e:
            errors.append(("device", repr(e)))

    def host_worker(t):
        try:
            for it in range(10):
                d = sets[(t + it) % len(sets)]
                out = _run(sv, d)
                if not (out == d["verdict"]).all():
                    errors.append(("host", t, it))
        except Exception as e:
            errors.append(("host", t, repr(e)))

    th = [threading.Thread(target=device_worker)] + [threading.Thread(target=host_worker, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]


def test_cache_off_is_octet_only(sv, gpu, golden):
    sv.set_key_cache(0)
    try:
        d = golden["adversarial"]
        w0 = sv.key_cache_stats(0)["warm_batches"]
        for _ in range(3):
            assert (_run(sv, d) == d["verdict"]).all()
        assert sv.key_cache_stats(0)["warm_batches"] == w0
    finally:
        sv.set_key_cache(1024)


@pytest.mark.parametrize("flags", ["none", "trivial_pair", "max_windows"])
@pytest.mark.parametrize("n", [700, 3000])
def test_cold_three_wave_splits(sv, gpu, golden, n, flags):
    """Cold latency batches of <= 4096 signatures take the three-wave octet
    kernel (SV_OCT_HI_MAX): the high wave starts from the decoded points
    through LDS hand-overs and takes W / 6 of the windows, or W / 4 above
    2048 signatures (SV_KP_OCT_HI_WIDE).  Both splits, with the forced
    fallback pair and 64 windows (W up to 64), against the golden verdicts."""
    f = {"none": 0, "trivial_pair": sv.DBG_TRIVIAL_PAIR, "max_windows": sv.DBG_MAX_WINDOWS}[flags]
    a, e = golden["adversarial"], golden["lattice_edge"]
    rows_a = np.arange(n) % len(a["verdict"])
    rows_e = np.arange(n) % len(e["verdict"])
    sv.set_key_cache(0)
    prev = sv.set_debug_flags(f)
    try:
        for d, rows in ((a, rows_a), (e, rows_e)):
            out = _run(sv, d, rows)
            bad = np.nonzero(out != d["verdict"][rows])[0]
            assert len(bad) == 0, [(int(i), str(d["class_names"][d["cls"][rows[i]]])) for i in bad[:10]]
    finally:
        sv.set_debug_flags(prev)
        sv.set_key_cache(1024)


def _mirror(sv):
    import ctypes
    lib = ctypes.CDLL(sv.HOSTLIB_PATH)
    lib.svh_last_error_string.restype = ctypes.c_char_p
    lib.svh_set_cpu_threshold.argtypes = [ctypes.c_size_t]
    lib.svh_set_keyed_threshold.argtypes = [ctypes.c_size_t]
    return lib


def _mirror_stats(host):
    import ctypes

    class EngineStats(ctypes.Structure):
        _fields_ = [("gpu_signatures", ctypes.c_uint64), ("gpu_batches", ctypes.c_uint64),
                    ("cpu_signatures", ctypes.c_uint64), ("fallbacks", ctypes.c_uint64)]
    s = EngineStats()
    host.svh_engine_counts_ex(ctypes.byref(s))
    h, m = ctypes.c_uint64(), ctypes.c_uint64()
    host.svh_cache_counts(ctypes.byref(h), ctypes.byref(m))
    return s, h.value, m.value


def _mirror_batch(host, d, rows):
    import ctypes
    pk, sig = np.ascontiguousarray(d["pk"][rows]), np.ascontiguousarray(d["sig"][rows])
    off, ln = np.ascontiguousarray(d["msg_off"][rows]), np.ascontiguousarray(d["msg_len"][rows])
    msg = np.ascontiguousarray(d["msg"])
    out = np.full(len(rows), 7, np.uint8)
    vp = ctypes.c_void_p
    rc = host.svh_verify_sig_batch(vp(pk.ctypes.data), vp(sig.ctypes.data), None, vp(msg.ctypes.data),
                                   vp(off.ctypes.data), vp(ln.ctypes.data), ctypes.c_size_t(len(rows)),
                                   vp(out.ctypes.data))
    assert rc == 0, host.svh_last_error_string()
    return out


@pytest.mark.parametrize("n", [64, 300])
def test_cold_three_wave_lost_handover_is_an_error(sv, gpu, golden, n):
    """A hand-over flag that never comes (SV_DBG_DROP_HANDOVER: the decode wave
    does not raise the tables' flag) ends the verify wave's bounded wait
    (~0.5 s).  The kernel writes fail-closed rejects AND raises the launch's
    failure word, so the C-ABI returns SV_ERR_KERNEL instead of rejects
    (include/stellar_sigverify.h: an error is never a reject).  The C++ mirror's
    verifySigBatch over the same valid rows (n = 64: host-hashed miss batch;
    n = 300: the keyed pass, whose cache walk has already run when the error
    comes back) re-runs them on the CPU path: all true, one fallback, no GPU
    signature counted, and no false verdict enters the verify cache -- the
    same rows afterwards are all cache hits, all true
    (/root/reference/src/crypto/SecretKey.cpp:446-466)."""
    import time
    d = golden["valid"]
    rows = np.arange(n)
    assert d["verdict"][rows].all()
    host = _mirror(sv)
    sv.set_key_cache(0)
    host.svh_set_cpu_threshold(0)
    host.svh_set_keyed_threshold(256)
    host.svh_cache_clear()
    _mirror_stats(host)
    prev = sv.set_debug_flags(sv.DBG_DROP_HANDOVER)
    try:
        t = time.perf_counter()
        with pytest.raises(sv.SigVerifyError, match="SV_ERR_KERNEL"):
            _run(sv, d, rows)
        assert 0.1 < time.perf_counter() - t < 30  # (the bounded wait ran)
        out = _mirror_batch(host, d, rows)
        assert out.all()
        s, hits, misses = _mirror_stats(host)
        assert s.fallbacks == 1 and s.gpu_signatures == 0 and s.cpu_signatures == n, (
            s.fallbacks, s.gpu_signatures, s.cpu_signatures)
        assert hits == 0 and misses == n
    finally:
        sv.set_debug_flags(prev)
        host.svh_set_cpu_threshold(1)
        sv.set_key_cache(1024)
    try:
        out = _mirror_batch(host, d, rows)
        assert out.all()
        s, hits, misses = _mirror_stats(host)
        assert hits == n and misses == 0 and s.fallbacks == 0
    finally:
        host.svh_cache_clear()
    # and the next cold launch is exact again
    sv.set_key_cache(0)
    try:
        assert (_run(sv, d, rows) == 1).all()
    finally:
        sv.set_key_cache(1024)


_STAGED_CHILD = r"""
import ctypes, os, sys
import numpy as np
import torch  # noqa: F401  (the HIP runtime torch ships, as in the parent)
z = np.load(sys.argv[2], allow_pickle=False)
lib = ctypes.CDLL(os.path.join(sys.argv[1], "stellar-core_amd", "libstellar_sigverify.so"))
class Opts(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("device", ctypes.c_int32), ("max_devices", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]
opts = Opts(ctypes.sizeof(Opts), 0, 0, 0x2)  # SV_FLAG_PATH_LATENCY
arrs = [np.ascontiguousarray(z[k]) for k in ("pk", "sig", "msg", "msg_off", "msg_len")]
n = len(arrs[4])
assert lib.sv_init() == 0
outs = []
for it in range(12):  # cold first, warm once the keys are built
    out = np.zeros(n, np.uint8)
    rc = lib.sv_ed25519_verify_batch(*[ctypes.c_void_p(a.ctypes.data) for a in arrs], ctypes.c_size_t(n),
                                     ctypes.c_void_p(out.ctypes.data), ctypes.byref(opts))
    assert rc == 0, rc
    outs.append(out)
    if it == 1:
        assert lib.sv_key_cache_wait(0) == 0
np.save(sys.argv[3], np.stack(outs))
"""


def test_staged_copy_lane_matches(sv, gpu, oracle, tmp_path):
    """The lane with its staged copies (env switches read once per process,
    hence a child process) against the oracle, cold and warm."""
    d = _scp_set(oracle, 1000, seed=77)
    src = tmp_path / "set.npz"
    np.savez(src, pk=d["pk"], sig=d["sig"], msg=d["msg"], msg_off=d["msg_off"].astype(np.uint64),
             msg_len=d["msg_len"].astype(np.uint32))
    dst = tmp_path / "out.npy"
    env = dict(os.environ, SV_LAT_ZC_IN="0", SV_LAT_ZERO_COPY="0")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _STAGED_CHILD, repo, str(src), str(dst)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    outs = np.load(dst, allow_pickle=False)
    for it, out in enumerate(outs):
        assert (out == d["verdict"]).all(), (it, np.nonzero(out != d["verdict"])[0][:10])


_STAGED_KEYED_CHILD = r"""
import ctypes, os, sys
import numpy as np
import torch  # noqa: F401  (the HIP runtime torch ships, as in the parent)
z = np.load(sys.argv[2], allow_pickle=False)
lib = ctypes.CDLL(os.path.join(sys.argv[1], "stellar-core_amd", "libstellar_sigverify.so"))
class Opts(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("device", ctypes.c_int32), ("max_devices", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]
vp = ctypes.c_void_p
arrs = [np.ascontiguousarray(z[k]) for k in ("pk", "sig", "msg", "msg_off", "msg_len")]
n = len(arrs[4])
assert lib.sv_init() == 0
res = {}
for name, flags in (("lane", 0x2), ("bulk", 0x1)):
    opts = Opts(ctypes.sizeof(Opts), 0, 0, flags)
    for it in range(3):
        out = np.zeros(n, np.uint8)
        keys = np.zeros((n, 32), np.uint8)
        rc = lib.sv_ed25519_verify_batch_keyed(*[vp(a.ctypes.data) for a in arrs], ctypes.c_size_t(n),
                                               vp(out.ctypes.data), vp(keys.ctypes.data), ctypes.byref(opts))
        assert rc == 0, rc
        res["%s_keyed_%d_v" % (name, it)] = out
        res["%s_keyed_%d_k" % (name, it)] = keys
        out = np.zeros(n, np.uint8)
        rc = lib.sv_ed25519_verify_batch(*[vp(a.ctypes.data) for a in arrs], ctypes.c_size_t(n),
                                         vp(out.ctypes.data), ctypes.byref(opts))
        assert rc == 0, rc
        res["%s_plain_%d_v" % (name, it)] = out
# the pieced progress path: a one-chunk keyed bulk batch with a keys-ready
# callback (keys come back in pieces while the GPU verifies), 12x the set
reps = 12
m = n * reps
msg = arrs[2]
P = lambda a, stride, k: (ctypes.c_void_p * m)(*[a.ctypes.data + stride * (i % n) for i in range(m)])
ppk, psig = P(arrs[0], 32, 0), P(arrs[1], 64, 0)
pmsg = (ctypes.c_void_p * m)(*[msg.ctypes.data + int(arrs[3][i % n]) for i in range(m)])
plen = np.ascontiguousarray(np.tile(arrs[4], reps))
seen = []
CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_size_t)
cb = CB(lambda ctx, ready: seen.append(ready))
out = np.zeros(m, np.uint8)
keys = np.zeros((m, 32), np.uint8)
opts = Opts(ctypes.sizeof(Opts), 0, 0, 0x1)
rc = lib.sv_ed25519_verify_batch_gather_progress(ppk, psig, pmsg, vp(plen.ctypes.data), ctypes.c_size_t(m),
                                                  vp(out.ctypes.data), vp(keys.ctypes.data), cb, None,
                                                  ctypes.byref(opts))
assert rc == 0, rc
assert seen and seen[-1] == m and seen == sorted(seen), seen
res["pieced_pieces"] = np.array([len(seen)])
res["pieced_v"] = out
res["pieced_k"] = keys
np.savez(sys.argv[3], **res)
"""


@pytest.mark.parametrize("variant", ["staged", "alternates"])
def test_staged_fallbacks_keyed_and_bulk(sv, gpu, oracle, tmp_path, variant):
    """staged: SV_LAT_ZC_IN=0, SV_LAT_ZERO_COPY=0 and SV_BULK_ZC_IN=0 (the
    staged fallbacks); alternates: one lane context (SV_LAT_CONTEXTS=1), the
    two-wave cold octet kernel (SV_OCT_HI_MAX=0) and copied bulk verdicts
    (SV_BULK_ZC_OUT=0).  Env switches are read once per process, hence a
    child: keyed and unkeyed lane and one-chunk bulk batches, and the pieced
    progress path, against the oracle's verdicts and hashlib's BLAKE2b-256 keys."""
    import hashlib
    d = _scp_set(oracle, 1000, seed=78)
    src = tmp_path / "set.npz"
    np.savez(src, pk=d["pk"], sig=d["sig"], msg=d["msg"], msg_off=d["msg_off"].astype(np.uint64),
             msg_len=d["msg_len"].astype(np.uint32))
    dst = tmp_path / "out.npz"
    env = dict(os.environ, **({"SV_LAT_ZC_IN": "0", "SV_LAT_ZERO_COPY": "0", "SV_BULK_ZC_IN": "0"} if variant == "staged"
                              else {"SV_LAT_CONTEXTS": "1", "SV_OCT_HI_MAX": "0", "SV_BULK_ZC_OUT": "0"}))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _STAGED_KEYED_CHILD, repo, str(src), str(dst)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = dict(np.load(dst, allow_pickle=False))
    n = len(d["verdict"])
    want_k = np.zeros((n, 32), np.uint8)
    for i in range(n):
        o, ln = int(d["msg_off"][i]), int(d["msg_len"][i])
        want_k[i] = np.frombuffer(hashlib.blake2b(d["pk"][i].tobytes() + d["sig"][i].tobytes()
                                                  + d["msg"][o:o + ln].tobytes(), digest_size=32).digest(), np.uint8)
    for k, v in res.items():
        if k.endswith("_v"):
            reps = len(v) // n
            assert (v == np.tile(d["verdict"], reps)).all(), k
        elif k.endswith("_k"):
            reps = len(v) // n
            assert (v == np.tile(want_k, (reps, 1))).all(), k
    assert res["pieced_pieces"][0] >= 2
