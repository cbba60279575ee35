"""C++ host mirror of the reference's verification callers (libstellar_host.so).

CPU tests: the engine is replaced by the oracle through the library's test
hook (svh_set_test_verifier, the analogue of the reference's BUILD_TESTS
doubles, SignatureChecker.h:41-63), so the cache / size-64 / counter
semantics of PubKeyUtils::verifySig (SecretKey.cpp:435-468) and the greedy
SignatureChecker logic (SignatureChecker.cpp:30-158) are checked without a GPU.
The GPU variants at the bottom run the same checks through the real engine.
"""
import ctypes
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import txset_gen as tg
from conftest import REPO

VERIFY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


@pytest.fixture(scope="module")
def host(sv):
    path = sv.HOSTLIB_PATH
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-j4"], cwd=os.path.join(REPO, "stellar-core_amd"), check=True)
    lib = ctypes.CDLL(path)
    lib.svh_verify_sig.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                   ctypes.c_size_t]
    lib.svh_last_error_string.restype = ctypes.c_char_p
    lib.svh_set_test_verifier.argtypes = [ctypes.c_void_p]
    lib.svh_set_test_keyed_verifier.argtypes = [ctypes.c_void_p]
    lib.svh_set_keyed_threshold.argtypes = [ctypes.c_size_t]
    lib.svh_set_cpu_threshold.argtypes = [ctypes.c_size_t]
    lib.svh_cache_keys.restype = ctypes.c_size_t
    lib.svh_cache_seed.argtypes = [ctypes.c_uint]
    lib.svh_scp_run.restype = ctypes.c_int
    return lib


class OracleEngine:
    """Batch verifier callback backed by the oracle; counts calls."""

    def __init__(self, oracle):
        self.oracle = oracle
        self.calls = 0
        self.sigs = 0

        def fn(pk, sig, msg, off, ln, n, out):
            self.calls += 1
            self.sigs += n
            pkb = ctypes.string_at(pk, 32 * n)
            sgb = ctypes.string_at(sig, 64 * n)
            offs = np.ctypeslib.as_array(ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64)), (n,))
            lens = np.ctypeslib.as_array(ctypes.cast(ln, ctypes.POINTER(ctypes.c_uint32)), (n,))
            res = np.ctypeslib.as_array(ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8)), (n,))
            for i in range(n):
                m = ctypes.string_at(msg + int(offs[i]), int(lens[i])) if lens[i] else b""
                res[i] = 1 if oracle.oracle_ed25519_verify(sgb[64 * i:64 * i + 64], m, len(m),
                                                           pkb[32 * i:32 * i + 32]) == 0 else 0
            return 0

        self.fn_plain = fn
        self.cfn = VERIFY_FN(fn)


KEYED_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p)


class OracleKeyedEngine(OracleEngine):
    """Keyed engine stand-in (f4): oracle verdicts + hashlib BLAKE2b-256 keys."""

    def __init__(self, oracle):
        super().__init__(oracle)

        def kfn(pk, sig, msg, off, ln, n, out, keys):
            self.fn_plain(pk, sig, msg, off, ln, n, out)
            offs = np.ctypeslib.as_array(ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64)), (n,))
            lens = np.ctypeslib.as_array(ctypes.cast(ln, ctypes.POINTER(ctypes.c_uint32)), (n,))
            kb = np.ctypeslib.as_array(ctypes.cast(keys, ctypes.POINTER(ctypes.c_uint8)), (n * 32,))
            for i in range(n):
                m = ctypes.string_at(msg + int(offs[i]), int(lens[i])) if lens[i] else b""
                d = hashlib.blake2b(ctypes.string_at(pk + 32 * i, 32) + ctypes.string_at(sig + 64 * i, 64) + m,
                                    digest_size=32).digest()
                kb[32 * i:32 * i + 32] = np.frombuffer(d, np.uint8)
            return 0

        self.kcfn = KEYED_FN(kfn)


@pytest.fixture()
def engine(host, oracle):
    e = OracleEngine(oracle)
    host.svh_set_test_verifier(ctypes.cast(e.cfn, ctypes.c_void_p))
    host.svh_cache_clear()
    host.svh_cache_counts(None, None)
    host.svh_engine_counts(None, None)
    yield e
    host.svh_set_test_verifier(None)
    host.svh_cache_clear()


def _counts(host):
    h, m = ctypes.c_uint64(), ctypes.c_uint64()
    host.svh_cache_counts(ctypes.byref(h), ctypes.byref(m))
    return h.value, m.value


def test_blake2b256_and_sha256_match_hashlib(host):
    out = ctypes.create_string_buffer(32)
    rng = np.random.default_rng(3)
    for n in [0, 1, 3, 64, 127, 128, 129, 255, 256, 257, 1000]:
        b = rng.bytes(n)
        host.svh_blake2b256(out, b, ctypes.c_size_t(n))
        assert out.raw == hashlib.blake2b(b, digest_size=32).digest(), n
        host.svh_sha256(out, b, ctypes.c_size_t(n))
        assert out.raw == hashlib.sha256(b).digest(), n


def test_blake2b256_without_avx512_matches_hashlib():
    """The AVX2 / scalar compression (hosts without AVX-512VL) in a process
    that opts out of the AVX-512 path (SVH_NO_AVX512)."""
    import subprocess
    import sys
    code = (
        "import ctypes, hashlib, os\n"
        "lib = ctypes.CDLL(%r)\n"
        "out = ctypes.create_string_buffer(32)\n"
        "for n in (0, 1, 127, 128, 129, 256, 352, 1000):\n"
        "    b = bytes((i * 131 + n) & 255 for i in range(n))\n"
        "    lib.svh_blake2b256(out, b, ctypes.c_size_t(n))\n"
        "    assert out.raw == hashlib.blake2b(b, digest_size=32).digest(), n\n"
        % os.path.join(REPO, "stellar-core_amd", "libstellar_host.so"))
    env = dict(os.environ, SVH_NO_AVX512="1")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=120)


def test_verify_sig_cache_semantics(host, engine, golden):
    d = golden["valid"]
    pk, sig = d["pk"][0].tobytes(), d["sig"][0].tobytes()
    o, ln = int(d["msg_off"][0]), int(d["msg_len"][0])
    m = d["msg"][o:o + ln].tobytes()
    assert host.svh_verify_sig(pk, sig, 64, m, len(m)) == 1       # miss -> engine
    assert host.svh_verify_sig(pk, sig, 64, m, len(m)) == 1       # hit
    bad = bytearray(sig)
    bad[4] ^= 1                                                   # CryptoTests.cpp:292-296
    assert host.svh_verify_sig(pk, bytes(bad), 64, m, len(m)) == 0
    assert host.svh_verify_sig(pk, bytes(bad), 64, m, len(m)) == 0  # false verdicts are cached too
    assert host.svh_verify_sig(pk, sig, 64, m + b"o", len(m) + 1) == 0  # wrong message
    assert _counts(host) == (2, 3)
    assert engine.sigs == 3
    # size != 64: rejected before the cache and the engine (SecretKey.cpp:441-444)
    assert host.svh_verify_sig(pk, sig, 63, m, len(m)) == 0
    assert _counts(host) == (0, 0) and engine.sigs == 3
    host.svh_cache_clear()
    assert host.svh_verify_sig(pk, sig, 64, m, len(m)) == 1
    assert _counts(host) == (0, 1)


def test_verify_sig_batch_dedup_and_verdicts(host, engine, golden):
    d = golden["adversarial"]
    rows = np.arange(0, len(d["verdict"]), 11)
    rows = np.concatenate([rows, rows[:20]])  # duplicates inside one batch
    n = len(rows)
    pk = np.ascontiguousarray(d["pk"][rows])
    sig = np.ascontiguousarray(d["sig"][rows])
    off = np.ascontiguousarray(d["msg_off"][rows])
    ln = np.ascontiguousarray(d["msg_len"][rows])
    msg = np.ascontiguousarray(d["msg"])
    out = np.zeros(n, np.uint8)
    rc = host.svh_verify_sig_batch(pk.ctypes.data_as(ctypes.c_void_p), sig.ctypes.data_as(ctypes.c_void_p), None,
                                   msg.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p),
                                   ln.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n),
                                   out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    assert (out == d["verdict"][rows]).all()
    assert engine.calls == 1 and engine.sigs == n - 20
    assert _counts(host) == (20, n - 20)


_HOST_KEYS_CHILD = r"""
import ctypes, sys
import numpy as np
z = np.load(sys.argv[2], allow_pickle=False)
h = ctypes.CDLL(sys.argv[1])
vp = ctypes.c_void_p
pk, sig, msg, off, ln = (np.ascontiguousarray(z[k]) for k in ("pk", "sig", "msg", "msg_off", "msg_len"))
n = len(ln)
h.svh_set_keyed_threshold(ctypes.c_size_t(64))
h.svh_cache_clear()
outs = []
for _ in range(2):
    h.svh_cache_counts(None, None)
    out = np.zeros(n, np.uint8)
    assert h.svh_verify_sig_batch(vp(pk.ctypes.data), vp(sig.ctypes.data), None, vp(msg.ctypes.data),
                                  vp(off.ctypes.data), vp(ln.ctypes.data), ctypes.c_size_t(n), vp(out.ctypes.data)) == 0
    hit, miss = ctypes.c_uint64(), ctypes.c_uint64()
    h.svh_cache_counts(ctypes.byref(hit), ctypes.byref(miss))
    outs.append((out, hit.value, miss.value))
np.savez(sys.argv[3], v0=outs[0][0], v1=outs[1][0], c=np.array([outs[0][1], outs[0][2], outs[1][1], outs[1][2]]))
"""


def test_keyed_batch_host_keys_beside_engine(host, golden, tmp_path):
    """SV_HOST_KEYS=1 (read once per process, hence a child): a keyed batch
    hashes its cache keys on the host pool while the engine call runs and the
    last hashing helper walks the cache.  Here the engine has no device, so the
    call fails over to the CPU path after the walk: verdicts must still equal
    the golden ones, the first batch must miss every distinct item and the
    second hit every one (the keys the walk inserted are the cache's keys)."""
    d = golden["adversarial"]
    rows = np.arange(len(d["verdict"]))[:300]
    src = tmp_path / "in.npz"
    np.savez(src, pk=d["pk"][rows], sig=d["sig"][rows], msg=d["msg"], msg_off=d["msg_off"][rows],
             msg_len=d["msg_len"][rows])
    dst = tmp_path / "out.npz"
    env = dict(os.environ, SV_HOST_KEYS="1")
    r = subprocess.run([sys.executable, "-c", _HOST_KEYS_CHILD, host._name, str(src), str(dst)], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    z = np.load(dst)
    want = d["verdict"][rows]
    assert (z["v0"] == want).all() and (z["v1"] == want).all()
    eligible = int((d["sig"][rows].shape[1] == 64) * len(rows))
    hit0, miss0, hit1, miss1 = (int(x) for x in z["c"])
    assert hit0 + miss0 == eligible and hit1 == eligible and miss1 == 0


def test_cache_cleared_during_batch(host, oracle, golden):
    """clearVerifySigCache between a batch's cache walk and the resolve of its
    pending inserts (here: from inside the engine call) must neither touch the
    cleared table nor change the batch's verdicts (resolve() bounds)."""
    e = OracleEngine(oracle)

    def clearing(*a):
        host.svh_cache_clear()
        return e.fn_plain(*a)

    cfn = VERIFY_FN(clearing)
    d = golden["adversarial"]
    rows = np.concatenate([np.arange(0, 600, 3), np.arange(0, 60, 3)])  # with in-batch duplicates
    n = len(rows)
    pk, sig = np.ascontiguousarray(d["pk"][rows]), np.ascontiguousarray(d["sig"][rows])
    off, ln = np.ascontiguousarray(d["msg_off"][rows]), np.ascontiguousarray(d["msg_len"][rows])
    msg = np.ascontiguousarray(d["msg"])
    vp = ctypes.c_void_p
    host.svh_set_test_verifier(ctypes.cast(cfn, ctypes.c_void_p))
    try:
        for _ in range(3):
            host.svh_cache_clear()
            out = np.zeros(n, np.uint8)
            assert host.svh_verify_sig_batch(vp(pk.ctypes.data), vp(sig.ctypes.data), None, vp(msg.ctypes.data),
                                             vp(off.ctypes.data), vp(ln.ctypes.data), ctypes.c_size_t(n),
                                             vp(out.ctypes.data)) == 0
            assert (out == d["verdict"][rows]).all()
            assert host.svh_cache_keys(None, 0) == 0  # cleared mid-batch: nothing of it was resolved in
        # the cache keeps working afterwards
        host.svh_set_test_verifier(ctypes.cast(e.cfn, ctypes.c_void_p))
        out = np.zeros(n, np.uint8)
        assert host.svh_verify_sig_batch(vp(pk.ctypes.data), vp(sig.ctypes.data), None, vp(msg.ctypes.data),
                                         vp(off.ctypes.data), vp(ln.ctypes.data), ctypes.c_size_t(n),
                                         vp(out.ctypes.data)) == 0
        assert (out == d["verdict"][rows]).all()
    finally:
        host.svh_set_test_verifier(None)
        host.svh_cache_clear()


def test_engine_histograms(host, engine, golden):
    """Batch-size / latency histograms beside the crypto.verify.* counters
    (docs/metrics.md:48-50): one bucket count per engine call, log2 buckets,
    flushed on read."""
    host.svh_engine_histograms.argtypes = [ctypes.c_void_p]
    h = np.zeros(128, np.uint64)
    host.svh_engine_histograms(h.ctypes.data)  # (flush earlier tests)
    d = golden["valid"]
    for n, start in ((1, 0), (3, 10), (300, 100)):
        rows = np.arange(n) + start
        pk, sig = np.ascontiguousarray(d["pk"][rows]), np.ascontiguousarray(d["sig"][rows])
        off, ln = np.ascontiguousarray(d["msg_off"][rows]), np.ascontiguousarray(d["msg_len"][rows])
        msg = np.ascontiguousarray(d["msg"])
        out = np.zeros(n, np.uint8)
        vp = ctypes.c_void_p
        assert host.svh_verify_sig_batch(vp(pk.ctypes.data), vp(sig.ctypes.data), None, vp(msg.ctypes.data),
                                         vp(off.ctypes.data), vp(ln.ctypes.data), ctypes.c_size_t(n),
                                         vp(out.ctypes.data)) == 0
        assert out.all()
    host.svh_engine_histograms(h.ctypes.data)
    gpu_size, gpu_lat = h[0:32], h[32:64]
    assert gpu_size[0] == 1 and gpu_size[1] == 1 and gpu_size[8] == 1  # sizes 1, 3, 300
    assert int(gpu_size.sum()) == 3 == int(gpu_lat.sum()) == engine.calls
    host.svh_engine_histograms(h.ctypes.data)
    assert int(h.sum()) == 0  # flushed


def test_verify_sig_batch_keyed_path(host, oracle, golden):
    """f4: with the keyed pass (verdicts + cache keys from the engine, no host
    hashing) verdicts, hit/miss counters and cache contents match the hashed
    path exactly; the engine sees every eligible row in ONE call."""
    e = OracleKeyedEngine(oracle)
    host.svh_set_test_verifier(None)
    host.svh_set_test_keyed_verifier(ctypes.cast(e.kcfn, ctypes.c_void_p))
    host.svh_set_keyed_threshold(1)
    host.svh_cache_clear()
    host.svh_cache_counts(None, None)
    try:
        d = golden["adversarial"]
        rows = np.arange(0, len(d["verdict"]), 13)
        rows = np.concatenate([rows, rows[:15]])
        n = len(rows)
        pk = np.ascontiguousarray(d["pk"][rows])
        sig = np.ascontiguousarray(d["sig"][rows])
        off = np.ascontiguousarray(d["msg_off"][rows])
        ln = np.ascontiguousarray(d["msg_len"][rows])
        msg = np.ascontiguousarray(d["msg"])
        for rep in range(2):
            out = np.zeros(n, np.uint8)
            rc = host.svh_verify_sig_batch(pk.ctypes.data_as(ctypes.c_void_p), sig.ctypes.data_as(ctypes.c_void_p),
                                           None, msg.ctypes.data_as(ctypes.c_void_p),
                                           off.ctypes.data_as(ctypes.c_void_p), ln.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.c_size_t(n), out.ctypes.data_as(ctypes.c_void_p))
            assert rc == 0, host.svh_last_error_string()
            assert (out == d["verdict"][rows]).all()
            if rep == 0:
                assert _counts(host) == (15, n - 15)  # in-batch duplicates count as hits
            else:
                assert _counts(host) == (n, 0)        # every key now cached
        assert e.sigs == 2 * n and e.calls == 2       # one keyed engine pass per batch
        # a single verifySig now hits the entry the keyed batch stored
        i = 0
        o, L = int(off[i]), int(ln[i])
        assert host.svh_verify_sig(pk[i].tobytes(), sig[i].tobytes(), 64, msg[o:o + L].tobytes(), L) == d["verdict"][rows[i]]
        assert _counts(host) == (1, 0)
    finally:
        host.svh_set_test_keyed_verifier(None)
        host.svh_set_keyed_threshold(256)
        host.svh_cache_clear()


def _oracle_sign_fn(oracle):
    def sign(reqs):
        out = []
        for seed, msg in reqs:
            pk = ctypes.create_string_buffer(32)
            sk = ctypes.create_string_buffer(64)
            oracle.oracle_ed25519_seed_keypair(pk, sk, seed)
            s = ctypes.create_string_buffer(64)
            oracle.oracle_ed25519_sign(s, msg, len(msg), sk.raw)
            out.append((pk.raw, s.raw))
        return out
    return sign


def _check(host, txs, prefetch):
    T, S, G = tg.to_ctypes(txs)
    ok = np.zeros(len(txs), np.uint8)
    used = np.zeros(len(txs), np.uint8)
    pairs = ctypes.c_uint64()
    rc = host.svh_check_txset(T, ctypes.c_size_t(len(txs)), S, G, prefetch, ok.ctypes.data_as(ctypes.c_void_p),
                              used.ctypes.data_as(ctypes.c_void_p), ctypes.byref(pairs))
    assert rc == 0, host.svh_last_error_string()
    return ok, used, pairs.value


def test_signature_checker_matches_python_replay(host, engine, oracle):
    sign = _oracle_sign_fn(oracle)
    txs = tg.generate(60, sign, seed=11)
    tg.add_payload_signatures(txs, sign)

    def verify(pk, sig, msg):
        return oracle.oracle_ed25519_verify(sig, msg, len(msg), pk) == 0

    want_ok, want_used = tg.replay(txs, verify)
    ok0, used0, _ = _check(host, txs, 0)
    host.svh_cache_clear()
    calls_before = engine.calls
    ok1, used1, pairs = _check(host, txs, 1)
    assert (ok0 == want_ok).all() and (used0 == want_used).all()
    assert (ok1 == want_ok).all() and (used1 == want_used).all()
    assert engine.calls - calls_before == 1  # the whole set went out as ONE batch
    assert pairs > 0
    assert 0 < want_ok.sum() < len(txs) or want_ok.sum() == len(txs)


def test_txset_prefetch_parallel_batch_matches_replay(host, engine, oracle):
    """A set large enough that svh_check_txset enumerates the pairs in parallel
    parts (SignatureBatchPrefetch::addBatch) and runs the checkers on the host
    pool, each finding its pairs by position: outcomes equal the sequential
    no-prefetch path and the Python replay."""
    sign = _oracle_sign_fn(oracle)
    txs = tg.generate(1500, sign, seed=23)
    tg.add_payload_signatures(txs, sign)

    def verify(pk, sig, msg):
        return oracle.oracle_ed25519_verify(sig, msg, len(msg), pk) == 0

    want_ok, want_used = tg.replay(txs, verify)
    host.svh_cache_clear()
    ok0, used0, _ = _check(host, txs, 0)
    assert (ok0 == want_ok).all() and (used0 == want_used).all()
    host.svh_cache_clear()
    calls_before = engine.calls
    ok1, used1, pairs = _check(host, txs, 1)
    assert engine.calls - calls_before == 1
    assert (ok1 == want_ok).all() and (used1 == want_used).all()
    assert pairs > 0 and 0 < want_ok.sum() < len(txs)
    # the same pre-pass, checkers without their tx's position (table lookups only)
    host.svh_cache_clear()
    calls_before = engine.calls
    ok3, used3, pairs3 = _check(host, txs, 3)
    assert engine.calls - calls_before == 1 and pairs3 == pairs
    assert (ok3 == want_ok).all() and (used3 == want_used).all()
    # pipelined in two halves (use_prefetch 4): two engine batches, the same pairs and outcomes
    host.svh_cache_clear()
    calls_before = engine.calls
    ok4, used4, pairs4 = _check(host, txs, 4)
    assert engine.calls - calls_before == 2 and pairs4 == pairs
    assert (ok4 == want_ok).all() and (used4 == want_used).all()
    # (a set below the pipeline's minimum runs as one batch)
    small = txs[:200]
    calls_before = engine.calls
    ok5, used5, _ = _check(host, small, 4)
    assert engine.calls - calls_before == 1
    assert (ok5 == want_ok[:200]).all() and (used5 == want_used[:200]).all()


def test_txset_bad_signer_in_parallel_marshal_is_an_error(host, engine, oracle):
    """A malformed signer deep inside a set marshalled in parallel parts comes
    back as SVH_ERR_INVALID_ARG with its message (never an exception escaping a
    pool thread)."""
    sign = _oracle_sign_fn(oracle)
    txs = tg.generate(1100, sign, seed=5)  # (>= 1024: the pipelined mode 4 splits it; the bad signer is in half 1)
    T, S, G = tg.to_ctypes(txs)
    G[len(G) - 3].type = 7  # no such signer type
    ok = np.zeros(len(txs), np.uint8)
    used = np.zeros(len(txs), np.uint8)
    for prefetch in (1, 0, 4):
        rc = host.svh_check_txset(T, ctypes.c_size_t(len(txs)), S, G, prefetch, ok.ctypes.data_as(ctypes.c_void_p),
                                  used.ctypes.data_as(ctypes.c_void_p), None)
        assert rc != 0
        assert b"signer" in host.svh_last_error_string()


@pytest.mark.gpu
def test_gpu_host_mirror_verify_sig(host, sv, golden):
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    host.svh_set_test_verifier(None)
    host.svh_cache_clear()
    d = golden["intree"]
    for i in range(len(d["verdict"])):
        o, ln = int(d["msg_off"][i]), int(d["msg_len"][i])
        m = d["msg"][o:o + ln].tobytes()
        assert host.svh_verify_sig(d["pk"][i].tobytes(), d["sig"][i].tobytes(), 64, m, ln) == d["verdict"][i]


@pytest.mark.gpu
def test_gpu_txset_prefetch_matches_replay(host, sv, oracle):
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    host.svh_set_test_verifier(None)
    host.svh_cache_clear()
    sign = _oracle_sign_fn(oracle)
    txs = tg.generate(120, sign, seed=5)
    tg.add_payload_signatures(txs, sign)

    def verify(pk, sig, msg):
        return oracle.oracle_ed25519_verify(sig, msg, len(msg), pk) == 0

    want_ok, want_used = tg.replay(txs, verify)
    ok1, used1, pairs = _check(host, txs, 1)
    assert (ok1 == want_ok).all() and (used1 == want_used).all()
    host.svh_cache_clear()
    ok0, used0, _ = _check(host, txs, 0)
    assert (ok0 == want_ok).all() and (used0 == want_used).all()


class MbStats(ctypes.Structure):
    _fields_ = [("items", ctypes.c_uint64), ("batches", ctypes.c_uint64), ("flushed_by_size", ctypes.c_uint64),
                ("flushed_by_deadline", ctypes.c_uint64), ("max_batch", ctypes.c_uint64),
                ("lat_p50_us", ctypes.c_double), ("lat_p99_us", ctypes.c_double)]


def _mb_run(host, d, rows, producers, max_batch, max_delay_us, gap_us=0, workers=1):
    n = len(rows)
    pk = np.ascontiguousarray(d["pk"][rows])
    sig = np.ascontiguousarray(d["sig"][rows])
    off = np.ascontiguousarray(d["msg_off"][rows])
    ln = np.ascontiguousarray(d["msg_len"][rows])
    msg = np.ascontiguousarray(d["msg"])
    out = np.full(n, 7, np.uint8)
    st = MbStats()
    vp = ctypes.c_void_p
    if workers == 1:
        rc = host.svh_mb_run(vp(pk.ctypes.data), vp(sig.ctypes.data), vp(msg.ctypes.data), vp(off.ctypes.data),
                             vp(ln.ctypes.data), ctypes.c_size_t(n), producers, ctypes.c_uint32(max_batch),
                             ctypes.c_uint32(max_delay_us), ctypes.c_uint32(gap_us), vp(out.ctypes.data),
                             ctypes.byref(st))
    else:
        rc = host.svh_mb_run_workers(vp(pk.ctypes.data), vp(sig.ctypes.data), vp(msg.ctypes.data),
                                     vp(off.ctypes.data), vp(ln.ctypes.data), ctypes.c_size_t(n), producers, workers,
                                     ctypes.c_uint32(max_batch), ctypes.c_uint32(max_delay_us),
                                     ctypes.c_uint32(gap_us), vp(out.ctypes.data), ctypes.byref(st))
    assert rc == 0, host.svh_last_error_string()
    return out, st


def test_micro_batcher_size_flush_many_producers(host, engine, golden):
    """concurrent producers, flush at maxBatch; every future
    gets its own row's verdict."""
    d = golden["adversarial"]
    rows = np.arange(0, len(d["verdict"]), 5)
    out, st = _mb_run(host, d, rows, producers=6, max_batch=32, max_delay_us=200_000)
    assert (out == d["verdict"][rows]).all()
    assert st.items == len(rows) and st.max_batch <= 32
    assert st.flushed_by_size >= 1
    assert st.batches == st.flushed_by_size + st.flushed_by_deadline
    assert engine.sigs <= len(rows)


def test_micro_batcher_deadline_flush(host, engine, golden):
    """A trickle below maxBatch is flushed by the oldest item's deadline."""
    d = golden["valid"]
    rows = np.arange(5)
    out, st = _mb_run(host, d, rows, producers=1, max_batch=1000, max_delay_us=3000, gap_us=500)
    assert (out == 1).all()
    assert st.flushed_by_size == 0 and st.flushed_by_deadline >= 1
    assert st.lat_p99_us >= 0 and st.items == 5


def test_micro_batcher_multiple_workers(host, engine, golden):
    """Several flush workers (batches in flight at once): same verdicts, every
    item in exactly one batch, size and deadline flushes both still honoured."""
    d = golden["adversarial"]
    rows = np.arange(0, len(d["verdict"]), 3)
    out, st = _mb_run(host, d, rows, producers=6, max_batch=16, max_delay_us=100_000, workers=3)
    assert (out == d["verdict"][rows]).all()
    assert st.items == len(rows) and st.max_batch <= 16
    assert st.batches >= (len(rows) + 15) // 16 and st.flushed_by_size >= 1
    assert st.batches == st.flushed_by_size + st.flushed_by_deadline
    d = golden["valid"]
    rows = np.arange(6)
    out, st = _mb_run(host, d, rows, producers=1, max_batch=1000, max_delay_us=3000, gap_us=500, workers=3)
    assert (out == 1).all()
    assert st.flushed_by_size == 0 and st.flushed_by_deadline >= 1 and st.items == 6


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


def scp_run(host, d, rows, producers, burst, interval_us, max_batch=8192, max_delay_us=2000, workers=2, policy=0,
            linger_us=0, quiet_us=0, max_linger_us=0, batch_post=0):
    """svh_scp_run (config 4 through the micro-batcher: continuation submits,
    a main thread calling verifySig per envelope) over golden rows."""
    n = len(rows)
    pk = np.ascontiguousarray(d["pk"][rows])
    sig = np.ascontiguousarray(d["sig"][rows])
    off = np.ascontiguousarray(d["msg_off"][rows])
    ln = np.ascontiguousarray(d["msg_len"][rows])
    msg = np.ascontiguousarray(d["msg"])
    out = np.full(n, 7, np.uint8)
    p = ScpParams(ctypes.sizeof(ScpParams), producers, burst, interval_us, max_batch, max_delay_us, workers, policy,
                  linger_us, 1, quiet_us, max_linger_us, batch_post)
    r = ScpResult()
    vp = ctypes.c_void_p
    rc = host.svh_scp_run(vp(pk.ctypes.data), vp(sig.ctypes.data), vp(msg.ctypes.data), vp(off.ctypes.data),
                          vp(ln.ctypes.data), ctypes.c_size_t(n), ctypes.byref(p), vp(out.ctypes.data),
                          ctypes.byref(r))
    assert rc == 0, host.svh_last_error_string()
    return out, r


def test_scp_run_idle_flush_trickle(host, engine, golden):
    """WhenIdle policy (VerifyMicroBatcher.h): a trickle of lone envelopes is
    flushed as each arrives -- no batch waits out maxDelay (200 ms here) --
    every continuation precedes the main thread's verifySig, which hits the
    cache (the Peer.cpp:963-979 -> HerderImpl.cpp:2414-2432 order)."""
    d = golden["adversarial"]
    rows = np.arange(0, len(d["verdict"]), 7)[:24]
    out, r = scp_run(host, d, rows, producers=1, burst=1, interval_us=3000, max_delay_us=200_000)
    assert (out == d["verdict"][rows]).all()
    assert r.main_hits == len(rows) and r.main_misses == 0 and r.main_mismatches == 0
    assert r.flushed_idle == r.batches and r.flushed_by_deadline == 0 and r.flushed_by_size == 0
    assert r.verdict_max_us < 100_000  # (far below the 200 ms deadline)


def test_scp_run_bursts_many_producers(host, engine, golden):
    """Bursts from several producers under WhenIdle: batches grow while one is
    in flight; every item's verdict and the main thread's hit are exact.
    (Distinct envelopes: a duplicate in flight in two batches is pending under
    the later one until it resolves, and a verifySig meanwhile is a miss, as
    for concurrent verifySig calls; the overlay drops duplicates before the
    pre-verify, Peer.cpp:957-960.)"""
    d = golden["adversarial"]
    seen, rows = set(), []
    for i in range(len(d["verdict"])):
        o, ln = int(d["msg_off"][i]), int(d["msg_len"][i])
        k = d["pk"][i].tobytes() + d["sig"][i].tobytes() + d["msg"][o:o + ln].tobytes()
        if k not in seen:
            seen.add(k)
            rows.append(i)
    rows = np.array(rows)
    out, r = scp_run(host, d, rows, producers=4, burst=64, interval_us=20_000, max_delay_us=500_000)
    assert (out == d["verdict"][rows]).all()
    assert r.main_hits == len(rows) and r.main_mismatches == 0
    assert r.batches == r.flushed_by_size + r.flushed_by_deadline + r.flushed_idle
    assert r.flushed_idle >= 1 and r.max_batch <= 8192


def test_scp_run_batched_post(host, engine, golden):
    """The overlay posting one main-thread task per verified batch
    (VerifyMicroBatcher::submitTagged + Options::onBatch): the same verdicts,
    every main-thread verifySig a hit, every envelope delivered once; and a
    caller built against the struct without `batch_post` (struct_size ending
    before it) still runs, per-envelope."""
    d = golden["adversarial"]
    seen, rows = set(), []
    for i in range(len(d["verdict"])):
        o, ln = int(d["msg_off"][i]), int(d["msg_len"][i])
        k = d["pk"][i].tobytes() + d["sig"][i].tobytes() + d["msg"][o:o + ln].tobytes()
        if k not in seen:
            seen.add(k)
            rows.append(i)
    rows = np.array(rows)
    out, r = scp_run(host, d, rows, producers=4, burst=64, interval_us=20_000, max_delay_us=500_000, batch_post=1)
    assert (out == d["verdict"][rows]).all()
    assert r.main_hits == len(rows) and r.main_misses == 0 and r.main_mismatches == 0
    assert r.batches >= 1

    class OldScpParams(ctypes.Structure):  # (the round-5 layout: no batch_post)
        _fields_ = ScpParams._fields_[:-1]
    n = 64
    p = OldScpParams(ctypes.sizeof(OldScpParams), 2, 16, 1000, 8192, 2000, 2, 0, 0, 1, 0, 0)
    res = ScpResult()
    out = np.full(n, 7, np.uint8)
    vp = ctypes.c_void_p
    sub = rows[:n]
    pk, sig = np.ascontiguousarray(d["pk"][sub]), np.ascontiguousarray(d["sig"][sub])
    off, ln = np.ascontiguousarray(d["msg_off"][sub]), np.ascontiguousarray(d["msg_len"][sub])
    rc = host.svh_scp_run(vp(pk.ctypes.data), vp(sig.ctypes.data), vp(d["msg"].ctypes.data), vp(off.ctypes.data),
                          vp(ln.ctypes.data), ctypes.c_size_t(n), ctypes.byref(p), vp(out.ctypes.data),
                          ctypes.byref(res))
    assert rc == 0, host.svh_last_error_string()
    assert (out == d["verdict"][sub]).all() and res.main_hits == n


def test_scp_run_deadline_policy_waits(host, engine, golden):
    """The round-2 Deadline policy, for contrast: a lone envelope waits out
    maxDelay before its batch is flushed."""
    d = golden["valid"]
    rows = np.arange(6)
    out, r = scp_run(host, d, rows, producers=1, burst=1, interval_us=20_000, max_delay_us=5000, policy=1)
    assert (out == 1).all() and r.main_hits == len(rows)
    assert r.flushed_idle == 0 and r.flushed_by_deadline == r.batches
    assert r.verdict_p50_us >= 4900


def test_scp_run_linger_collects_a_burst(host, engine, golden):
    """linger: an idle flush waits until the oldest item is that old, so a
    burst that arrives within it becomes one batch."""
    d = golden["valid"]
    rows = np.arange(32)
    out, r = scp_run(host, d, rows, producers=1, burst=32, interval_us=0, max_delay_us=400_000, linger_us=200_000)
    assert (out == 1).all() and r.main_hits == len(rows)
    assert r.batches == 1 and r.max_batch == 32


def test_scp_run_quiet_period_makes_one_batch_per_burst(host, engine, golden):
    """WhenIdle with a quiet period: a burst that is still arriving is waited
    for (until it has been quiet for quiet_us) and flushed as ONE batch; lone
    items still go at once."""
    d = golden["valid"]
    rows = np.arange(96)
    # (a first run in a fresh process pays one-time setup inside its first
    # batch, long enough to split that burst: run the shape once untimed)
    scp_run(host, d, rows[:8], producers=1, burst=8, interval_us=1000, max_delay_us=400_000)
    out, r = scp_run(host, d, rows, producers=1, burst=32, interval_us=60_000, max_delay_us=400_000,
                     quiet_us=20_000, max_linger_us=300_000)
    assert (out == 1).all() and r.main_hits == len(rows)
    assert r.batches == 3 and r.max_batch == 32 and r.burst_waits >= 1
    out, r = scp_run(host, d, rows[:6], producers=1, burst=1, interval_us=5000, max_delay_us=400_000,
                     quiet_us=20_000, max_linger_us=300_000)
    # (lone items are not held for the quiet period: each normally goes as a
    # batch of its own; on a loaded host a slow batch can still be in flight
    # when the next item arrives, which then rides the following flush)
    assert (out == 1).all() and r.batches >= 3 and r.verdict_p50_us < 20_000


@pytest.mark.gpu
def test_gpu_verify_sig_batch_keyed_matches_hashed(host, sv, golden):
    """f4 on the GPU: the keyed pass (engine returns cache keys) gives the same
    verdicts and hit/miss counts as host BLAKE2b hashing."""
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    host.svh_set_test_verifier(None)
    host.svh_set_test_keyed_verifier(None)
    d = golden["adversarial"]
    rows = np.arange(len(d["verdict"]))
    rows = np.concatenate([rows, rows[:100]])
    n = len(rows)
    pk = np.ascontiguousarray(d["pk"][rows])
    sig = np.ascontiguousarray(d["sig"][rows])
    off = np.ascontiguousarray(d["msg_off"][rows])
    ln = np.ascontiguousarray(d["msg_len"][rows])
    msg = np.ascontiguousarray(d["msg"])
    res = []
    try:
        for thr in (0, 1):
            host.svh_set_keyed_threshold(thr)
            host.svh_cache_clear()
            host.svh_cache_counts(None, None)
            out = np.zeros(n, np.uint8)
            rc = host.svh_verify_sig_batch(pk.ctypes.data_as(ctypes.c_void_p), sig.ctypes.data_as(ctypes.c_void_p),
                                           None, msg.ctypes.data_as(ctypes.c_void_p),
                                           off.ctypes.data_as(ctypes.c_void_p), ln.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.c_size_t(n), out.ctypes.data_as(ctypes.c_void_p))
            assert rc == 0, host.svh_last_error_string()
            res.append((out.copy(), _counts(host)))
    finally:
        host.svh_set_keyed_threshold(256)
        host.svh_cache_clear()
    assert (res[0][0] == d["verdict"][rows]).all()
    assert (res[1][0] == res[0][0]).all()
    assert res[0][1] == res[1][1]


@pytest.mark.gpu
def test_gpu_verify_sig_batch_keyed_large_equals_hashed_cache_state(host, sv, golden):
    """The large keyed path (threaded walk over key pieces, eviction draws
    queued while the keys are on their way, misses inserted with their verdict
    once the engine has returned) against the host-hashed three-phase path on
    100k items with re-submissions and more than 0xffff distinct keys: equal
    verdicts, equal hit/miss counts and the same cache contents in the same
    eviction-vector order."""
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    host.svh_set_test_verifier(None)
    host.svh_set_test_keyed_verifier(None)
    d = golden["adversarial"]
    rng = np.random.default_rng(77)
    n_rand, n = 90000, 100000
    # random items (invalid) plus golden rows (valid and invalid), then repeats
    gold = rng.choice(len(d["verdict"]), n - n_rand, replace=True)
    pk = np.concatenate([rng.integers(0, 256, (n_rand, 32), dtype=np.uint8), d["pk"][gold]])
    sig = np.concatenate([rng.integers(0, 256, (n_rand, 64), dtype=np.uint8), d["sig"][gold]])
    rmsg = rng.integers(0, 256, 32 * n_rand, dtype=np.uint8)
    msg = np.concatenate([rmsg, d["msg"]])
    off = np.concatenate([np.arange(n_rand, dtype=np.uint64) * 32, d["msg_off"][gold] + len(rmsg)])
    ln = np.concatenate([np.full(n_rand, 32, np.uint32), d["msg_len"][gold]])
    perm = rng.permutation(n)
    perm[5000::97] = perm[100:100 + len(perm[5000::97])]  # re-submissions of early items
    pk, sig, off, ln = (np.ascontiguousarray(a[perm]) for a in (pk, sig, off, ln))
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    res = []
    try:
        for thr in (0, 256):  # host-hashed, keyed
            host.svh_set_keyed_threshold(thr)
            host.svh_cache_clear()
            host.svh_cache_seed(99)
            host.svh_cache_counts(None, None)
            out = np.zeros(n, np.uint8)
            for a, b in ((0, 30000), (30000, n)):  # two batches: the second walks a full cache
                rc = host.svh_verify_sig_batch(P(pk[a:b]), P(sig[a:b]), None, P(msg), P(off[a:b]), P(ln[a:b]),
                                               ctypes.c_size_t(b - a), P(out[a:]))
                assert rc == 0, host.svh_last_error_string()
            keys = np.zeros((0x10000, 32), np.uint8)
            size = host.svh_cache_keys(P(keys), ctypes.c_size_t(0x10000))
            res.append((out.copy(), _counts(host), keys[:size].copy()))
    finally:
        host.svh_set_keyed_threshold(256)
        host.svh_cache_clear()
    (o0, c0, k0), (o1, c1, k1) = res
    assert (o0 == o1).all() and c0 == c1
    assert len(k0) == 0xFFFF and (k0 == k1).all()
    gold_rows = perm >= n_rand
    assert (o1[gold_rows] == d["verdict"][gold[perm[gold_rows] - n_rand]]).all()


# ---------------------------------------------------------------- round 2
class EngineStats(ctypes.Structure):
    _fields_ = [("gpu_signatures", ctypes.c_uint64), ("gpu_batches", ctypes.c_uint64),
                ("cpu_signatures", ctypes.c_uint64), ("fallbacks", ctypes.c_uint64)]


def _estats(host):
    s = EngineStats()
    host.svh_engine_counts_ex(ctypes.byref(s))
    return s


def _batch(host, d, rows):
    pk = np.ascontiguousarray(d["pk"][rows])
    sig = np.ascontiguousarray(d["sig"][rows])
    off = np.ascontiguousarray(d["msg_off"][rows])
    ln = np.ascontiguousarray(d["msg_len"][rows])
    msg = np.ascontiguousarray(d["msg"])
    out = np.full(len(rows), 7, np.uint8)
    rc = host.svh_verify_sig_batch(pk.ctypes.data_as(ctypes.c_void_p), sig.ctypes.data_as(ctypes.c_void_p), None,
                                   msg.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p),
                                   ln.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(len(rows)),
                                   out.ctypes.data_as(ctypes.c_void_p))
    return rc, out


def test_engine_error_is_never_a_reject(host, golden):
    """an engine error re-runs the batch on the engine's CPU
    path -- the mirror returns libsodium's verdicts and raises nothing (the
    reference's verifySig never throws, SecretKey.cpp:435-468)."""
    failing = VERIFY_FN(lambda *a: -3)  # SV_ERR_HIP
    host.svh_set_test_verifier(ctypes.cast(failing, ctypes.c_void_p))
    host.svh_set_keyed_threshold(0)
    host.svh_cache_clear()
    _estats(host)
    try:
        for name in ("intree", "msglen", "adversarial"):
            d = golden[name]
            rows = np.arange(len(d["verdict"]))
            rc, out = _batch(host, d, rows)
            assert rc == 0
            assert (out == d["verdict"]).all(), name
        s = _estats(host)
        assert s.fallbacks == 3 and s.gpu_signatures == 0 and s.cpu_signatures > 0
    finally:
        host.svh_set_test_verifier(None)
        host.svh_set_keyed_threshold(256)
        host.svh_cache_clear()


def test_single_verify_sig_runs_on_cpu_path(host, golden):
    """verifySig of one signature never pays a GPU round trip: the miss runs on
    the engine's CPU path (works on this GPU-less host)."""
    host.svh_set_test_verifier(None)
    host.svh_cache_clear()
    host.svh_cache_counts(None, None)
    _estats(host)
    d = golden["adversarial"]
    for i in range(0, len(d["verdict"]), 211):
        o, ln = int(d["msg_off"][i]), int(d["msg_len"][i])
        m = d["msg"][o:o + ln].tobytes()
        assert host.svh_verify_sig(d["pk"][i].tobytes(), d["sig"][i].tobytes(), 64, m, ln) == d["verdict"][i]
    s = _estats(host)
    assert s.gpu_signatures == 0 and s.cpu_signatures == len(range(0, len(d["verdict"]), 211))
    host.svh_cache_clear()


class RefCache:
    """Sequential restatement of RandomEvictionCache<Hash,bool>(0xffff, separatePRNG)
    (src/util/RandomEvictionCache.h:20-245) with rand_uniform = stellar's pinned
    libc++ uniform_int_distribution (lib/util/stdrandom.h) over std::minstd_rand."""

    def __init__(self, max_size=0xFFFF, seed=None):
        self.max, self.gen, self.map, self.ptrs = max_size, 0, {}, []
        self.x = 1 if seed is None else (seed % 2147483647 or 1)

    def _engine(self):
        self.x = self.x * 48271 % 2147483647
        return self.x

    def _uniform(self, lo, hi):
        r = hi - lo + 1
        if r == 1:
            return lo
        w = (r - 1).bit_length()
        R, m = 2147483646, 30
        n = -(-w // m)
        w0 = w // n
        y0 = (R >> w0) << w0
        if R - y0 > y0 // n:
            n += 1
            w0 = w // n
            y0 = (R >> w0) << w0
        n0 = n - w % n
        y1 = (R >> (w0 + 1)) << (w0 + 1)
        while True:
            s = 0
            for k in range(n):
                lim, bits = (y0, w0) if k < n0 else (y1, w0 + 1)
                while True:
                    u = self._engine() - 1
                    if u < lim:
                        break
                s = (s << bits) + (u & ((1 << bits) - 1))
            if s < r:
                return s + lo

    def get(self, k):
        self.gen += 1
        self.map[k][0] = self.gen

    def put(self, k):
        self.gen += 1
        if k in self.map:
            self.map[k][0] = self.gen
            return
        self.map[k] = [self.gen]
        self.ptrs.append(k)
        if len(self.ptrs) > self.max:
            a = self._uniform(0, len(self.ptrs) - 1)
            b = self._uniform(0, len(self.ptrs) - 1)
            v = a if self.map[self.ptrs[a]][0] < self.map[self.ptrs[b]][0] else b
            del self.map[self.ptrs[v]]
            self.ptrs[v], self.ptrs[-1] = self.ptrs[-1], self.ptrs[v]
            self.ptrs.pop()


@pytest.mark.parametrize("keyed,n_odd", [(False, 700), (True, 700), (True, 0)])
def test_large_batch_rows_with_mixed_signature_sizes(host, hostcore, keyed, n_odd):
    """A batch large enough for the pooled eligibility pass (>= 2 x 16384
    items), with signatures of sizes 0..63 mixed in: the same verdicts, counts
    and cache contents as the same item stream fed in batches of 1000 (the
    serial pass).  Items whose signature is not 64 bytes are rejected without
    touching the cache (SecretKey.cpp:441-444)."""
    rng = np.random.default_rng(515)
    n = 50000
    pk = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    sig = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    sl = np.full(n, 64, np.uint32)
    odd = rng.choice(n, n_odd, replace=False)  # (0: every row eligible, the one-pass case)
    sl[odd] = rng.choice([0, 1, 32, 63], len(odd))  # (the C-ABI takes n x 64 signature bytes)
    msg = rng.integers(0, 256, 32 * n, dtype=np.uint8)
    off = np.arange(n, dtype=np.uint64) * 32
    ln = np.full(n, 32, np.uint32)
    h = n // 2  # the second half repeats the first: hits in both feeds
    pk[h:], sig[h:], off[h:] = pk[:h], sig[:h], off[:h]
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    stub = ctypes.cast(hostcore.hc_stub_keyed if keyed else hostcore.hc_stub_verify, ctypes.c_void_p)
    res = []
    try:
        if keyed:
            host.svh_set_test_keyed_verifier(stub)
            host.svh_set_keyed_threshold(1)
        else:
            host.svh_set_test_verifier(stub)
            host.svh_set_keyed_threshold(0)
        for step in (n, 1000):
            host.svh_cache_clear()
            host.svh_cache_seed(5)
            host.svh_cache_counts(None, None)
            out = np.zeros(n, np.uint8)
            for a in range(0, n, step):
                b = min(n, a + step)
                rc = host.svh_verify_sig_batch(P(pk[a:]), P(sig[a:]), P(sl[a:]), P(msg), P(off[a:]), P(ln[a:]),
                                               ctypes.c_size_t(b - a), P(out[a:]))
                assert rc == 0, host.svh_last_error_string()
            keys = np.zeros((0x10000, 32), np.uint8)
            size = host.svh_cache_keys(P(keys), ctypes.c_size_t(0x10000))
            res.append((out.copy(), _counts(host), keys[:size].copy()))
    finally:
        host.svh_set_test_verifier(None)
        host.svh_set_test_keyed_verifier(None)
        host.svh_set_keyed_threshold(256)
        host.svh_cache_clear()
    (o0, c0, k0), (o1, c1, k1) = res
    assert (o0 == o1).all() and c0 == c1 and (k0 == k1).all()
    assert not o0[odd].any() and o0[sl == 64].all()
    assert sum(c0) == n - len(odd) and c0[0] > 0


@pytest.mark.parametrize("keyed", [False, True])
def test_cache_eviction_matches_sequential_reference(host, hostcore, keyed):
    """Overfill the 0xffff cache through verifySigBatch (3-phase pending
    inserts, or the keyed single walk) and compare the surviving keys, their
    order in the eviction vector, and the hit/miss counts with a sequential
    restatement of the reference cache fed the same items one by one."""
    rng = np.random.default_rng(4242)
    n_distinct = 72000
    pk = rng.integers(0, 256, (n_distinct, 32), dtype=np.uint8)
    sig = rng.integers(0, 256, (n_distinct, 64), dtype=np.uint8)
    msg = rng.integers(0, 256, (n_distinct, 32), dtype=np.uint8)
    # item stream: every distinct item once plus re-submissions of recent and old ones
    order = list(range(n_distinct))
    for k in range(6000):
        j = int(rng.integers(0, len(order)))
        order.insert(j + 1, order[max(0, j - int(rng.integers(0, 3000)))])
    order = np.array(order)
    if keyed:
        keys = [sig[i, :32].tobytes() for i in order]  # hc_stub_keyed's "key"
    else:
        keys = [hashlib.blake2b(pk[i].tobytes() + sig[i].tobytes() + msg[i].tobytes(), digest_size=32).digest()
                for i in order]
    ref = RefCache(seed=1234)
    hits = misses = 0
    for k in keys:
        if k in ref.map:
            hits += 1
            ref.get(k)
        else:
            misses += 1
            ref.put(k)
    stub = ctypes.cast(hostcore.hc_stub_keyed if keyed else hostcore.hc_stub_verify, ctypes.c_void_p)
    if keyed:
        host.svh_set_test_keyed_verifier(stub)
        host.svh_set_keyed_threshold(1)
    else:
        host.svh_set_test_verifier(stub)
        host.svh_set_keyed_threshold(0)
    host.svh_cache_clear()
    host.svh_cache_seed(1234)
    host.svh_cache_counts(None, None)
    try:
        P, S = pk[order], sig[order]
        M = np.ascontiguousarray(msg[order]).reshape(-1)
        off = np.arange(len(order), dtype=np.uint64) * 32
        ln = np.full(len(order), 32, np.uint32)
        out = np.zeros(len(order), np.uint8)
        pos = 0
        while pos < len(order):  # batches of varied sizes
            size = int(rng.choice([1, 7, 1000, 4096, 333, 20000]))
            hi = min(len(order), pos + size)
            rc = host.svh_verify_sig_batch(P[pos:hi].ctypes.data_as(ctypes.c_void_p),
                                           np.ascontiguousarray(S[pos:hi]).ctypes.data_as(ctypes.c_void_p), None,
                                           M.ctypes.data_as(ctypes.c_void_p),
                                           (off[pos:hi]).ctypes.data_as(ctypes.c_void_p),
                                           ln[pos:hi].ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(hi - pos),
                                           out[pos:hi].ctypes.data_as(ctypes.c_void_p))
            assert rc == 0, host.svh_last_error_string()
            pos = hi
        assert out.all()
        assert _counts(host) == (hits, misses)
        buf = np.zeros((0x10000, 32), np.uint8)
        size = host.svh_cache_keys(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(0x10000))
        assert size == len(ref.ptrs) == 0xFFFF
        got = [buf[i].tobytes() for i in range(size)]
        assert got == ref.ptrs
    finally:
        host.svh_set_test_verifier(None)
        host.svh_set_test_keyed_verifier(None)
        host.svh_set_keyed_threshold(256)
        host.svh_cache_clear()


@pytest.mark.gpu
def test_gpu_config3_full_5000_tx(host, sv, oracle):
    """BASELINE config 3 at full size: a 5000-tx set with 1-20 ED25519 signers
    per tx (plus PRE_AUTH_TX / HASH_X / signed-payload signers, colliding-hint
    wrong keys, unused and short signatures), checked after ONE GPU pre-pass
    (side table, and seeding the cache) and after the pipelined two-half
    pre-pass; outcomes == the independent Python
    replay of SignatureChecker.cpp:30-158 with oracle verdicts."""
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    import torch
    dev = torch.device("cuda", 0)

    def gpu_sign(reqs):
        seeds = np.frombuffer(b"".join(r[0] for r in reqs), np.uint8).reshape(-1, 32)
        msgs = np.frombuffer(b"".join(r[1] for r in reqs), np.uint8).reshape(-1, 32)
        n = len(reqs)
        ts, tm = torch.from_numpy(seeds.copy()).to(dev), torch.from_numpy(msgs.copy()).to(dev)
        tpk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        tsig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        sv.sign_device(0, ts.data_ptr(), tm.data_ptr(), n, tpk.data_ptr(), tsig.data_ptr(),
                       torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        pk, sg = tpk.cpu().numpy(), tsig.cpu().numpy()
        return [(pk[i].tobytes(), sg[i].tobytes()) for i in range(n)]

    txs = tg.generate(5000, gpu_sign, seed=2025)
    tg.add_payload_signatures(txs, _oracle_sign_fn(oracle))

    def verify(pk, sig, msg):
        return oracle.oracle_ed25519_verify(sig, msg, len(msg), pk) == 0

    want_ok, want_used = tg.replay(txs, verify)
    host.svh_set_test_verifier(None)
    for mode in (1, 2, 4):  # (4: the pipelined pre-pass, two engine batches)
        host.svh_cache_clear()
        ok, used, pairs = _check(host, txs, mode)
        assert (ok == want_ok).all() and (used == want_used).all(), mode
        assert pairs > 25000  # (~5.8 signatures per tx on average)
    assert 0 < want_ok.sum() < len(txs)
    host.svh_cache_clear()


_POOL_STRESS = r"""
import ctypes, sys
import numpy as np
host = ctypes.CDLL(sys.argv[1])
stub = ctypes.CDLL(sys.argv[2])
host.svh_set_test_verifier.argtypes = [ctypes.c_void_p]
host.svh_set_keyed_threshold.argtypes = [ctypes.c_size_t]
host.svh_set_test_verifier(ctypes.cast(stub.hc_stub_verify, ctypes.c_void_p))
host.svh_set_keyed_threshold(1 << 30)  # host-hashed: BLAKE2b keys over the helper pool
n = 1024
rng = np.random.default_rng(1)
pk = rng.integers(0, 256, (n, 32), dtype=np.uint8)
sig = rng.integers(0, 256, (n, 64), dtype=np.uint8)
msg = rng.integers(0, 256, 32 * n, dtype=np.uint8)
off = (np.arange(n, dtype=np.uint64) * 32)
ln = np.full(n, 32, np.uint32)
out = np.zeros(n, np.uint8)
for it in range(8000):
    host.svh_cache_clear()
    sig[:, 0] = it & 255
    sig[:, 1] = it >> 8
    rc = host.svh_verify_sig_batch(pk.ctypes.data_as(ctypes.c_void_p), sig.ctypes.data_as(ctypes.c_void_p), None,
                                   msg.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p),
                                   ln.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n),
                                   out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0 and out.all(), (it, rc)
print("ok")
"""


def test_helper_pool_many_runs_then_exit(host):
    """Regression: 8000 host-hashed batches, each fanned out over the helper
    pool (sv::Pool::run), then a normal interpreter exit.  A helper must never
    touch the caller's stack group after run() returned (pool.h): the old
    unlocked decrement left a helper asleep on a dead mutex and the process
    never exited (static ~Pool joins its threads)."""
    stub = os.path.join(REPO, "tests", "native", "libhostcore.so")
    r = subprocess.run([sys.executable, "-c", _POOL_STRESS, host._name, stub], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=90)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:]


_MEMO_CHILD = r"""
import ctypes, hashlib, json, sys
import numpy as np
lib = ctypes.CDLL(sys.argv[1])
lib.svh_verify_sig.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
lib.svh_cache_keys.restype = ctypes.c_size_t
lib.svh_cache_seed.argtypes = [ctypes.c_uint]
lib.svh_set_cpu_threshold.argtypes = [ctypes.c_size_t]
lib.svh_set_cpu_threshold(1 << 20)  # every miss on the CPU path (no GPU here)
lib.svh_cache_clear()
lib.svh_cache_seed(7)
d = np.load(sys.argv[2], allow_pickle=False)
rows = list(range(0, len(d["verdict"]), 3))[:180]
def item(i):
    o, l = int(d["msg_off"][i]), int(d["msg_len"][i])
    return d["pk"][i].tobytes(), d["sig"][i].tobytes(), d["msg"][o:o + l].tobytes()
out = {"verdicts": [], "counts": []}
def counts():
    h, m = ctypes.c_uint64(), ctypes.c_uint64()
    lib.svh_cache_counts(ctypes.byref(h), ctypes.byref(m))
    out["counts"].append([h.value, m.value])
for p in range(3):
    for i in rows:
        pk, sg, m = item(i)
        out["verdicts"].append(lib.svh_verify_sig(pk, sg, 64, m, len(m)))
        # the same signature and key over another message, and another key:
        # never the memoized key of the original bytes
        out["verdicts"].append(lib.svh_verify_sig(pk, sg, 64, m + b"x", len(m) + 1))
        if m:
            mm = bytearray(m); mm[-1] ^= 1
            out["verdicts"].append(lib.svh_verify_sig(pk, sg, 64, bytes(mm), len(m)))
        pk2 = bytearray(pk); pk2[0] ^= 1
        out["verdicts"].append(lib.svh_verify_sig(bytes(pk2), sg, 64, m, len(m)))
    counts()
n = lib.svh_cache_keys(None, 0)
buf = ctypes.create_string_buffer(32 * n)
lib.svh_cache_keys(buf, n)
out["keys"] = hashlib.sha256(buf.raw).hexdigest()
print(json.dumps(out))
"""


def test_key_memo_keeps_verify_cache_semantics(host, sv, golden, tmp_path):
    """The key memo (csrc/host/KeyMemo.h) skips re-deriving a cache key from
    byte-identical (pk, sig, msg) only: with it on and off the same verifySig
    sequence -- repeats, the same signature over altered messages, altered keys
    -- gives the same verdicts, the same hit / miss counts and the same cache
    contents (in the reference's eviction order, SecretKey.cpp:446-466)."""
    d = golden["msglen"]
    f = tmp_path / "msglen.npz"
    np.savez(f, **{k: d[k] for k in ("pk", "sig", "msg", "msg_off", "msg_len", "verdict")})
    res = {}
    for memo in ("1", "0"):
        env = dict(os.environ, SV_KEY_MEMO=memo, SV_NO_TORCH="1")
        r = subprocess.run([sys.executable, "-c", _MEMO_CHILD, sv.HOSTLIB_PATH, str(f)], env=env,
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        res[memo] = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["1"] == res["0"]
    assert res["1"]["counts"][1][1] == 0 and res["1"]["counts"][1][0] > 0  # the later passes all hit
