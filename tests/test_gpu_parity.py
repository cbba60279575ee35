"""GPU parity: every verdict from the HIP path (through the C-ABI) must equal
libsodium 1.0.18 crypto_sign_verify_detached / the oracle, bit for bit.

Covers: all golden fixtures (reference in-tree vectors, libsodium valid set,
message lengths 0..300, every adversarial class) through the variable-length
host API; the fixed-32 fast path; the fixed-non-32 path (256-byte reference
benchmark shape, SecretKey.cpp:182-189); the device-resident API incl. the
ballot-compacted bitmap at ragged sizes; the GPU RFC 8032 signer against the
libsodium-generated dataset digests; and full-size (2^20) size-independent
properties (all-valid set accepted; exactly the corrupted rows rejected;
random rows cross-checked with the oracle).
"""
import ctypes
import hashlib
import json
import os
import struct
import threading

import numpy as np
import pytest

from conftest import GOLDEN, oracle_verdicts

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev(sv):
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(params=["auto", "throughput", "quad", "latency"])
def kpath(sv, request):
    """Runs the test on each kernel path (include/stellar_sigverify.h SV_PATH_*)
    and throughput-path geometry: the one-lane prep + main kernels
    (throughput, SV_DBG_NO_QUAD), one signature per quad (quad, SV_DBG_QUAD:
    the medium-batch kernel) and the octet latency kernel must give identical
    verdicts."""
    code = {"auto": sv.PATH_AUTO, "throughput": sv.PATH_THROUGHPUT, "quad": sv.PATH_THROUGHPUT,
            "latency": sv.PATH_LATENCY}[request.param]
    geom = {"throughput": sv.DBG_NO_QUAD, "quad": sv.DBG_QUAD}.get(request.param, 0)
    prev = sv.set_kernel_path(code)
    prev_dbg = sv.set_debug_flags(geom)
    yield request.param
    sv.set_kernel_path(prev)
    sv.set_debug_flags(prev_dbg)


def _seed_msg(lo, hi):
    s, m = bytearray(), bytearray()
    for i in range(lo, hi):
        p = struct.pack("<Q", i)
        s += hashlib.sha256(b"SVSEED" + p).digest()
        m += hashlib.sha256(b"SVMSG" + p).digest()
    return np.frombuffer(bytes(s), np.uint8).reshape(-1, 32), np.frombuffer(bytes(m), np.uint8).reshape(-1, 32)


def _gpu_sign(sv, dev, seeds, msgs):
    n = seeds.shape[0]
    ts = torch.from_numpy(np.array(seeds, copy=True)).to(dev)
    tm = torch.from_numpy(np.array(msgs, copy=True)).to(dev)
    tpk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    tsig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    sv.sign_device(0, ts.data_ptr(), tm.data_ptr(), n, tpk.data_ptr(), tsig.data_ptr(), st)
    torch.cuda.synchronize(dev)
    return tpk, tsig, tm


@pytest.mark.parametrize("name", ["intree", "valid", "msglen", "adversarial", "lattice_edge"])
def test_golden_fixtures_variable_path(sv, dev, golden, name, kpath):
    d = golden[name]
    out = sv.verify_batch(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"], device=0)
    bad = np.nonzero(out != d["verdict"])[0]
    assert len(bad) == 0, [(int(i), str(d["class_names"][d["cls"][i]])) for i in bad[:10]]


def test_per_call_path_flags(sv, dev, golden):
    """sv_opts.flags selects the kernel path per call; both give libsodium's
    verdicts; contradictory flags are rejected."""
    d = golden["adversarial"]
    for path in ("throughput", "latency"):
        out = sv.verify_batch(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"], device=0, path=path)
        assert (out == d["verdict"]).all(), path
    with pytest.raises(sv.SigVerifyError):  # both geometries forced at once
        sv.set_debug_flags(sv.DBG_QUAD | sv.DBG_NO_QUAD)
    with pytest.raises(sv.SigVerifyError):
        sv.verify_batch(d["pk"][:1], d["sig"][:1], d["msg"], d["msg_off"][:1], d["msg_len"][:1], device=0, path=3)


def test_intree_reference_expectations(sv, dev, golden):
    d = golden["intree"]
    out = sv.verify_batch(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"])
    iacr = d["expect"] >= 0
    assert (out[iacr] == d["expect"][iacr]).all()
    assert out.tolist()[:12] == [0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0]
    assert out[12:].sum() == 0  # all 196 Zcash vectors rejected


def test_fixed32_path_on_golden_rows(sv, dev, golden, kpath):
    for name in ("valid", "adversarial", "lattice_edge"):
        d = golden[name]
        rows = np.nonzero(d["msg_len"] == 32)[0]
        msgs = np.stack([d["msg"][o:o + 32] for o in d["msg_off"][rows]])
        out = sv.verify_fixed(d["pk"][rows], d["sig"][rows], msgs, 32)
        assert (out == d["verdict"][rows]).all(), name


def test_fixed_256_reference_bench_shape(sv, dev, golden, oracle, kpath):
    d = golden["valid"]
    rows = np.nonzero(d["msg_len"] == 256)[0]
    msgs = np.stack([d["msg"][o:o + 256] for o in d["msg_off"][rows]])
    sig = d["sig"][rows].copy()
    sig[::2, 5] ^= 0x20
    out = sv.verify_fixed(d["pk"][rows], sig, msgs, 256)
    want = np.array([oracle.oracle_ed25519_verify(sig[k].tobytes(), msgs[k].tobytes(), 256, d["pk"][rows[k]].tobytes())
                     == 0 for k in range(len(rows))], np.uint8)
    assert (out == want).all() and want.sum() == len(rows) // 2


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 63, 64, 65, 255, 256, 257, 1000, 4097, 12288, 12289])
def test_device_api_ragged_sizes_and_bitmap(sv, dev, oracle, n, kpath):
    seeds, msgs = _seed_msg(10_000, 10_000 + n)
    tpk, tsig, tm = _gpu_sign(sv, dev, seeds, msgs)
    sig = tsig.cpu().numpy()
    rng = np.random.default_rng(n)
    bad_rows = rng.choice(n, max(1, n // 7), replace=False)
    sig[bad_rows, rng.integers(0, 64, len(bad_rows))] ^= 0x04
    tsig.copy_(torch.from_numpy(sig))
    tv = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    tb = torch.full(((n + 63) // 64,), -1, dtype=torch.int64, device=dev)  # bits past n must come back 0
    st = torch.cuda.current_stream(dev).cuda_stream
    sv.verify_device(0, tpk.data_ptr(), tsig.data_ptr(), tm.data_ptr(), n, tv.data_ptr(), tb.data_ptr(), st)
    torch.cuda.synchronize(dev)
    got = tv.cpu().numpy()
    want = np.ones(n, np.uint8)
    want[bad_rows] = 0
    assert (got == want).all()
    words = tb.cpu().numpy().view(np.uint64)
    bits = np.array([(int(words[i // 64]) >> (i % 64)) & 1 for i in range(64 * len(words))], np.uint8)
    assert (bits[:n] == want).all() and not bits[n:].any()
    # a few rows against the oracle directly
    pk = tpk.cpu().numpy()
    for i in list(bad_rows[:3]) + [0, n - 1]:
        ok = oracle.oracle_ed25519_verify(sig[i].tobytes(), msgs[i].tobytes(), 32, pk[i].tobytes()) == 0
        assert ok == bool(got[i])


def test_zero_batch_is_noop(sv, dev):
    out = sv.verify_batch(np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8), np.zeros(0, np.uint8), [], [])
    assert out.shape == (0,)


def test_gpu_signer_reproduces_libsodium(sv, dev, golden):
    d = golden["valid"]
    rows = np.nonzero(d["msg_len"] == 32)[0][:1024]
    seeds, msgs = _seed_msg(0, len(rows))
    tpk, tsig, _ = _gpu_sign(sv, dev, seeds, msgs)
    assert np.array_equal(tpk.cpu().numpy(), d["pk"][rows])
    assert np.array_equal(tsig.cpu().numpy(), d["sig"][rows])


def test_gpu_signer_dataset_digest_64k(sv, dev):
    want = json.load(open(os.path.join(GOLDEN, "digests.json")))
    n = 65536
    seeds, msgs = _seed_msg(0, n)
    tpk, tsig, _ = _gpu_sign(sv, dev, seeds, msgs)
    stream = np.concatenate([tpk.cpu().numpy(), tsig.cpu().numpy(), msgs], axis=1).tobytes()
    assert hashlib.sha256(stream).hexdigest() == want[str(n)]


def test_full_size_properties_1m(sv, dev, oracle):
    """2^20 + 17 signatures (two prep/main chunks): all valid accepted, exactly
    the corrupted 1% rejected, verdict bytes and bitmap agree, 64 random rows
    agree with the oracle (size-independent properties)."""
    n = (1 << 20) + 17
    rng = np.random.default_rng(2025)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    tpk, tsig, tm = _gpu_sign(sv, dev, seeds, msgs)
    tv = torch.zeros(n, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    sv.verify_device(0, tpk.data_ptr(), tsig.data_ptr(), tm.data_ptr(), n, tv.data_ptr(), 0, st)
    torch.cuda.synchronize(dev)
    assert int(tv.sum(dtype=torch.int64).item()) == n
    bad = np.sort(rng.choice(n, n // 100, replace=False))
    sig = tsig.cpu().numpy()
    sig[bad, 32 + rng.integers(0, 32, len(bad))] ^= 0x01
    tsig.copy_(torch.from_numpy(sig))
    tb = torch.full(((n + 63) // 64,), -1, dtype=torch.int64, device=dev)  # bits past n must come back 0
    sv.verify_device(0, tpk.data_ptr(), tsig.data_ptr(), tm.data_ptr(), n, tv.data_ptr(), tb.data_ptr(), st)
    torch.cuda.synchronize(dev)
    got = tv.cpu().numpy()
    want = np.ones(n, np.uint8)
    want[bad] = 0
    assert np.array_equal(got, want)
    # the ballot bitmap across the 2^20-signature chunk boundary
    words = tb.cpu().numpy().view(np.uint64)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:n]
    assert np.array_equal(bits, want)
    pk = tpk.cpu().numpy()
    for i in rng.choice(n, 64, replace=False):
        ok = oracle.oracle_ed25519_verify(sig[i].tobytes(), msgs[i].tobytes(), 32, pk[i].tobytes()) == 0
        assert ok == bool(got[i])


def test_concurrent_host_calls(sv, dev, golden):
    d = golden["adversarial"]
    results = {}

    def run(k):
        results[k] = sv.verify_batch(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"], device=0)

    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for k in range(4):
        assert (results[k] == d["verdict"]).all()


def test_error_paths_raise(sv, dev):
    with pytest.raises(sv.SigVerifyError):
        sv.verify_batch(np.zeros((1, 32), np.uint8), np.zeros((1, 64), np.uint8), np.zeros(1, np.uint8), [0], [1],
                        device=64)
    buf = torch.zeros(256, dtype=torch.uint8, device=dev)
    with pytest.raises(sv.SigVerifyError):  # misaligned pk
        sv.verify_device(0, buf.data_ptr() + 1, buf.data_ptr() + 64, buf.data_ptr() + 128, 1, buf.data_ptr())
    with pytest.raises(sv.SigVerifyError):
        sv.verify_device(7, buf.data_ptr(), buf.data_ptr(), buf.data_ptr(), 1, buf.data_ptr())


def test_oracle_crosscheck_random_adversarial_gpu(sv, dev, oracle):
    """Fresh random garbage / mutations, GPU vs oracle (not only fixture rows)."""
    rng = np.random.default_rng(77)
    n = 512
    seeds, msgs = _seed_msg(500_000, 500_000 + n)
    tpk, tsig, _ = _gpu_sign(sv, dev, seeds, msgs)
    pk, sig = tpk.cpu().numpy(), tsig.cpu().numpy()
    for i in range(n):
        k = i % 6
        if k == 1:
            sig[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
        elif k == 2:
            pk[i, rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)
        elif k == 3:
            pk[i] = rng.integers(0, 256, 32)
        elif k == 4:
            sig[i, 32:] = rng.integers(0, 256, 32)
    out = sv.verify_fixed(pk, sig, msgs, 32)
    d = {"pk": pk, "sig": sig, "msg": msgs.reshape(-1), "msg_off": np.arange(n, dtype=np.uint64) * 32,
         "msg_len": np.full(n, 32, np.uint32), "verdict": out}
    want = oracle_verdicts(oracle, d)
    assert np.array_equal(out, want)


@pytest.mark.gpu
def test_gpu_cache_keys_and_keyed_verify(sv, golden):
    """f4: BLAKE2b-256(pk||sig||msg) cache keys on the GPU == hashlib; the keyed
    verify returns the same verdicts as the plain one (libsodium's)."""
    for name in ("intree", "msglen", "adversarial"):
        d = golden[name]
        keys = sv.cache_keys(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"])
        v2, k2 = sv.verify_batch_keyed(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"])
        assert (v2 == d["verdict"]).all(), name
        assert (k2 == keys).all(), name
        for i in range(0, len(keys), max(1, len(keys) // 300)):
            o, ln = int(d["msg_off"][i]), int(d["msg_len"][i])
            want = hashlib.blake2b(d["pk"][i].tobytes() + d["sig"][i].tobytes() + d["msg"][o:o + ln].tobytes(),
                                   digest_size=32).digest()
            assert keys[i].tobytes() == want, (name, i)


@pytest.mark.gpu
def test_gpu_sha256_batch(sv):
    """f4: batch SHA-256 on the GPU == hashlib for every length 0..300 and
    4 KiB tx-sized bodies at arbitrary (unaligned) offsets."""
    rng = np.random.default_rng(21)
    lens = np.array(list(range(0, 301)) + [4096, 4097, 65535], np.uint32)
    off = np.zeros(len(lens), np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 3)  # odd gaps: misaligned starts
    data = rng.integers(0, 256, int(off[-1] + lens[-1]), dtype=np.uint8)
    got = sv.sha256_batch(data, off, lens)
    for i in range(len(lens)):
        o, ln = int(off[i]), int(lens[i])
        assert got[i].tobytes() == hashlib.sha256(data[o:o + ln].tobytes()).digest(), ln
