"""GPU parity of medium one-chunk host batches (csrc/sv_api.cpp host_slice_locked):
the image read in place from mapped memory, the verdicts written in place
(SV_BULK_ZC_OUT), on the medium geometry (quad) and the one-lane geometry.

Every verdict must equal the expected one (GPU-signed rows with known
corruptions; golden fixture rows with libsodium's verdicts) at the sizes
VERDICT r4 names (29,217 and 100k) and around the crossovers; consecutive
calls reuse the in-place image and verdict buffers.
"""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev(sv):
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def signed(sv, dev):
    """100k GPU-signed rows (32-byte messages), as numpy arrays."""
    n = 100000
    rng = np.random.default_rng(11)
    seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(dev)
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), n, pk.data_ptr(), sig.data_ptr(),
                   torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    return pk.cpu().numpy(), sig.cpu().numpy(), msgs.cpu().numpy()


def _corrupt(P, S, M, n, salt):
    p, s, m = P[:n].copy(), S[:n].copy(), M[:n].copy()
    want = np.ones(n, np.uint8)
    rng = np.random.default_rng(salt)
    rows = rng.choice(n, size=max(1, n // 13), replace=False)
    for k, r in enumerate(rows):
        w = k % 4
        if w == 0:
            s[r, 40] ^= 0x08   # S
        elif w == 1:
            s[r, 3] ^= 0x01    # R
        elif w == 2:
            m[r, 17] ^= 0x80   # message
        else:
            p[r, 9] ^= 0x02    # key
        want[r] = 0
    return p, s, m, want


@pytest.mark.parametrize("n", [12289, 16384, 16400, 29217, 32768, 32769, 50000, 100000])
def test_medium_fixed32_sizes(sv, dev, signed, n):
    P, S, M = signed
    p, s, m, want = _corrupt(P, S, M, n, n)
    out = sv.verify_fixed(p, s, m, 32, device=0)
    bad = np.nonzero(out != want)[0]
    assert len(bad) == 0, bad[:10]


def test_medium_back_to_back_changing_batches(sv, dev, signed):
    """Consecutive calls reuse the in-place image and the in-place verdicts:
    each call's verdicts are its own."""
    P, S, M = signed
    for k, n in enumerate([29217, 16384, 29217, 50000, 12289, 29217]):
        p, s, m, want = _corrupt(P, S, M, n, 1000 + k)
        out = sv.verify_fixed(p, s, m, 32, device=0)
        assert np.array_equal(out, want), (k, n)


@pytest.mark.parametrize("geom", ["quad", "one_lane"])
def test_medium_variable_length_fixture_rows(sv, dev, golden, geom):
    """Golden rows (every adversarial class, message lengths 0..300) tiled past
    the latency crossover on both geometries (per-key tables off: a one-lane
    launch with tables is covered by test_gpu_keytables.py)."""
    parts = [golden[n] for n in ("adversarial", "msglen", "valid", "lattice_edge")]
    pk = np.concatenate([d["pk"] for d in parts])
    sig = np.concatenate([d["sig"] for d in parts])
    verdict = np.concatenate([d["verdict"] for d in parts])
    msgs = [bytes(d["msg"][o:o + l]) for d in parts for o, l in zip(d["msg_off"], d["msg_len"])]
    reps = -(-20000 // len(msgs))
    pk_t, sig_t, want = np.tile(pk, (reps, 1)), np.tile(sig, (reps, 1)), np.tile(verdict, reps)
    msgs_t = msgs * reps
    lens = np.array([len(x) for x in msgs_t], np.uint32)
    offs = np.zeros(len(msgs_t), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(msgs_t), np.uint8)
    prev_kt = sv.set_key_tables(0)
    prev_dbg = sv.set_debug_flags(sv.DBG_QUAD if geom == "quad" else sv.DBG_NO_QUAD)
    try:
        out = sv.verify_batch(pk_t, sig_t, buf, offs, lens, device=0, path="throughput")
    finally:
        sv.set_debug_flags(prev_dbg)
        sv.set_key_tables(prev_kt)
    bad = np.nonzero(out != want)[0]
    assert len(bad) == 0, bad[:10]


@pytest.mark.parametrize("n", [1000, 12289, 29217, 50000])
def test_uniform_length_variable_batches(sv, dev, signed, n):
    """A variable-length call whose messages all have one length goes to the
    device as a fixed-length batch (sv_api.cpp uniform_form): messages found
    by their offsets (here shuffled, and rows sharing one message as a tx's
    pairs share its contents hash) and packed at a fixed stride."""
    P, S, M = signed
    p, s, m, want = _corrupt(P, S, M, n, 7000 + n)
    rng = np.random.default_rng(n)
    perm = rng.permutation(n)
    buf = np.ascontiguousarray(m[perm]).reshape(-1)  # message of row i at slot inv[i]
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    off = (inv * 32).astype(np.uint64)
    ln = np.full(n, 32, np.uint32)
    out = sv.verify_batch(p, s, buf, off, ln, device=0)
    assert np.array_equal(out, want), np.nonzero(out != want)[0][:10]
    # keyed: the cache keys are over the same bytes
    k = min(n, 2000)
    v2, k2 = sv.verify_batch_keyed(p[:k], s[:k], buf, off[:k], ln[:k], device=0)
    assert np.array_equal(v2, want[:k])
    for i in range(0, k, 97):
        o = int(off[i])
        h = hashlib.blake2b(p[i].tobytes() + s[i].tobytes() + buf[o:o + 32].tobytes(), digest_size=32).digest()
        assert k2[i].tobytes() == h, i


def test_uniform_length_shared_and_other_lengths(sv, dev, golden):
    """Rows sharing one message (one offset), and uniform lengths other than 32
    (every fixture row of one length), against libsodium's verdicts."""
    d = golden["msglen"]
    for L in sorted(set(int(x) for x in d["msg_len"]))[1::37]:
        rows = np.nonzero(d["msg_len"] == L)[0]
        if len(rows) == 0:
            continue
        reps = max(1, 400 // len(rows))
        r = np.tile(rows, reps)
        out = sv.verify_batch(d["pk"][r], d["sig"][r], d["msg"], d["msg_off"][r], d["msg_len"][r], device=0)
        assert np.array_equal(out, d["verdict"][r]), L
    # long messages (513 B .. 64 KiB - 1, every class): one length at a time,
    # the fixed path's read-from-memory branch on every kernel geometry
    d = golden["longmsg"]
    for L in sorted(set(int(x) for x in d["msg_len"])):
        rows = np.nonzero(d["msg_len"] == L)[0]
        for path in ("latency", "throughput"):
            out = sv.verify_batch(d["pk"][rows], d["sig"][rows], d["msg"], d["msg_off"][rows], d["msg_len"][rows],
                                  device=0, path=path)
            assert np.array_equal(out, d["verdict"][rows]), (L, path)
    v = golden["valid"]
    rows = np.nonzero(v["msg_len"] == 32)[0][:50]
    r = np.repeat(rows, 40)  # each message shared by 40 rows
    out = sv.verify_batch(v["pk"][r], v["sig"][r], v["msg"], v["msg_off"][r], v["msg_len"][r], device=0)
    assert np.array_equal(out, v["verdict"][r])
