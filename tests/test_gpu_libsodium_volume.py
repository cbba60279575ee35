"""GPU verdicts against libsodium itself, at volume.

The GPU box carries the image's conda libsodium 1.0.18 -- the library the
reference links (/root/reference/configure.ac:284-289) and calls from
PubKeyUtils::verifySig (/root/reference/src/crypto/SecretKey.cpp:461-463).
Here it is the checker for fresh random inputs at sizes the golden fixtures
do not reach: signatures from the engine's RFC 8032 signer, mutated into
twelve classes (bit flips in R, S, A and the message; S + L and S with its
top bits set; R and A replaced by the small-order blacklist with and without
bit 255; random A and R; A encodings with y >= p), each size picking another
kernel geometry through the host API:
  4,000    the latency lane's cold octet kernel
  24,000   the quad kernel (one signature per quad)
  131,077  the one-lane prep + main kernels (ragged last wave)
  2^20+3   BASELINE config 2's size: the staging pipeline over several chunks,
           two prep / main chunks per launch
libsodium runs through oracle/cpu_baseline.c's pthread harness (the same one
bench.py times), only as the checker.  Skipped where libsodium is absent.
"""
import ctypes
import hashlib
import os
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
SMALL_ORDER = [
    bytes(32),
    b"\x01" + bytes(31),
    bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"),
    bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"),
    (P - 1).to_bytes(32, "little"),
    P.to_bytes(32, "little"),
    (P + 1).to_bytes(32, "little"),
]
CLASSES = 12


def _sodium_path():
    for p in ("/opt/conda/lib/libsodium.so.23", "libsodium.so.23", "libsodium.so"):
        try:
            ctypes.CDLL(p)
            return p
        except OSError:
            continue
    return None


@pytest.fixture(scope="module")
def sodium_verdicts(oracle):
    path = _sodium_path()
    if path is None:
        pytest.skip("libsodium not present")
    oracle.cpubase_run.restype = ctypes.c_double
    oracle.cpubase_run.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_uint32, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    threads = max(1, min(16, len(os.sched_getaffinity(0))))

    def run(pk, sig, msg):
        out = np.zeros(pk.shape[0], np.uint8)
        dt = oracle.cpubase_run(path.encode(), pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, 32, pk.shape[0],
                                threads, out.ctypes.data)
        assert dt > 0, "libsodium harness failed (%s)" % dt
        return out
    return run


def _signed(sv, n, base):
    dev = torch.device("cuda", 0)
    s, m = bytearray(), bytearray()
    for i in range(base, base + n):
        p = struct.pack("<Q", i)
        s += hashlib.sha256(b"VOLSEED" + p).digest()
        m += hashlib.sha256(b"VOLMSG" + p).digest()
    ts = torch.from_numpy(np.frombuffer(bytes(s), np.uint8).reshape(n, 32).copy()).to(dev)
    tm = torch.from_numpy(np.frombuffer(bytes(m), np.uint8).reshape(n, 32).copy()).to(dev)
    tpk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    tsig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    sv.sign_device(0, ts.data_ptr(), tm.data_ptr(), n, tpk.data_ptr(), tsig.data_ptr(),
                   torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    return tpk.cpu().numpy(), tsig.cpu().numpy(), tm.cpu().numpy()


def _flip_bits(rng, arr, rows, lo, hi):
    pos = rng.integers(lo, hi, len(rows))
    arr[rows, pos] ^= (1 << rng.integers(0, 8, len(rows))).astype(np.uint8)


def _mutate(rng, pk, sig, msg):
    """Row i gets class i % CLASSES (0 = untouched), vectorized per class."""
    n = pk.shape[0]
    cls = np.arange(n) % CLASSES
    rows = [np.nonzero(cls == c)[0] for c in range(CLASSES)]
    _flip_bits(rng, sig, rows[1], 0, 32)  # R
    _flip_bits(rng, sig, rows[2], 32, 63)  # S (below its top byte)
    _flip_bits(rng, pk, rows[3], 0, 32)
    _flip_bits(rng, msg, rows[4], 0, 32)
    for i in rows[5]:  # S + L (< 2^253): non-canonical
        s = int.from_bytes(sig[i, 32:].tobytes(), "little") + L
        sig[i, 32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
    sig[rows[6], 63] |= np.uint8(0xE0)
    small = np.frombuffer(b"".join(SMALL_ORDER), np.uint8).reshape(-1, 32)
    for c, arr, col in ((7, sig, slice(0, 32)), (8, pk, slice(0, 32))):
        r = rows[c]
        arr[r, col] = small[rng.integers(0, len(small), len(r))]
        arr[r, 31] |= (rng.integers(0, 2, len(r)) * 0x80).astype(np.uint8)
    pk[rows[9]] = rng.integers(0, 256, (len(rows[9]), 32), dtype=np.uint8)
    sig[rows[10], :32] = rng.integers(0, 256, (len(rows[10]), 32), dtype=np.uint8)
    # y in [p, p + 19): non-canonical A encodings, sign bit either way
    big = np.frombuffer(b"".join((P + k).to_bytes(32, "little") for k in range(19)), np.uint8).reshape(-1, 32)
    r = rows[11]
    pk[r] = big[rng.integers(0, 19, len(r))]
    pk[r, 31] |= (rng.integers(0, 2, len(r)) * 0x80).astype(np.uint8)
    return cls


@pytest.mark.parametrize("n", [4000, 24000, 131077, (1 << 20) + 3])
def test_random_classes_against_libsodium(sv, sodium_verdicts, n):
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    pk, sig, msg = _signed(sv, n, base=n * 1000)
    cls = _mutate(np.random.default_rng(n), pk, sig, msg)
    want = sodium_verdicts(pk, sig, msg)
    # every class is present and the valid class is accepted in full
    assert (want[cls == 0] == 1).all() and 0 < int(want.sum()) < n
    assert all((cls == c).any() for c in range(CLASSES))
    if n <= 6144:
        sv.set_key_cache(0)  # (cold keys: the octet kernel)
    try:
        got = sv.verify_fixed(pk, sig, msg, 32, device=0)
    finally:
        if n <= 6144:
            sv.set_key_cache(1024)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(int(i), int(cls[i]), int(want[i])) for i in bad[:10]]
