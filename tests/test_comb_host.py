"""CPU checks of the warm-key latency path (stellar-core_amd/csrc/comb.h).

* The comb equation and table layout: a host build of the path's algorithm
  (tests/native/host_core.cpp hc_comb_verify_batch: per-key tables of
  d * 16^j * (-A), base tables of e * 256^j * B, 96-entry sums, projective test
  against the decoded R) must give libsodium's verdict on every golden row.
* The host key index (csrc/keycache.h: open addressing with backward-shift
  deletion, CLOCK eviction, second-sighting admission when full) against a map
  model under random and colliding traffic.
The GPU kernels themselves are checked in tests/test_gpu_comb.py.
"""
import ctypes

import numpy as np
import pytest


@pytest.mark.parametrize("name", ["intree", "lattice_edge", "valid", "msglen", "adversarial"])
def test_comb_model_matches_golden(hostcore, golden, name):
    d = golden[name]
    n = len(d["verdict"])
    if name in ("valid", "adversarial"):
        n = min(n, 1500)  # (keeps the CPU suite short; the GPU test runs every row)
    pk = np.ascontiguousarray(d["pk"][:n])
    sig = np.ascontiguousarray(d["sig"][:n])
    msg = np.ascontiguousarray(d["msg"])
    off = np.ascontiguousarray(d["msg_off"][:n])
    ln = np.ascontiguousarray(d["msg_len"][:n])
    out = np.zeros(n, np.uint8)
    f = hostcore.hc_comb_verify_batch
    f.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_void_p]
    f(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, off.ctypes.data, ln.ctypes.data, n, out.ctypes.data)
    bad = np.nonzero(out != d["verdict"][:n])[0]
    assert len(bad) == 0, [(int(i), str(d["class_names"][d["cls"][i]])) for i in bad[:10]]


@pytest.mark.parametrize("seed,cap,ops,universe", [(1, 16, 20000, 40), (2, 64, 50000, 70), (3, 64, 50000, 1000),
                                                   (4, 1024, 100000, 1500), (5, 1, 5000, 3)])
def test_key_index_fuzz(hostcore, seed, cap, ops, universe):
    f = hostcore.hc_keyindex_fuzz
    f.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    assert f(seed, cap, ops, universe) == 0


def test_comb_base_half_top_scalars(hostcore):
    """the comb path masks S before its radix-256 recoding.  The
    mask must leave every S < L unchanged, including S in [2^252, L) (bit 252
    set), which no valid signature can be constructed to reach (S = r + h a
    with h bound to R and A).  [S]B from the comb base tables against a plain
    Python scalar multiplication."""
    P = 2**255 - 19
    L = 2**252 + 27742317777372353535851937790883648493
    D = (-121665 * pow(121666, P - 2, P)) % P

    def add(p, q):  # extended coordinates, a = -1
        X1, Y1, Z1, T1 = p
        X2, Y2, Z2, T2 = q
        A = (Y1 - X1) * (Y2 - X2) % P
        B = (Y1 + X1) * (Y2 + X2) % P
        C = 2 * D * T1 * T2 % P
        Dd = 2 * Z1 * Z2 % P
        E, F, G, H = B - A, Dd - C, Dd + C, B + A
        return (E * F % P, G * H % P, F * G % P, E * H % P)

    def mul(k, p):
        r = (0, 1, 1, 0)
        while k:
            if k & 1:
                r = add(r, p)
            p = add(p, p)
            k >>= 1
        return r

    def enc(p):
        X, Y, Z, _ = p
        zi = pow(Z, P - 2, P)
        x, y = X * zi % P, Y * zi % P
        return (y | ((x & 1) << 255)).to_bytes(32, "little")

    by = 4 * pow(5, P - 2, P) % P
    x2 = (by * by - 1) * pow(D * by * by + 1, P - 2, P) % P
    bx = pow(x2, (P + 3) // 8, P)
    if (bx * bx - x2) % P:
        bx = bx * pow(2, (P - 1) // 4, P) % P
    if bx & 1:
        bx = P - bx
    B = (bx, by, 1, bx * by % P)
    f = hostcore.hc_comb_base_mul
    f.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    rng = np.random.default_rng(252)
    scalars = [L - 1, L - 2, 2**252, 2**252 + 1, 2**252 + 12345, 2**252 - 1, 1, 0]
    scalars += [2**252 + int(rng.integers(0, 2**62)) * 2**60 % (L - 2**252) for _ in range(4)]
    scalars += [int.from_bytes(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), "little") % L for _ in range(4)]
    for k in scalars:
        out = ctypes.create_string_buffer(32)
        f(k.to_bytes(32, "little"), out)
        assert out.raw == enc(mul(k, B)), hex(k)
