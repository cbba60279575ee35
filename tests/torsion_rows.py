"""Mixed-order (torsion) signature rows whose libsodium verdict is known by
construction, for parity tests at volume (tests/test_torsion_scale.py).

libsodium 1.0.18 crypto_sign_verify_detached -- the call PubKeyUtils::verifySig
makes (/root/reference/src/crypto/SecretKey.cpp:461-463) -- is cofactorless:
it accepts iff encode([S]B - [h]A) == R byte for byte, with A and R allowed to
carry a torsion component (only the 7 small-order encodings themselves are
blacklisted).  Given an RFC 8032 key (secret a, nonce r for message M, so
A = aB and R = rB) and torsion points T_A = [kA]T8, T_R = [kR]T8 (T8 of order
8), the row

    A' = A + T_A,  R' = R + T_R,  h' = SHA-512(R' || A' || M) mod L,
    S' = r + h' a mod L

gives [S']B - [h']A' = rB - [h' kA]T8, so libsodium accepts it iff
kR == -h' kA (mod 8) and rejects it otherwise -- a reject that differs from an
accept only by a torsion point, which a verifier working mod L instead of
mod 8L (stellar-core_amd/csrc/lattice.h) would get wrong.  The generator
grinds (kA, kR) until the wanted verdict holds.  The same construction is the
torsion_AR_* class of tests/golden/make_lattice_edge.py, whose rows carry
libsodium's own verdicts; here it needs only hashlib, so it runs on the GPU
box at any volume.

a and r are re-derived from the seed as RFC 8032 does (the engine's GPU signer
and libsodium's crypto_sign_seed_keypair / crypto_sign_detached), and A, R are
taken from that signer's output, so no scalar multiplication runs in Python.
"""
import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)
# one of libsodium's blacklisted order-8 encodings (ge25519_has_small_order)
T8_ENC = bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05")


def _dec(s):
    """Extended point (X, Y, Z, T) of a 32-byte encoding (None if off-curve)."""
    y = int.from_bytes(s, "little") & ((1 << 255) - 1)
    sign = s[31] >> 7
    if y >= P:
        return None
    u, v = (y * y - 1) % P, (D * y * y + 1) % P
    x = u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P) % P
    if (v * x * x - u) % P != 0:
        if (v * x * x + u) % P != 0:
            return None
        x = x * SQRTM1 % P
    if x == 0 and sign:
        return None
    if x & 1 != sign:
        x = P - x
    return (x, y, 1, x * y % P)


def _add(p, q):
    """Extended twisted-Edwards addition (a = -1), complete."""
    x1, y1, z1, t1 = p
    x2, y2, z2, t2 = q
    a = (y1 - x1) * (y2 - x2) % P
    b = (y1 + x1) * (y2 + x2) % P
    c = 2 * D * t1 * t2 % P
    d = 2 * z1 * z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def _enc(p):
    x, y, z, _ = p
    zi = pow(z, P - 2, P)
    x, y = x * zi % P, y * zi % P
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


_T8 = _dec(T8_ENC)
TORSION = [(0, 1, 1, 0)]  # [k]T8, k = 0..7
for _k in range(7):
    TORSION.append(_add(TORSION[-1], _T8))


def rfc8032_secrets(seed, msg):
    """(a, r) of RFC 8032 signing: a = clamp(SHA-512(seed)[0:32]),
    r = SHA-512(SHA-512(seed)[32:64] || M) mod L."""
    hs = hashlib.sha512(seed).digest()
    a = bytearray(hs[:32])
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    r = int.from_bytes(hashlib.sha512(hs[32:] + msg).digest(), "little") % L
    return int.from_bytes(bytes(a), "little"), r


def _hram(R, A, msg):
    return int.from_bytes(hashlib.sha512(R + A + msg).digest(), "little") % L


def torsion_row(seed, msg, pk, sig, accept, kA=None, start=0):
    """(pk', sig', kA, kR) for the key/signature pair (pk, sig) that the RFC
    8032 signer made from (seed, msg): A' = A + [kA]T8 (kA != 0, so A' is
    mixed-order), R' = R + [kR]T8, S' = r + h' a; libsodium's verdict on the
    row is `accept` (module docstring).  kA given: only kR is ground (one key
    for several messages); else both, `start` varying the order so rows cover
    every (kA, kR) pair.  RuntimeError when no pair gives the verdict (with
    kA fixed an accept fails for about (7/8)^8 of messages)."""
    a, r = rfc8032_secrets(seed, msg)
    A, R = _dec(pk), _dec(sig[:32])
    assert A is not None and R is not None
    h = _hram(sig[:32], pk, msg)
    assert (r + h * a) % L == int.from_bytes(sig[32:], "little"), "signer is not RFC 8032"
    tries = [(kA, (start + t) % 8) for t in range(8)] if kA is not None else \
        [(1 + (start + t) % 7, (start // 7 + t) % 8) for t in range(56)]
    enc_a = {}
    for ka, kr in tries:
        if ka not in enc_a:
            enc_a[ka] = _enc(_add(A, TORSION[ka]))
        A2 = enc_a[ka]
        R2 = _enc(_add(R, TORSION[kr]))
        h2 = _hram(R2, A2, msg)
        if ((kr + h2 * ka) % 8 == 0) == accept:
            S2 = (r + h2 * a) % L
            return A2, R2 + S2.to_bytes(32, "little"), ka, kr
    raise RuntimeError("no torsion pair gives the wanted verdict")
