#!/usr/bin/env python3
"""Derive every numeric constant the oracle and the HIP kernels need.

Nothing here is copied from libsodium: SHA-512's K/H0 are computed from their
FIPS 180-4 definition (fractional parts of cube / square roots of primes) and
the curve constants from RFC 8032 §5.1 (p, d, L, B).  Output is C source that
is pasted into oracle/ed25519_oracle.c and stellar-core_amd/csrc/*.h; the
unit test tests/test_constants.py re-derives them and compares.

Usage: python tools/gen_constants.py
"""

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRTM1 = pow(2, (P - 1) // 4, P)


def primes(n):
    out, k = [], 2
    while len(out) < n:
        if all(k % q for q in out if q * q <= k):
            out.append(k)
        k += 1
    return out


def iroot(x, k):
    """floor(x ** (1/k)) for big integers."""
    lo, hi = 0, 1
    while hi**k <= x:
        hi *= 2
    while lo < hi - 1:
        mid = (lo + hi) // 2
        if mid**k <= x:
            lo = mid
        else:
            hi = mid
    return lo


def frac_root_bits(p, k, bits=64):
    # first `bits` bits of the fractional part of p^(1/k)
    r = iroot(p << (k * bits), k)
    return r & ((1 << bits) - 1)


SHA512_K = [frac_root_bits(p, 3) for p in primes(80)]
SHA512_H0 = [frac_root_bits(p, 2) for p in primes(8)]


def base_point():
    y = (4 * pow(5, P - 2, P)) % P
    x2 = ((y * y - 1) * pow(D * y * y + 1, P - 2, P)) % P
    x = pow(x2, (P + 3) // 8, P)
    if (x * x - x2) % P != 0:
        x = (x * SQRTM1) % P
    if x & 1:
        x = P - x
    return x, y


BX, BY = base_point()

# radix 2^25.5 limb offsets used on the device: 0,26,51,77,102,128,153,179,204,230
R25_OFF = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
R25_W = [26, 25, 26, 25, 26, 25, 26, 25, 26, 25]


def limbs25(v):
    return [(v >> o) & ((1 << w) - 1) for o, w in zip(R25_OFF, R25_W)]


def limbs51(v):
    return [(v >> (51 * i)) & ((1 << 51) - 1) for i in range(5)]


def words32(v, n=8):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def main():
    print("/* SHA-512 K (FIPS 180-4 4.2.3) */")
    for i in range(0, 80, 2):
        print("  0x%016xULL, 0x%016xULL," % (SHA512_K[i], SHA512_K[i + 1]))
    print("/* SHA-512 H0 (FIPS 180-4 5.3.5) */")
    print(", ".join("0x%016xULL" % h for h in SHA512_H0))
    for name, v in [("d", D), ("2d", D2), ("sqrtm1", SQRTM1), ("Bx", BX), ("By", BY)]:
        print("/* %s */" % name)
        print("  r51: {" + ", ".join("0x%xULL" % x for x in limbs51(v)) + "}")
        print("  r25: {" + ", ".join("0x%07x" % x for x in limbs25(v)) + "}")
    print("/* L words32 */ {" + ", ".join("0x%08xu" % w for w in words32(L)) + "}")
    mu = (1 << 512) // L
    print("/* mu = floor(2^512/L), %d bits */ {" % mu.bit_length()
          + ", ".join("0x%08xu" % w for w in words32(mu, 9)) + "}")
    print("/* B encoding */", bytes(((BY | ((BX & 1) << 255)) >> (8 * i)) & 0xFF
                                     for i in range(32)).hex())


if __name__ == "__main__":
    main()
