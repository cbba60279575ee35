// Half-size scalars for the verification equation (one lane).
//
// libsodium (crypto_sign_verify_detached, called from stellar-core
// src/crypto/SecretKey.cpp:461-463) accepts iff encode([S]B - [h]A) == R,
// with h = SHA-512(R || A || M) mod L: a 253-bit scalar on the variable point
// A, i.e. ~253 doublings per signature.  This header finds, per signature, two
// integers (c0, c1) with
//
//     c0 == c1 * h  (mod 8L),   c1 odd,   |c0|, |c1| < 2^131 (almost always)
//
// so that the engine can instead evaluate
//
//     P' = [c1 S mod L] B + [c0](-A) + [c1](-R)                     (*)
//
// with ~130 doublings (the B part uses precomputed tables of B and 2^128 B).
// Why (*) decides exactly what libsodium decides (bit-exact, cofactorless):
//   * R is decoded as a point R_pt with encode(R_pt) == R (canonical y, on the
//     curve, sign bit = parity of x; x = 0 encodings are all on the small-order
//     blacklist that step (2) rejects).  If no such point exists libsodium's
//     byte comparison can never succeed, and the engine rejects too.  encode()
//     is injective, so libsodium accepts iff Q == R_pt, Q = [S]B - [h]A.
//   * E(F_p) is cyclic of order 8L, so [8L]X = 0 for every point X, and
//     [c0]A = [c1 h]A for EVERY A, including mixed-order keys (this is why the
//     modulus is 8L, not L).  B has order L, so [c1 S mod L]B = [c1 S]B.
//     Hence P' = [c1](Q - R_pt).
//   * c1 is odd and 0 < |c1| < L, so gcd(c1, 8L) = 1 and [c1] is a bijection
//     of the group: P' is the identity iff Q == R_pt.
// The pair comes from the extended Euclidean algorithm on (8L, h) stopped at
// the first remainder below 2^128 (rational reconstruction): r_i == t_i h and
// |t_i| <= 8L / r_{i-1} < 2^127 + 1.  If t_i is even, the previous pair
// (r_{i-1}, t_{i-1}) has odd t (consecutive t's are coprime) and the
// balanced combination r_{i-1} - k r_i, |t_{i-1}| + k |t_i| is used.  Any
// lane whose pair does not fit (or whose Euclid step would need a quotient
// >= 2^32) falls back to the trivial pair (h, 1), which is (*) with the full
// 253-bit scalar: correct, only slower for its wave.
//
// Quotients are estimated in double precision and always UNDER-estimated, so
// every step is an exact integer step of the same Euclidean sequence (a short
// estimate only splits one quotient over two iterations).
#pragma once

#include "sc25519.h"

// 8L (256 bits)
SV_HD uint32_t sc_N8(int i) {
  const uint32_t n[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0, 0, 0, 0x80000000u};
  return n[i];
}

SV_HD double sv_words_to_double(const uint32_t x[8]) {
  double d = 0.0;
  SV_UNROLL for (int i = 7; i >= 0; --i) d = d * 4294967296.0 + (double)x[i];
  return d;
}

SV_HD int sv_bitlen8(const uint32_t x[8]) {
  int b = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    if (x[i] != 0) b = 32 * i + (32 - __builtin_clz(x[i]));
  }
  return b;
}

// x < y (256-bit)
SV_HD bool sv_lt8(const uint32_t x[8], const uint32_t y[8]) {
  uint32_t br = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)x[i] - y[i] - br;
    br = (uint32_t)(d >> 63);
  }
  return br != 0;
}

// x -= q * y (caller guarantees q * y <= x)
SV_HD void sv_submul8(uint32_t x[8], uint32_t q, const uint32_t y[8]) {
  uint64_t carry = 0;
  uint32_t br = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    const uint64_t t = (uint64_t)q * y[i] + carry;
    carry = t >> 32;
    const uint64_t d = (uint64_t)x[i] - (uint32_t)t - br;
    x[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
}

// x += q * y (mod 2^256)
SV_HD void sv_addmul8(uint32_t x[8], uint32_t q, const uint32_t y[8]) {
  uint64_t carry = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    const uint64_t t = (uint64_t)q * y[i] + x[i] + carry;
    x[i] = (uint32_t)t;
    carry = t >> 32;
  }
}

struct sv_lat {
  uint32_t c0[8];  // c0 >= 0
  uint32_t c1[8];  // |c1|, odd
  bool c1neg;
  int bits;        // max(bitlen c0, bitlen |c1|)
};

#define SV_LAT_SPLIT_WORDS 4  // Euclid stops at the first remainder < 2^(32 * 4)
#define SV_LAT_MAX_ITERS 400  // > 1.45 * 256 (worst-case Euclid length)

// h < L (8 words).  Always returns a valid pair (falls back to (h, 1)).
SV_COLD void sc_lattice_reduce(sv_lat& o, const uint32_t h[8]) {
  uint32_t a[8], b[8], ta[8], tb[8];
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    a[i] = sc_N8(i);
    b[i] = h[i];
    ta[i] = 0;
    tb[i] = 0;
  }
  tb[0] = 1;
  bool bneg = false;  // sign of t for b; t for a has the opposite sign
  bool bail = false;
  SV_NOUNROLL for (int it = 0; it < SV_LAT_MAX_ITERS; ++it) {
    uint32_t hi = 0;
    SV_UNROLL for (int i = SV_LAT_SPLIT_WORDS; i < 8; ++i) hi |= b[i];
    if (hi == 0) break;
    const double qd = sv_words_to_double(a) / sv_words_to_double(b) * (1.0 - 0x1p-40);
    if (qd >= 4294967295.0) {  // (probability ~2^-32 per step) use (h, 1)
      bail = true;
      break;
    }
    uint32_t q = (uint32_t)qd;
    if (q == 0) q = 1;  // a >= b always holds here
    sv_submul8(a, q, b);
    sv_addmul8(ta, q, tb);
    if (sv_lt8(a, b)) {
      SV_UNROLL for (int i = 0; i < 8; ++i) {
        const uint32_t x = a[i], y = ta[i];
        a[i] = b[i];
        ta[i] = tb[i];
        b[i] = x;
        tb[i] = y;
      }
      bneg = !bneg;
    }
    if (it == SV_LAT_MAX_ITERS - 1) bail = true;
  }
  if (!bail) {
    if (tb[0] & 1u) {
      SV_UNROLL for (int i = 0; i < 8; ++i) {
        o.c0[i] = b[i];
        o.c1[i] = tb[i];
      }
      o.c1neg = bneg;
    } else {
      // t_{i-1} is odd: (a - k b, |ta| + k |tb|), k balancing the two
      const double num = sv_words_to_double(a) - sv_words_to_double(ta);
      const double den = sv_words_to_double(b) + sv_words_to_double(tb);
      double kd = num > 0.0 ? num / den * (1.0 - 0x1p-40) : 0.0;
      if (kd >= 4294967295.0) kd = 0.0;  // keep (a, ta); the size check decides
      const uint32_t k = (uint32_t)kd;
      SV_UNROLL for (int i = 0; i < 8; ++i) {
        o.c0[i] = a[i];
        o.c1[i] = ta[i];
      }
      sv_submul8(o.c0, k, b);   // k <= a / b
      sv_addmul8(o.c1, k, tb);  // (tb even: parity of ta kept)
      o.c1neg = !bneg;
    }
    const int b0 = sv_bitlen8(o.c0), b1 = sv_bitlen8(o.c1);
    o.bits = b0 > b1 ? b0 : b1;
    if (o.bits > 252) bail = true;
  }
  if (bail) {
    SV_UNROLL for (int i = 0; i < 8; ++i) {
      o.c0[i] = h[i];
      o.c1[i] = 0;
    }
    o.c1[0] = 1;
    o.c1neg = false;
    const int bh = sv_bitlen8(h);
    o.bits = bh > 1 ? bh : 1;
  }
}

// Windows (4 bits each, signed radix-16) needed for scalars of `bits` bits:
// the signed recoding of v < 2^(4W-1) fits W digits in [-8, 8].  At least
// SV_LAT_MIN_WINDOWS so the B split at 2^128 lands inside the window range.
#define SV_LAT_MIN_WINDOWS 33
SV_HD int sv_lat_windows(int bits) {
  const int w = (bits + 1 + 3) / 4;
  return w < SV_LAT_MIN_WINDOWS ? SV_LAT_MIN_WINDOWS : w;
}

// s = (+/-c1) * S mod L, S < 2^253, |c1| < 2^253.
SV_COLD void sc_mul_signed(uint32_t s[8], const uint32_t c1[8], bool neg, const uint32_t S[8]) {
  uint32_t x[16];
  SV_UNROLL for (int i = 0; i < 16; ++i) x[i] = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
    SV_UNROLL for (int j = 0; j < 8; ++j) {
      const uint64_t t = (uint64_t)c1[i] * S[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  uint32_t r[8];
  sc_reduce512(r, x);
  // neg: s = L - r (r != 0), else 0
  uint32_t nz = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) nz |= r[i];
  uint32_t br = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)sc_L(i) - r[i] - br;
    const uint32_t v = (uint32_t)d;
    br = (uint32_t)(d >> 63);
    s[i] = (neg && nz != 0) ? v : r[i];
  }
}
