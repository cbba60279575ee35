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
// The Euclid runs as Lehmer steps (sv_lehmer_step): ~12 quotients at a time on
// the leading 53 bits in exact double arithmetic, then one 2x2 matrix applied
// to the 256-bit pair -- about 6 matrix applications and one exact step per
// signature instead of ~75 exact 256-bit steps (-2.9 % kernel time measured).
// The exact steps estimate their quotient in double precision and always
// UNDER-estimate it, so each is an exact integer step of the same Euclidean
// sequence (a short estimate only splits one quotient over two iterations).
#pragma once

#include <math.h>

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

// 1: Lehmer steps (below); 0: one 256-bit step per quotient only.

// d = u*x - v*y over 8 words (u, v < 2^32); returns true iff the exact value
// is negative (the values combined here are always within (-2^256, 2^256)).
SV_HD bool sv_lincomb8(uint32_t d[8], uint32_t u, const uint32_t x[8], uint32_t v, const uint32_t y[8]) {
  uint64_t cx = 0, cy = 0;
  uint32_t br = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    const uint64_t px = (uint64_t)u * x[i] + cx;
    const uint64_t py = (uint64_t)v * y[i] + cy;
    cx = px >> 32;
    cy = py >> 32;
    const uint64_t t = (uint64_t)(uint32_t)px - (uint32_t)py - br;
    d[i] = (uint32_t)t;
    br = (uint32_t)(t >> 63);
  }
  return (int64_t)cx - (int64_t)cy - (int64_t)br < 0;
}

// d = u*x + v*y (mod 2^256), u, v < 2^30
SV_HD void sv_addcomb8(uint32_t d[8], uint32_t u, const uint32_t x[8], uint32_t v, const uint32_t y[8]) {
  uint64_t c = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    uint64_t t = (uint64_t)u * x[i] + c;
    t += (uint64_t)v * y[i];
    d[i] = (uint32_t)t;
    c = t >> 32;
  }
}

// d = -d (two's complement) when neg
SV_HD void sv_condneg8(uint32_t d[8], bool neg) {
  const uint32_t m = neg ? 0xffffffffu : 0u;
  uint32_t c = neg ? 1u : 0u;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    const uint64_t t = (uint64_t)(d[i] ^ m) + c;
    d[i] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
  }
}

// Lehmer step (Knuth 4.5.2 Algorithm L, with Jebelean's a-priori test): runs
// Euclid on the leading 53 bits of (a, b) in exact double arithmetic and
// applies the accumulated 2x2 matrix to (a, b) and the cofactors once.
//   A = a / 2^sh, B ~ b / 2^sh (integers < 2^53), |a - A 2^sh|, |b - B 2^sh| < 8 2^sh.
//   After k steps r_k = (-1)^k (u_k A - v_k B) with u, v >= 0 (cofactor
//   magnitudes add: the matrix has a checkerboard sign pattern for ANY
//   quotients q >= 0), and the exact remainder with the same quotients is
//   2^sh (r_k + e_k), |e_k| < 8 (u_k + v_k).  A step is taken only if
//   r_{k+1} >= 8 (u_{k+1} + v_{k+1}) + 2^(128 - sh): then every exact remainder
//   stays >= 2^128 > 0, so (a', b') >= 0 and the cofactors keep opposite signs,
//   i.e. a' |tb'| + b' |ta'| = 8L still holds (the size bound the caller uses).
//   A quotient that is off by one only costs progress, never correctness; the
//   sign test after applying the matrix is a belt-and-braces guard.
// Returns false (state unchanged) if no step could be taken.
SV_HD bool sv_lehmer_step(uint32_t a[8], uint32_t b[8], uint32_t ta[8], uint32_t tb[8], bool& bneg) {
  const double ad = sv_words_to_double(a), bd = sv_words_to_double(b);
  int e;
  (void)frexp(ad, &e);
  const int sh = e - 53;  // a >= 2^128: sh >= 76
  const double T = ldexp(1.0, 128 - sh);
  double r0 = ldexp(ad, -sh), r1 = rint(ldexp(bd, -sh));
  double u0 = 1.0, v0 = 0.0, u1 = 0.0, v1 = 1.0;
  int k = 0;
  SV_NOUNROLL for (; k < 48; ++k) {
    double q = floor(r0 / r1);
    double r2 = fma(-q, r1, r0);
    if (r2 >= r1) {  // quotient rounded low
      r2 -= r1;
      q += 1.0;
    }
    const double u2 = fma(q, u1, u0), v2 = fma(q, v1, v0);
    if (!(r2 >= 8.0 * (u2 + v2) + T)) break;  // (also catches r2 < 0)
    r0 = r1;
    r1 = r2;
    u0 = u1;
    v0 = v1;
    u1 = u2;
    v1 = v2;
  }
  if (k == 0) return false;
  const uint32_t U0 = (uint32_t)u0, V0 = (uint32_t)v0, U1 = (uint32_t)u1, V1 = (uint32_t)v1;
  const bool odd = (k & 1) != 0;
  uint32_t na[8], nb[8];
  bool nega = sv_lincomb8(na, U0, a, V0, b);  // a' = (-1)^k (u0 a - v0 b)
  bool negb = sv_lincomb8(nb, U1, a, V1, b);  // b' = (-1)^(k+1) (u1 a - v1 b)
  sv_condneg8(na, odd);
  sv_condneg8(nb, !odd);
  nega = nega != odd;
  negb = negb == odd;
  if (nega || negb) return false;  // (unreachable by the bound above)
  uint32_t nta[8], ntb[8];
  sv_addcomb8(nta, U0, ta, V0, tb);
  sv_addcomb8(ntb, U1, ta, V1, tb);
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    a[i] = na[i];
    b[i] = nb[i];
    ta[i] = nta[i];
    tb[i] = ntb[i];
  }
  if (odd) bneg = !bneg;
  return true;
}

// h < L (8 words).  Always returns a valid pair (falls back to (h, 1)).
// trivial (test knob, sv_set_debug_flags SV_DBG_TRIVIAL_PAIR): skip the
// reduction and take the fallback pair (h, 1) -- the full-length equation.
SV_COLD void sc_lattice_reduce(sv_lat& o, const uint32_t h[8], bool trivial = false) {
  uint32_t a[8], b[8], ta[8], tb[8];
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    a[i] = sc_N8(i);
    b[i] = h[i];
    ta[i] = 0;
    tb[i] = 0;
  }
  tb[0] = 1;
  bool bneg = false;  // sign of t for b; t for a has the opposite sign
  bool bail = trivial;
  SV_NOUNROLL for (int it = 0; it < SV_LAT_MAX_ITERS && !trivial; ++it) {
    uint32_t hi = 0;
    SV_UNROLL for (int i = SV_LAT_SPLIT_WORDS; i < 8; ++i) hi |= b[i];
    if (hi == 0) break;
    if (sv_lehmer_step(a, b, ta, tb, bneg)) {
      if (sv_lt8(a, b)) {  // (a quotient rounded low)
        SV_UNROLL for (int i = 0; i < 8; ++i) {
          const uint32_t x = a[i], y = ta[i];
          a[i] = b[i];
          ta[i] = tb[i];
          b[i] = x;
          tb[i] = y;
        }
        bneg = !bneg;
      }
      continue;
    }
    // one exact Euclid step (a >= b)
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
