// Scalars mod L = 2^252 + 27742317777372353535851937790883648493 for one lane.
//
// Restates, from their definitions, libsodium 1.0.18's sc25519_is_canonical
// (S < L, step (1) of crypto_sign_verify_detached) and sc25519_reduce (512-bit
// SHA-512 output mod L, step (6)), plus the signed-digit recodings the
// fixed-window double-scalar multiplication consumes.  Reference call site:
// stellar-core src/crypto/SecretKey.cpp:461-463.
#pragma once

#include "sv_common.h"

// L and mu = floor(2^512 / L) (tools/gen_constants.py)
SV_HD uint32_t sc_L(int i) {
  const uint32_t l[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0, 0, 0, 0x10000000u};
  return l[i];
}
SV_HD uint32_t sc_mu(int i) {
  const uint32_t m[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                         0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
  return m[i];
}

// s < L (s as 8 little-endian words)
SV_HD bool sc_is_canonical(const uint32_t s[8]) {
  // borrow-propagating s - L: s < L iff the subtraction borrows out
  uint64_t br = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)s[i] - sc_L(i) - br;
    br = (d >> 63) & 1;
  }
  return br != 0;
}

// r = x mod L, x a 512-bit little-endian integer (16 words).  Barrett with
// base 2^32, k = 8: q3 = floor(floor(x / 2^224) * mu / 2^288),
// r = (x - q3 L) mod 2^288, then at most two subtractions of L.
SV_COLD void sc_reduce512(uint32_t r[8], const uint32_t x[16]) {
  uint32_t q2[18];
  SV_UNROLL for (int i = 0; i < 18; ++i) q2[i] = 0;
  // q2 = q1 * mu, q1 = x[7..15]
  SV_UNROLL for (int i = 0; i < 9; ++i) {
    uint64_t carry = 0;
    SV_UNROLL for (int j = 0; j < 9; ++j) {
      const uint64_t t = (uint64_t)x[7 + i] * sc_mu(j) + q2[i + j] + carry;
      q2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    q2[i + 9] = (uint32_t)carry;
  }
  // r2 = (q3 * L) mod 2^288, q3 = q2[9..17]
  uint32_t r2[9];
  SV_UNROLL for (int i = 0; i < 9; ++i) r2[i] = 0;
  SV_UNROLL for (int i = 0; i < 9; ++i) {
    uint64_t carry = 0;
    SV_UNROLL for (int j = 0; j < 8; ++j) {
      if (i + j < 9) {
        const uint64_t t = (uint64_t)q2[9 + i] * sc_L(j) + r2[i + j] + carry;
        r2[i + j] = (uint32_t)t;
        carry = t >> 32;
      }
    }
    if (i + 8 < 9) r2[i + 8] = (uint32_t)(r2[i + 8] + carry);
  }
  // r = x[0..8] - r2 (mod 2^288)
  uint32_t rr[9];
  uint64_t br = 0;
  SV_UNROLL for (int i = 0; i < 9; ++i) {
    const uint64_t d = (uint64_t)x[i] - r2[i] - br;
    rr[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
  // two conditional subtractions of L (branch-free)
  SV_UNROLL for (int rep = 0; rep < 2; ++rep) {
    uint32_t t[9];
    uint64_t b2 = 0;
    SV_UNROLL for (int i = 0; i < 9; ++i) {
      const uint64_t d = (uint64_t)rr[i] - (i < 8 ? sc_L(i) : 0u) - b2;
      t[i] = (uint32_t)d;
      b2 = (d >> 63) & 1;
    }
    const bool keep = b2 != 0;  // rr < L
    SV_UNROLL for (int i = 0; i < 9; ++i) rr[i] = keep ? rr[i] : t[i];
  }
  SV_UNROLL for (int i = 0; i < 8; ++i) r[i] = rr[i];
}

// Signed radix-16 digits of a scalar < 2^253: 64 digits in [-8, 7], digit i
// packed as 4-bit two's complement at bits 4(i%8) of out[i/8].
SV_HD void sc_digits_r16(uint32_t out[8], const uint32_t s[8]) {
  uint32_t carry = 0;
  SV_UNROLL for (int w = 0; w < 8; ++w) {
    uint32_t acc = 0;
    SV_UNROLL for (int k = 0; k < 8; ++k) {
      const uint32_t v = ((s[w] >> (4 * k)) & 15u) + carry;
      carry = (v + 8u) >> 4;       // v >= 8 (v <= 16)
      acc |= ((v - (carry << 4)) & 15u) << (4 * k);
    }
    out[w] = acc;
  }
}

// Signed radix-256 digits of a scalar < 2^253: 32 digits in [-128, 127],
// digit i packed as 8-bit two's complement at bits 8(i%4) of out[i/4].
SV_HD void sc_digits_r256(uint32_t out[8], const uint32_t s[8]) {
  uint32_t carry = 0;
  SV_UNROLL for (int w = 0; w < 8; ++w) {
    uint32_t acc = 0;
    SV_UNROLL for (int k = 0; k < 4; ++k) {
      const uint32_t v = ((s[w] >> (8 * k)) & 255u) + carry;
      carry = (v + 128u) >> 8;     // v >= 128 (v <= 256)
      acc |= ((v - (carry << 8)) & 255u) << (8 * k);
    }
    out[w] = acc;
  }
}

// Signed radix-2^16 digits of a scalar < 2^253: 16 digits in [-2^15, 2^15),
// digit i packed as 16-bit two's complement at bits 16(i%2) of out[i/2].
SV_HD void sc_digits_r65536(uint32_t out[8], const uint32_t s[8]) {
  uint32_t carry = 0;
  SV_UNROLL for (int w = 0; w < 8; ++w) {
    uint32_t acc = 0;
    SV_UNROLL for (int k = 0; k < 2; ++k) {
      const uint32_t v = ((s[w] >> (16 * k)) & 0xffffu) + carry;
      carry = (v + 0x8000u) >> 16;  // v >= 2^15 (v <= 2^16)
      acc |= ((v - (carry << 16)) & 0xffffu) << (16 * k);
    }
    out[w] = acc;
  }
}

// Pop the most significant packed digit: returns it sign-extended and shifts
// the 256-bit digit string left by `bits`.
SV_HD int32_t sc_pop_top(uint32_t d[8], int bits) {
  const int32_t top = ((int32_t)d[7]) >> (32 - bits);
  SV_UNROLL for (int i = 7; i > 0; --i) d[i] = (d[i] << bits) | (d[i - 1] >> (32 - bits));
  d[0] <<= bits;
  return top;
}
