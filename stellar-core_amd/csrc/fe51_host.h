// GF(2^255 - 19) for the host CPU path (sv_cpu.cpp): radix 2^51, five 64-bit
// limbs, 64x64->128-bit products -- the shape x86-64 multiplies fastest (25
// products per multiplication instead of the device form's 100 32x32->64).
//
// Same interface and the same bound contract as fe25519.h's device form, so
// ge25519.h / lattice.h / verify_core.h run unchanged over it:
//   R  = output of mul / sq / weak: limbs < 2^51 + 2^14
//   fe_add(R, R) -> M2, fe_sub(f, g <= R) = f + 2p - g -> M3,
//   fe_sub4(f, g <= M3) = f + 4p - g -> M5; mul / sq accept limbs < 2^54
//   (5 * 19 * 2^54 * 2^54 < 2^128).
// Storage: the five limbs alias ten 32-bit words `v`, which is all the shared
// code touches when it packs an element into a table entry (a raw 40-byte
// copy), so tables built and read by the CPU path round-trip exactly.
//
// Selected by SV_HOST_FE51 (defined by sv_cpu.cpp only; tests/native builds
// the device form on the host to fuzz ITS limb bounds).  Reference semantics:
// libsodium 1.0.18 fe25519_* (ref10, 64-bit "fe51" form) as used by
// crypto_sign_verify_detached, called at stellar-core
// src/crypto/SecretKey.cpp:461-463 -- values mod p and canonical encodings
// only.
#pragma once

#include "sv_common.h"

typedef unsigned __int128 sv_u128;

struct fe {
  union {
    uint64_t l[5];
    uint32_t v[10];
  };
};

#define SV_M51 0x7ffffffffffffull

SV_HD void fe_0(fe& h) {
  for (int i = 0; i < 5; ++i) h.l[i] = 0;
}
SV_HD void fe_1(fe& h) {
  fe_0(h);
  h.l[0] = 1;
}
SV_HD void fe_add(fe& h, const fe& f, const fe& g) {
  for (int i = 0; i < 5; ++i) h.l[i] = f.l[i] + g.l[i];
}
// h = f - g + 2p; requires g <= R
SV_HD void fe_sub(fe& h, const fe& f, const fe& g) {
  h.l[0] = f.l[0] + 0xfffffffffffdaull - g.l[0];
  for (int i = 1; i < 5; ++i) h.l[i] = f.l[i] + 0xffffffffffffeull - g.l[i];
}
// h = f - g + 4p; requires g <= M3
SV_HD void fe_sub4(fe& h, const fe& f, const fe& g) {
  h.l[0] = f.l[0] + 0x1fffffffffffb4ull - g.l[0];
  for (int i = 1; i < 5; ++i) h.l[i] = f.l[i] + 0x1ffffffffffffcull - g.l[i];
}
SV_HD void fe_neg(fe& h, const fe& f) {
  fe z;
  fe_0(z);
  fe_sub(h, z, f);
}
// one parallel carry round: limbs < 2^63 in, R out
SV_HD void fe_weak(fe& h) {
  uint64_t c[5];
  for (int i = 0; i < 5; ++i) {
    c[i] = h.l[i] >> 51;
    h.l[i] &= SV_M51;
  }
  h.l[0] += 19 * c[4];
  for (int i = 1; i < 5; ++i) h.l[i] += c[i - 1];
}
// (radix 2^51: every limb carried, as fe_weak; the device form carries the
// even limbs only)
SV_HD void fe_weak_even(fe& h) { fe_weak(h); }

// column sums (< 2^120) -> R; the carries stay 128-bit
SV_HD void fe51_carry(fe& h, sv_u128 r0, sv_u128 r1, sv_u128 r2, sv_u128 r3, sv_u128 r4) {
  r1 += r0 >> 51;
  r2 += r1 >> 51;
  r3 += r2 >> 51;
  r4 += r3 >> 51;
  const sv_u128 l0 = (r0 & SV_M51) + 19 * (r4 >> 51);
  const uint64_t l1 = ((uint64_t)r1 & SV_M51) + (uint64_t)(l0 >> 51);
  h.l[0] = (uint64_t)l0 & SV_M51;
  h.l[1] = l1;
  h.l[2] = (uint64_t)r2 & SV_M51;
  h.l[3] = (uint64_t)r3 & SV_M51;
  h.l[4] = (uint64_t)r4 & SV_M51;
}

SV_HD void fe_mul(fe& h, const fe& f, const fe& g) {
  const uint64_t f0 = f.l[0], f1 = f.l[1], f2 = f.l[2], f3 = f.l[3], f4 = f.l[4];
  const uint64_t g0 = g.l[0], g1 = g.l[1], g2 = g.l[2], g3 = g.l[3], g4 = g.l[4];
  const uint64_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4;
  const sv_u128 r0 = (sv_u128)f0 * g0 + (sv_u128)f1 * g4_19 + (sv_u128)f2 * g3_19 + (sv_u128)f3 * g2_19 +
                     (sv_u128)f4 * g1_19;
  const sv_u128 r1 = (sv_u128)f0 * g1 + (sv_u128)f1 * g0 + (sv_u128)f2 * g4_19 + (sv_u128)f3 * g3_19 +
                     (sv_u128)f4 * g2_19;
  const sv_u128 r2 = (sv_u128)f0 * g2 + (sv_u128)f1 * g1 + (sv_u128)f2 * g0 + (sv_u128)f3 * g4_19 +
                     (sv_u128)f4 * g3_19;
  const sv_u128 r3 = (sv_u128)f0 * g3 + (sv_u128)f1 * g2 + (sv_u128)f2 * g1 + (sv_u128)f3 * g0 +
                     (sv_u128)f4 * g4_19;
  const sv_u128 r4 = (sv_u128)f0 * g4 + (sv_u128)f1 * g3 + (sv_u128)f2 * g2 + (sv_u128)f3 * g1 +
                     (sv_u128)f4 * g0;
  fe51_carry(h, r0, r1, r2, r3, r4);
}
// h = 2 f g
// (device form: a product with the 19-multiples of g given; here nothing to share)
struct fe19 {
  int unused;
};
SV_HD void fe_premul19(fe19& t, const fe& g) {
  (void)g;
  t.unused = 0;
}
SV_HD void fe_mul_g19(fe& h, const fe& f, const fe& g, const fe19& t) {
  (void)t;
  fe_mul(h, f, g);
}
SV_HD void fe_mul2(fe& h, const fe& f, const fe& g) {
  fe f2;
  for (int i = 0; i < 5; ++i) f2.l[i] = f.l[i] << 1;
  fe_mul(h, f2, g);
}
template <bool DBL>
SV_HD void fe51_sq(fe& h, const fe& f) {
  const uint64_t f0 = f.l[0], f1 = f.l[1], f2 = f.l[2], f3 = f.l[3], f4 = f.l[4];
  const uint64_t d0 = 2 * f0, d1 = 2 * f1, d2 = 2 * f2, d3 = 2 * f3;
  const uint64_t f3_19 = 19 * f3, f4_19 = 19 * f4;
  sv_u128 r0 = (sv_u128)f0 * f0 + (sv_u128)d1 * f4_19 + (sv_u128)d2 * f3_19;
  sv_u128 r1 = (sv_u128)d0 * f1 + (sv_u128)d2 * f4_19 + (sv_u128)f3 * f3_19;
  sv_u128 r2 = (sv_u128)d0 * f2 + (sv_u128)f1 * f1 + (sv_u128)d3 * f4_19;
  sv_u128 r3 = (sv_u128)d0 * f3 + (sv_u128)d1 * f2 + (sv_u128)f4 * f4_19;
  sv_u128 r4 = (sv_u128)d0 * f4 + (sv_u128)d1 * f3 + (sv_u128)f2 * f2;
  if (DBL) {
    r0 <<= 1;
    r1 <<= 1;
    r2 <<= 1;
    r3 <<= 1;
    r4 <<= 1;
  }
  fe51_carry(h, r0, r1, r2, r3, r4);
}
SV_HD void fe_sq(fe& h, const fe& f) { fe51_sq<false>(h, f); }
// h = 2 f^2
SV_HD void fe_sq2(fe& h, const fe& f) { fe51_sq<true>(h, f); }
SV_HD void fe_sqn(fe& h, const fe& f, int n) {
  fe_sq(h, f);
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

SV_HD void fe_cmov(fe& h, const fe& f, bool cond) {
  for (int i = 0; i < 5; ++i) h.l[i] = cond ? f.l[i] : h.l[i];
}

// 255-bit little-endian value (bit 255 ignored, value may be >= p) -> fe
SV_HD void fe_frombytes(fe& h, const uint32_t w[8]) {
  uint64_t q[4];
  for (int i = 0; i < 4; ++i) q[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  h.l[0] = q[0] & SV_M51;
  h.l[1] = ((q[0] >> 51) | (q[1] << 13)) & SV_M51;
  h.l[2] = ((q[1] >> 38) | (q[2] << 26)) & SV_M51;
  h.l[3] = ((q[2] >> 25) | (q[3] << 39)) & SV_M51;
  h.l[4] = (q[3] >> 12) & SV_M51;
}

// canonical little-endian encoding (value mod p, < p) as 8 words
SV_HD void fe_tobytes(uint32_t out[8], const fe& f) {
  uint64_t t[5];
  for (int i = 0; i < 5; ++i) t[i] = f.l[i];
  // two carry passes: limbs < 2^51, value < 2^255
  for (int pass = 0; pass < 2; ++pass) {
    for (int i = 0; i < 4; ++i) {
      t[i + 1] += t[i] >> 51;
      t[i] &= SV_M51;
    }
    t[0] += 19 * (t[4] >> 51);
    t[4] &= SV_M51;
  }
  // q = [value >= p] = [value + 19 >= 2^255]
  uint64_t q = (t[0] + 19) >> 51;
  for (int i = 1; i < 5; ++i) q = (t[i] + q) >> 51;
  t[0] += 19 * q;
  for (int i = 0; i < 4; ++i) {
    t[i + 1] += t[i] >> 51;
    t[i] &= SV_M51;
  }
  t[4] &= SV_M51;  // drops 2^255 (subtracts p together with the +19)
  const uint64_t o0 = t[0] | (t[1] << 51), o1 = (t[1] >> 13) | (t[2] << 38), o2 = (t[2] >> 26) | (t[3] << 25),
                 o3 = (t[3] >> 39) | (t[4] << 12);
  const uint64_t o[4] = {o0, o1, o2, o3};
  for (int i = 0; i < 4; ++i) {
    out[2 * i] = (uint32_t)o[i];
    out[2 * i + 1] = (uint32_t)(o[i] >> 32);
  }
}

SV_HD bool fe_iszero(const fe& f) {
  uint32_t s[8];
  fe_tobytes(s, f);
  uint32_t acc = 0;
  for (int i = 0; i < 8; ++i) acc |= s[i];
  return acc == 0;
}
SV_HD uint32_t fe_isnegative(const fe& f) {
  uint32_t s[8];
  fe_tobytes(s, f);
  return s[0] & 1u;
}

// z^(2^250 - 1) and z^11 (fe25519.h's chain)
SV_COLD void fe_pow_2_250_1(fe& z250, fe& z11, const fe& z) {
  fe t0, t1, t2, z9, z_5_0, z_10_0, z_20_0, z_50_0, z_100_0;
  fe_sq(t0, z);
  fe_sqn(t1, t0, 2);
  fe_mul(z9, t1, z);
  fe_mul(z11, z9, t0);
  fe_sq(t2, z11);
  fe_mul(z_5_0, t2, z9);
  fe_sqn(t0, z_5_0, 5);
  fe_mul(z_10_0, t0, z_5_0);
  fe_sqn(t0, z_10_0, 10);
  fe_mul(z_20_0, t0, z_10_0);
  fe_sqn(t0, z_20_0, 20);
  fe_mul(t0, t0, z_20_0);
  fe_sqn(t0, t0, 10);
  fe_mul(z_50_0, t0, z_10_0);
  fe_sqn(t0, z_50_0, 50);
  fe_mul(z_100_0, t0, z_50_0);
  fe_sqn(t0, z_100_0, 100);
  fe_mul(t0, t0, z_100_0);
  fe_sqn(t0, t0, 50);
  fe_mul(z250, t0, z_50_0);
}
SV_COLD void fe_pow22523(fe& h, const fe& z) {
  fe z250, z11;
  fe_pow_2_250_1(z250, z11, z);
  fe_sqn(z250, z250, 2);
  fe_mul(h, z250, z);
}
SV_COLD void fe_invert(fe& h, const fe& z) {
  fe z250, z11;
  fe_pow_2_250_1(z250, z11, z);
  fe_sqn(z250, z250, 5);
  fe_mul(h, z250, z11);
}

SV_HD void fe51_set(fe& h, const uint64_t c[5]) {
  for (int i = 0; i < 5; ++i) h.l[i] = c[i];
}
SV_HD void fe_const_d(fe& h) {
  const uint64_t c[5] = {0x34dca135978a3ull, 0x1a8283b156ebdull, 0x5e7a26001c029ull, 0x739c663a03cbbull,
                         0x52036cee2b6ffull};
  fe51_set(h, c);
}
SV_HD void fe_const_2d(fe& h) {
  const uint64_t c[5] = {0x69b9426b2f159ull, 0x35050762add7aull, 0x3cf44c0038052ull, 0x6738cc7407977ull,
                         0x2406d9dc56dffull};
  fe51_set(h, c);
}
SV_HD void fe_const_sqrtm1(fe& h) {
  const uint64_t c[5] = {0x61b274a0ea0b0ull, 0x0d5a5fc8f189dull, 0x7ef5e9cbd0c60ull, 0x78595a6804c9eull,
                         0x2b8324804fc1dull};
  fe51_set(h, c);
}
