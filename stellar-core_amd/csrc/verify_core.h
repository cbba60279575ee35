// Per-lane ed25519 verification core (one lane = one signature).
//
// Accept/reject is bit-exact with libsodium 1.0.18 crypto_sign_verify_detached,
// the function stellar-core's PubKeyUtils::verifySig calls on a cache miss
// (/root/reference/src/crypto/SecretKey.cpp:461-463).  Steps, in libsodium's
// order (all evaluated branch-free per lane; the verdict is their AND):
//   (1) S < L                              sc_is_canonical
//   (2) R not one of 7 small-order encodings (bit 255 masked)
//   (3) A canonical (y < p, sign ignored)   (4) A not small-order
//   (5) -A = decompress(A) succeeds
//   (6) h = SHA-512(R || A || M) mod L      (computed by the caller)
//   (7) R' = [h](-A) + [S]B, cofactorless
//   (8) encode(R') == R byte-for-byte
//
// Step (7) schedule (wave-uniform, no per-lane branches):
//   64 windows of 4 bits.  Per window: 4 doublings; add table_A[d_A] with
//   d_A in [-8, 8] (signed radix 16 of h); on every 4th window also add
//   table_B[d_B], d_B in [-2^15, 2^15] (signed radix 2^16 of S; SV_B_BITS).
//   table_A = {0..8}·(-A) in cached form, built per lane into a workspace
//   slot; table_B = {0..2^15}·B in affine precomp form, one global copy per
//   device.  Zero digits add the identity entry, so every lane does
//   identical work.  This full-length form (sv_double_scalarmult) serves the
//   signer and host builds; the verify kernels evaluate the half-size
//   equation of lattice.h (sv_lat_* below, sv_kernels.hip, sv_comb.hip).
#pragma once

#include "ge25519.h"
#include "lattice.h"
#include "sc25519.h"
#include "sha512_dev.h"

struct __attribute__((aligned(16))) sv_u4 {
  uint32_t x, y, z, w;
};

// Every table field element is padded to 12 dwords (3 quads) so a negative
// digit's (Y+X) <-> (Y-X) swap is an address choice at load time.
// B-table: entry e = e·B as 36 dwords: ypx[12] ymx[12] xy2d[12].  Signed
// radix-2^16 digits of S, one B addition every 4th window (16 per signature),
// 2^15 + 1 entries = 4.7 MB read from global memory (L2/MALL-resident).
#define SV_B_BITS 16
#define SV_BTAB_ENTRIES ((1 << (SV_B_BITS - 1)) + 1)
#define SV_BTAB_STRIDE 36
#define SV_BTAB_DWORDS (SV_BTAB_ENTRIES * SV_BTAB_STRIDE)
// A-table (HBM workspace): 9 entries x 11 quads: YpX (3 quads) YmX (3 quads)
// then Z and T2d packed back to back (20 dwords = 5 quads; only the pair that
// a negative digit swaps needs the 3-quad padding).
#define SV_ATAB_ENTRIES 9
#define SV_ATAB_QUADS 11
// Per-lane workspace slot of the signer (sv_sign_kernel): its table_A.
#define SV_SLOT_QUADS_W (SV_ATAB_ENTRIES * SV_ATAB_QUADS)
// Half-size path (lattice.h): tables of -A and -R, 9 entries x 10 quads each
// (YpX, YmX, Z, T2d as 4 x 10 dwords back to back; a negative digit swaps
// YpX/YmX by select after the load).
#define SV_LTAB_QUADS 10
#define SV_SLOT_QUADS_L (2 * SV_ATAB_ENTRIES * SV_LTAB_QUADS)
#define SV_SLOT_QUADS (SV_SLOT_QUADS_W > SV_SLOT_QUADS_L ? SV_SLOT_QUADS_W : SV_SLOT_QUADS_L)

SV_HD bool sv_small_order(const uint32_t s[8]) {
  const uint32_t bl[7][8] = {
      {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u},
      {0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u},
      {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u, 0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du},
      {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du, 0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u},
      {0xffffffecu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
      {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
      {0xffffffeeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu}};
  bool hit = false;
  SV_UNROLL for (int k = 0; k < 7; ++k) {
    uint32_t diff = (s[7] & 0x7fffffffu) ^ bl[k][7];
    SV_UNROLL for (int i = 0; i < 7; ++i) diff |= s[i] ^ bl[k][i];
    hit |= (diff == 0);
  }
  return hit;
}

// y < p with the sign bit ignored (libsodium ge25519_is_canonical)
SV_HD bool sv_point_canonical(const uint32_t s[8]) {
  uint32_t ones = (s[7] & 0x7fffffffu) ^ 0x7fffffffu;
  SV_UNROLL for (int i = 1; i < 7; ++i) ones |= s[i] ^ 0xffffffffu;
  return !(ones == 0 && s[0] >= 0xffffffedu);
}

SV_HD void sv_store_fe3(sv_u4* p, int qstride, const fe& f) {
  p[0] = sv_u4{f.v[0], f.v[1], f.v[2], f.v[3]};
  p[qstride] = sv_u4{f.v[4], f.v[5], f.v[6], f.v[7]};
  p[2 * qstride] = sv_u4{f.v[8], f.v[9], 0u, 0u};
}
SV_HD void sv_load_fe3(fe& f, const sv_u4* p, int qstride) {
  const sv_u4 a = p[0], b = p[qstride], c = p[2 * qstride];
  f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
  f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
  f.v[8] = c.x; f.v[9] = c.y;
}

// two field elements packed in 5 quads (20 dwords)
SV_HD void sv_store_fe_pair(sv_u4* p, int qstride, const fe& a, const fe& b) {
  p[0] = sv_u4{a.v[0], a.v[1], a.v[2], a.v[3]};
  p[qstride] = sv_u4{a.v[4], a.v[5], a.v[6], a.v[7]};
  p[2 * qstride] = sv_u4{a.v[8], a.v[9], b.v[0], b.v[1]};
  p[3 * qstride] = sv_u4{b.v[2], b.v[3], b.v[4], b.v[5]};
  p[4 * qstride] = sv_u4{b.v[6], b.v[7], b.v[8], b.v[9]};
}
SV_HD void sv_load_fe_pair(fe& a, fe& b, const sv_u4* p, int qstride) {
  const sv_u4 q0 = p[0], q1 = p[qstride], q2 = p[2 * qstride], q3 = p[3 * qstride], q4 = p[4 * qstride];
  a.v[0] = q0.x; a.v[1] = q0.y; a.v[2] = q0.z; a.v[3] = q0.w;
  a.v[4] = q1.x; a.v[5] = q1.y; a.v[6] = q1.z; a.v[7] = q1.w;
  a.v[8] = q2.x; a.v[9] = q2.y; b.v[0] = q2.z; b.v[1] = q2.w;
  b.v[2] = q3.x; b.v[3] = q3.y; b.v[4] = q3.z; b.v[5] = q3.w;
  b.v[6] = q4.x; b.v[7] = q4.y; b.v[8] = q4.z; b.v[9] = q4.w;
}

SV_HD void sv_store_cached(sv_u4* slot, int qstride, int e, const ge_cached& c) {
  sv_u4* base = slot + e * SV_ATAB_QUADS * qstride;
  sv_store_fe3(base, qstride, c.YpX);
  sv_store_fe3(base + 3 * qstride, qstride, c.YmX);
  sv_store_fe_pair(base + 6 * qstride, qstride, c.Z, c.T2d);
}

// table_A = {0..8}·(-A) in cached form, written to the lane's workspace slot.
SV_COLD void sv_build_atab(sv_u4* slot, int qstride, const ge_p3& negA) {
  ge_cached c1, ce;
  ge_p3_to_cached(c1, negA);
  ge_cached_identity(ce);
  sv_store_cached(slot, qstride, 0, ce);
  sv_store_cached(slot, qstride, 1, c1);
  ge_p3 P3 = negA;
  ge_p1p1 Q;
  SV_NOUNROLL for (int e = 2; e < SV_ATAB_ENTRIES; ++e) {
    ge_add_preswapped(Q, P3, c1.YpX, c1.YmX, c1.Z, c1.T2d, false, false);
    ge_p1p1_to_p3(P3, Q);
    ge_p3_to_cached(ce, P3);
    sv_store_cached(slot, qstride, e, ce);
  }
}

// Computes the projective point [h](-A) + [S]B with table_A of -A built in the
// lane's workspace slot: 64 windows (MSB first), per window 4 doublings, an
// addition of table_A[d_A] and, every 4th window, of table_B[d_B] (signed
// radix-2^16 digits of S).  Used by the signer (h = 0: only the identity entry
// of table_A is read) and by host builds; the verify kernels run the
// half-size equation (sv_main_scalarmult, the octet and comb kernels).
#define SV_BTAB_QUADS (SV_BTAB_STRIDE / 4)

#if defined(__HIP_DEVICE_COMPILE__)
// LDS-DMA of quad Q of an entry at per-lane address SRC + 16*OFF bytes into
// stage row ROW (lane-linear, 1 KiB per row).  The instruction's immediate
// offset is added to BOTH the global and the LDS address (tools/glds_off.hip,
// measured on MI355X), so the LDS pointer handed over is pre-biased by it:
// one per-lane base address serves all quads of an entry.  (With a pointer
// per quad the compiler hoisted ~30 64-bit addresses per window and kept them
// live: ~60 VGPRs, spilled at 3 waves/SIMD.)
#define SV_GLDS(SRC, OFF, STAGE, ROW)                                                                 \
  __builtin_amdgcn_global_load_lds(                                                                   \
      (const void*)(SRC),                                                                             \
      (__attribute__((address_space(3))) void*)((char*)((STAGE) + (ROW) * 64) - 16 * (OFF)), 16, 16 * (OFF), 0)
// A base-point table entry (affine: y+x, y-x, 2dxy; 4.7 MB tables, L2 /
// Infinity-Cache-hot) into a lane-linear LDS stage, the +/- swap of (y+x, y-x)
// done by the per-lane source address.
SV_HD void sv_stage_bentry(sv_u4* stageB, const sv_u4* btab, int32_t d) {
  const bool neg = d < 0;
  const sv_u4* e = btab + (neg ? -d : d) * SV_BTAB_QUADS;
  const sv_u4* ea = e + (neg ? 3 : 0);
  const sv_u4* eb = e + (neg ? 0 : 3);
  // rows 0-2 from ea, 3-5 from eb, 6-8 from e + 6.. (three base addresses)
  SV_GLDS(ea, 0, stageB, 0); SV_GLDS(ea, 1, stageB, 1); SV_GLDS(ea, 2, stageB, 2);
  SV_GLDS(eb, 0, stageB, 3); SV_GLDS(eb, 1, stageB, 4); SV_GLDS(eb, 2, stageB, 5);
  SV_GLDS(e, 6, stageB, 6); SV_GLDS(e, 7, stageB, 7); SV_GLDS(e, 8, stageB, 8);
  static_assert(SV_BTAB_QUADS == 9, "entry size");
}
#endif

SV_HD void sv_double_scalarmult(ge_p3& P, const ge_p3& negA, const uint32_t h[8], const uint32_t S[8],
                                sv_u4* slot, int qstride, const sv_u4* btab) {
  sv_build_atab(slot, qstride, negA);
  uint32_t da[8], db[8];
  sc_digits_r16(da, h);
  sc_digits_r65536(db, S);

  fe_0(P.X); fe_1(P.Y); fe_1(P.Z); fe_0(P.T);
  ge_p1p1 Q;
  SV_NOUNROLL for (int w = 63; w >= 0; --w) {
    const int nsteps = (w & (SV_B_BITS / 4 - 1)) ? 5 : 6;
    const int32_t dA = sc_pop_top(da, 4);
    const int32_t dB = nsteps == 6 ? sc_pop_top(db, SV_B_BITS) : 0;
    SV_NOUNROLL for (int s = 0; s < nsteps; ++s) {
      if (s < 4) {
        ge_dbl(Q, P.X, P.Y, P.Z);
      } else {
        fe qa, qb, qz, qt;
        bool neg;
        const bool zone = s == 5;
        if (!zone) {
          neg = dA < 0;
          const sv_u4* e = slot + (neg ? -dA : dA) * SV_ATAB_QUADS * qstride;
          sv_load_fe3(qa, e + (neg ? 3 : 0) * qstride, qstride);
          sv_load_fe3(qb, e + (neg ? 0 : 3) * qstride, qstride);
          sv_load_fe_pair(qz, qt, e + 6 * qstride, qstride);
        } else {
          neg = dB < 0;
          fe_1(qz);
          const sv_u4* e = btab + (neg ? -dB : dB) * SV_BTAB_QUADS;
          sv_load_fe3(qa, e + (neg ? 3 : 0), 1);
          sv_load_fe3(qb, e + (neg ? 0 : 3), 1);
          sv_load_fe3(qt, e + 6, 1);
        }
        ge_add_preswapped(Q, P, qa, qb, qz, qt, neg, zone);
      }
      ge_p1p1_to_p3_opt(P, Q, s + 1 >= 4 && s + 1 < nsteps);
    }
  }
}

SV_HD void sv_double_scalarmult_encode(uint32_t enc[8], const ge_p3& negA, const uint32_t h[8],
                                       const uint32_t S[8], sv_u4* slot, int qstride,
                                       const sv_u4* btab) {
  ge_p3 P;
  sv_double_scalarmult(P, negA, h, S, slot, qstride, btab);
  ge_p2_tobytes(enc, P.X, P.Y, P.Z);
}

// Steps (1)-(7) given the SHA-512(R||A||M) digest as a 512-bit LE integer:
// returns the verdict of checks (1)-(5) and the projective R' in P.  For a
// lane rejected by (1)-(5), P.Z is set to 1 so that a batch inversion over
// several signatures (sv_finalize_batch) can never be poisoned by a garbage
// point; its encoding is irrelevant to its (already false) verdict.
SV_HD bool sv_verify_pre(ge_p3& P, const uint32_t A[8], const sv_u4* Rp, const uint32_t S[8],
                         const uint32_t hram[16], sv_u4* slot, int qstride, const sv_u4* btab) {
  bool ok;
  {
    uint32_t R[8];
    const sv_u4 r0 = Rp[0], r1 = Rp[1];
    R[0] = r0.x; R[1] = r0.y; R[2] = r0.z; R[3] = r0.w;
    R[4] = r1.x; R[5] = r1.y; R[6] = r1.z; R[7] = r1.w;
    ok = sc_is_canonical(S) && !sv_small_order(R) && sv_point_canonical(A) && !sv_small_order(A);
  }
  ge_p3 negA;
  ok = ge_frombytes(negA, A, true) && ok;
  uint32_t h[8];
  sc_reduce512(h, hram);
  // Lanes with S >= L are already rejected by (1); clearing bits 253..255
  // keeps their recoding inside the table bounds.  Every S < 2^253 (so every
  // S < L, the lanes that can be accepted) is left unchanged.
  uint32_t Sc[8];
  SV_UNROLL for (int i = 0; i < 8; ++i) Sc[i] = S[i];
  Sc[7] &= 0x1fffffffu;
  sv_double_scalarmult(P, negA, h, Sc, slot, qstride, btab);
  if (!ok) fe_1(P.Z);
  return ok;
}

// Step (8): encode(X/Z, Y/Z) == R, given zi = 1/Z.
SV_HD bool sv_encode_matches(const fe& X, const fe& Y, const fe& zi, const sv_u4* Rp) {
  uint32_t enc[8];
  ge_p2_tobytes_zinv(enc, X, Y, zi);
  const sv_u4 r0 = Rp[0], r1 = Rp[1];
  const uint32_t diff = (enc[0] ^ r0.x) | (enc[1] ^ r0.y) | (enc[2] ^ r0.z) | (enc[3] ^ r0.w) |
                        (enc[4] ^ r1.x) | (enc[5] ^ r1.y) | (enc[6] ^ r1.z) | (enc[7] ^ r1.w);
  return diff == 0;
}

// Steps (1)-(8) for one signature (single inversion).  R is read from memory
// (Rp: its 2 quads) rather than kept live across the scalar multiplication.
SV_HD bool sv_verify_core(const uint32_t A[8], const sv_u4* Rp, const uint32_t S[8],
                          const uint32_t hram[16], sv_u4* slot, int qstride, const sv_u4* btab) {
  ge_p3 P;
  const bool ok = sv_verify_pre(P, A, Rp, S, hram, slot, qstride, btab);
  fe zi;
  fe_invert(zi, P.Z);
  return sv_encode_matches(P.X, P.Y, zi, Rp) && ok;
}

// Base-point table entry e = e·B in affine precomp form (used at init).
// Computes e·B by binary double-and-add from B (e <= 2^15) and normalises.
SV_HD void sv_btab_entry(uint32_t out[SV_BTAB_STRIDE], int e) {
  const uint32_t benc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                            0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  ge_p3 B, acc;
  ge_frombytes(B, benc, false);
  ge_cached bc;
  ge_p3_to_cached(bc, B);
  // acc = identity
  fe_0(acc.X); fe_1(acc.Y); fe_1(acc.Z); fe_0(acc.T);
  ge_p1p1 Q;
  for (int bit = SV_B_BITS - 1; bit >= 0; --bit) {
    ge_dbl(Q, acc.X, acc.Y, acc.Z);
    ge_p1p1_to_p3(acc, Q);
    if ((e >> bit) & 1) {
      ge_add_preswapped(Q, acc, bc.YpX, bc.YmX, bc.Z, bc.T2d, false, false);
      ge_p1p1_to_p3(acc, Q);
    }
  }
  fe zi, x, y, xy, d2, ypx, ymx, xy2d;
  fe_invert(zi, acc.Z);
  fe_mul(x, acc.X, zi);
  fe_mul(y, acc.Y, zi);
  fe_mul(xy, x, y);
  fe_const_2d(d2);
  fe_mul(xy2d, xy, d2);
  fe_add(ypx, y, x);
  fe_weak(ypx);
  fe_sub(ymx, y, x);
  fe_weak(ymx);
  for (int i = 0; i < SV_BTAB_STRIDE; ++i) out[i] = 0;
  for (int i = 0; i < 10; ++i) {
    out[i] = ypx.v[i];
    out[12 + i] = ymx.v[i];
    out[24 + i] = xy2d.v[i];
  }
}

// ---------------------------------------------------------------- signing
// RFC 8032 deterministic signing (== libsodium crypto_sign_seed_keypair +
// crypto_sign_detached), used only to synthesise benchmark datasets on the
// device.  [k]B runs through the same double-scalar routine with h = 0 (every
// table_A digit is 0, so only the identity entry is read).

// one-block SHA-512 of NW little-endian-packed words (NW*4 <= 111 bytes)
template <int NW>
SV_HD void sha512_words(uint32_t out[16], const uint32_t* in) {
  uint64_t st[8], w[16];
  sha512_init(st);
  SV_UNROLL for (int t = 0; t < 16; ++t) w[t] = 0;
  SV_UNROLL for (int t = 0; t < NW / 2; ++t) w[t] = sv_be64(in[2 * t], in[2 * t + 1]);
  w[NW / 2] = 0x8000000000000000ULL;
  w[15] = (uint64_t)NW * 32;
  sha512_compress(st, w);
  sha512_digest_le(out, st);
}

SV_HD void sc_muladd(uint32_t s[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t x[16];
  SV_UNROLL for (int i = 0; i < 16; ++i) x[i] = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
    SV_UNROLL for (int j = 0; j < 8; ++j) {
      const uint64_t t = (uint64_t)a[i] * b[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  uint64_t carry = 0;
  SV_UNROLL for (int i = 0; i < 16; ++i) {
    const uint64_t t = (uint64_t)x[i] + (i < 8 ? c[i] : 0u) + carry;
    x[i] = (uint32_t)t;
    carry = t >> 32;
  }
  sc_reduce512(s, x);
}

SV_HD void sv_sign_lane(uint32_t pk[8], uint32_t sig[16], const uint32_t seed[8], const uint32_t M[8],
                        sv_u4* slot, int qstride, const sv_u4* btab) {
  uint32_t az[16], wide[16], a[8], zero[8], enc[8];
  sha512_words<8>(az, seed);
  az[0] &= ~7u;
  az[7] &= 0x7fffffffu;
  az[7] |= 0x40000000u;
  SV_UNROLL for (int i = 0; i < 16; ++i) wide[i] = i < 8 ? az[i] : 0u;
  sc_reduce512(a, wide);
  SV_UNROLL for (int i = 0; i < 8; ++i) zero[i] = 0;
  ge_p3 ident;
  fe_0(ident.X); fe_1(ident.Y); fe_1(ident.Z); fe_0(ident.T);
  sv_double_scalarmult_encode(enc, ident, zero, a, slot, qstride, btab);  // A = aB
  SV_UNROLL for (int i = 0; i < 8; ++i) pk[i] = enc[i];
  uint32_t pm[16], nonce[16], r[8];
  SV_UNROLL for (int i = 0; i < 8; ++i) { pm[i] = az[8 + i]; pm[8 + i] = M[i]; }
  sha512_words<16>(nonce, pm);
  sc_reduce512(r, nonce);
  sv_double_scalarmult_encode(enc, ident, zero, r, slot, qstride, btab);  // R = rB
  uint32_t hram[16], h[8];
  sha512_ram32(hram, enc, pk, M);
  sc_reduce512(h, hram);
  uint32_t S[8];
  sc_muladd(S, h, a, r);
  SV_UNROLL for (int i = 0; i < 8; ++i) { sig[i] = enc[i]; sig[8 + i] = S[i]; }
}

// ------------------------------------------------ half-size path (lattice.h)
// Base-point tables for the half-size path: entry e of table t is e·(2^(128 t) B)
// (t = 0, 1), same 36-dword affine precomp layout as table_B.
// Half-size path base-point digits: signed radix 2^SV_LB_BITS (a multiple of
// the 4-bit window, dividing 128).  s = c1 S mod L (< 2^253) is recoded as ONE
// 256-bit signed digit string; digits 0..SV_LB_DIGITS-1 go to table 0 (e·B),
// the next SV_LB_DIGITS to table 1 (e·2^128 B), so the recoding carry out of
// the low half flows into the high half and never needs a digit of its own
// (16 base-point additions per signature at radix 2^16, was 18 when each half
// was recoded separately).  Digit j of both halves is added at window
// SV_LB_WIN * j.  Tables: e * 2^(128 t) * B for e in [0, 2^(SV_LB_BITS-1)].
// (Radix 2^20, 151 MB of tables, measured no faster than radix 2^16 (9.4 MB,
// L2/MALL-resident): the saved additions came back as exposed latency of the
// DMA'd entries.)
#ifndef SV_LB_BITS
#define SV_LB_BITS 16
#endif
static_assert(SV_LB_BITS % 4 == 0 && 128 % SV_LB_BITS == 0 && SV_LB_BITS <= 16, "base-point digit radix");
#define SV_LB_WIN (SV_LB_BITS / 4)
#define SV_LB_DIGITS (128 / SV_LB_BITS)
#define SV_LBTAB_ENTRIES ((1 << (SV_LB_BITS - 1)) + 1)

SV_HD void sv_btab_entry_shift(uint32_t out[SV_BTAB_STRIDE], int e, int shift) {
  const uint32_t benc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                            0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  ge_p3 B, acc;
  ge_frombytes(B, benc, false);
  ge_p1p1 Q;
  for (int i = 0; i < shift; ++i) {
    ge_dbl(Q, B.X, B.Y, B.Z);
    ge_p1p1_to_p3(B, Q);
  }
  ge_cached bc;
  ge_p3_to_cached(bc, B);
  fe_0(acc.X); fe_1(acc.Y); fe_1(acc.Z); fe_0(acc.T);
  for (int bit = SV_LB_BITS - 1; bit >= 0; --bit) {
    ge_dbl(Q, acc.X, acc.Y, acc.Z);
    ge_p1p1_to_p3(acc, Q);
    if ((e >> bit) & 1) {
      ge_add_preswapped(Q, acc, bc.YpX, bc.YmX, bc.Z, bc.T2d, false, false);
      ge_p1p1_to_p3(acc, Q);
    }
  }
  fe zi, x, y, xy, d2, ypx, ymx, xy2d;
  fe_invert(zi, acc.Z);
  fe_mul(x, acc.X, zi);
  fe_mul(y, acc.Y, zi);
  fe_mul(xy, x, y);
  fe_const_2d(d2);
  fe_mul(xy2d, xy, d2);
  fe_add(ypx, y, x);
  fe_weak(ypx);
  fe_sub(ymx, y, x);
  fe_weak(ymx);
  for (int i = 0; i < SV_BTAB_STRIDE; ++i) out[i] = 0;
  for (int i = 0; i < 10; ++i) {
    out[i] = ypx.v[i];
    out[12 + i] = ymx.v[i];
    out[24 + i] = xy2d.v[i];
  }
}

// cached entry as 40 packed dwords (10 quads): YpX YmX Z T2d
SV_HD void sv_store_lentry(sv_u4* p, const ge_cached& c) {
  uint32_t w[40];
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    w[i] = c.YpX.v[i];
    w[10 + i] = c.YmX.v[i];
    w[20 + i] = c.Z.v[i];
    w[30 + i] = c.T2d.v[i];
  }
  SV_UNROLL for (int q = 0; q < 10; ++q) p[q] = sv_u4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
}
// loads an entry with a digit's sign applied: (qa, qb) = (YpX, YmX) or swapped
SV_HD void sv_load_lentry(fe& qa, fe& qb, fe& qz, fe& qt, const sv_u4* p, int qstride, bool neg) {
  uint32_t w[40];
  SV_UNROLL for (int q = 0; q < 10; ++q) {
    const sv_u4 v = p[q * qstride];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    qa.v[i] = neg ? w[10 + i] : w[i];
    qb.v[i] = neg ? w[i] : w[10 + i];
    qz.v[i] = w[20 + i];
    qt.v[i] = w[30 + i];
  }
}

// {0..8}·P in cached form into tab (9 entries x 10 quads, lane-contiguous).
// P comes straight from ge_frombytes, so it is affine (Z = 1): each step adds
// it with the mixed law (2 Z1 Z2 = 2 Z1, no product).  Device builds do not
// write entry 0 (the identity): the main kernel stages digit 0 from one shared
// copy (sv_kernels.hip sv_ident_lentry), 1 in 9 table bytes fewer written and,
// for digit-0 windows, an L2-resident line read (A/B: -1.5 % / -4.9 % per 2^20
// on two boxes, profiles/r04/ab_mem/).  Host builds (the CPU path) keep it.
SV_COLD void sv_build_ltab(sv_u4* tab, const ge_p3& P) {
  ge_cached c1, ce;
  ge_p3_to_cached(c1, P);
  ge_cached_identity(ce);
#if !defined(__HIP_DEVICE_COMPILE__)
  sv_store_lentry(tab, ce);
#endif
  sv_store_lentry(tab + SV_LTAB_QUADS, c1);
  ge_p3 P3 = P;
  ge_p1p1 Q;
  SV_NOUNROLL for (int e = 2; e < SV_ATAB_ENTRIES; ++e) {
    ge_add_preswapped(Q, P3, c1.YpX, c1.YmX, c1.Z, c1.T2d, false, true);
    ge_p1p1_to_p3(P3, Q);
    ge_p3_to_cached(ce, P3);
    sv_store_lentry(tab + e * SV_LTAB_QUADS, ce);
  }
}

// Shifts a packed signed radix-16 digit string (64 digits) left by k digits.
SV_HD void sv_digits_shift(uint32_t d[8], int k) {
  SV_NOUNROLL while (k >= 8) {
    SV_UNROLL for (int i = 7; i > 0; --i) d[i] = d[i - 1];
    d[0] = 0;
    k -= 8;
  }
  SV_NOUNROLL for (; k > 0; --k) (void)sc_pop_top(d, 4);
}

// Per-signature digit strings of (*) in lattice.h for W windows:
//   dA: c0, dR: |c1| (signed radix 16, top digit = window W-1),
//   dB0[j], dB1[j] = signed radix-2^SV_LB_BITS digits j and SV_LB_DIGITS + j of
//   s = c1 S mod L (one string, sc_digits_lb); both are added at window
//   SV_LB_WIN * j, from the tables e·B and e·2^128 B.
// A scalar of 4W-1 bits can carry out of digit W-1: that digit is then -8 and
// the carry is 1, i.e. the top digit is really +8 (table entries go to 8);
// top8A / top8R record it (4-bit two's complement digits stop at 7).
struct sv_lat_digits {
  uint32_t dA[8], dR[8];
  int32_t dB0[SV_LB_DIGITS], dB1[SV_LB_DIGITS];
  bool rneg, top8A, top8R;
};

// Signed radix-2^SV_LB_BITS digits of x < 2^253 (8 words), as one string:
// d0 = digits 0..SV_LB_DIGITS-1 (weights 2^(B j)), d1 = the next SV_LB_DIGITS
// (weights 2^128 2^(B j)); every digit in [-2^(B-1), 2^(B-1)).  The top digit
// is < 2^(253-256+B) + 1 <= 2^(B-1), so no carry is left over.
SV_HD void sc_digits_lb(int32_t d0[SV_LB_DIGITS], int32_t d1[SV_LB_DIGITS], const uint32_t x[8]) {
  uint32_t carry = 0;
  SV_UNROLL for (int j = 0; j < 2 * SV_LB_DIGITS; ++j) {
    const int o = j * SV_LB_BITS, q = o >> 5, r = o & 31;  // (B divides 32: never straddles a word)
    uint32_t v = ((x[q] >> r) & ((1u << SV_LB_BITS) - 1u)) + carry;
    carry = (v + (1u << (SV_LB_BITS - 1))) >> SV_LB_BITS;  // v >= 2^(B-1)
    const int32_t d = (int32_t)v - (int32_t)(carry << SV_LB_BITS);
    if (j < SV_LB_DIGITS) d0[j] = d;
    else d1[j - SV_LB_DIGITS] = d;
  }
}

// The window's base-point digits, popped from the top (windows run MSB
// first, so the first window carrying one is SV_LB_WIN * (SV_LB_DIGITS - 1)).
SV_HD bool sv_lat_bdigits(sv_lat_digits& D, int w, int32_t& dB0, int32_t& dB1) {
  dB0 = dB1 = 0;
  if (w % SV_LB_WIN != 0 || w / SV_LB_WIN >= SV_LB_DIGITS) return false;
  dB0 = D.dB0[SV_LB_DIGITS - 1];
  dB1 = D.dB1[SV_LB_DIGITS - 1];
  SV_UNROLL for (int k = SV_LB_DIGITS - 1; k > 0; --k) {
    D.dB0[k] = D.dB0[k - 1];
    D.dB1[k] = D.dB1[k - 1];
  }
  D.dB0[0] = D.dB1[0] = 0;
  return true;
}

SV_COLD void sv_lat_prepare(sv_lat_digits& D, const sv_lat& lat, const uint32_t S[8], int W) {
  sc_digits_r16(D.dA, lat.c0);
  sc_digits_r16(D.dR, lat.c1);
  if (W < 64) {  // (W = 64 only for full-length scalars < 2^253: no carry out)
    sv_digits_shift(D.dA, 63 - W);
    sv_digits_shift(D.dR, 63 - W);
    D.top8A = sc_pop_top(D.dA, 4) != 0;  // digit W: the carry
    D.top8R = sc_pop_top(D.dR, 4) != 0;
  } else {
    D.top8A = D.top8R = false;
  }
  D.rneg = lat.c1neg;
  uint32_t s[8];
  sc_mul_signed(s, lat.c1, lat.c1neg, S);
  sc_digits_lb(D.dB0, D.dB1, s);  // s < L: low / high 128-bit halves, one carry chain
}

// The main kernel's entry stage: ONE 10-quad region per wave (10 KB); each
// entry is DMA'd when the previous addition's entry has been read, so its
// latency hides behind one addition (sv_main_scalarmult), and LDS is left for
// more waves per CU.
#if defined(__HIP_DEVICE_COMPILE__)
// one lane-contiguous 10-quad table entry into a lane-linear stage
SV_HD void sv_stage_lentry(sv_u4* stage, const sv_u4* entry) {
  SV_GLDS(entry, 0, stage, 0); SV_GLDS(entry, 1, stage, 1); SV_GLDS(entry, 2, stage, 2);
  SV_GLDS(entry, 3, stage, 3); SV_GLDS(entry, 4, stage, 4); SV_GLDS(entry, 5, stage, 5);
  SV_GLDS(entry, 6, stage, 6); SV_GLDS(entry, 7, stage, 7); SV_GLDS(entry, 8, stage, 8);
  SV_GLDS(entry, 9, stage, 9);
  static_assert(SV_LTAB_QUADS == 10, "entry size");
}
#endif

// P' = [s]B + [c0](-A) + [c1](-R) over W windows (MSB first).  tabA / tabR:
// the lane's tables of -A / -R; btab0 / btab1: e·B / e·(2^128 B).
// Step machine per window w: s = 0..3 doubling (skipped in the top window,
// where P is the identity), s = 4 add tabA[dA], s = 5 add tabR[+-dR], and on
// windows w = 4j, j < SV_LB_DIGITS: s = 6 add btab0[dB0_j], s = 7 add btab1[dB1_j].
// The host form (the CPU path, sv_cpu.cpp); the main kernel runs the same
// step machine with its entries staged by LDS-DMA (sv_main_scalarmult).
SV_HD void sv_lat_scalarmult(ge_p3& P, sv_lat_digits& D, int W, const sv_u4* tabA, const sv_u4* tabR,
                             const sv_u4* btab0, const sv_u4* btab1) {
  fe_0(P.X); fe_1(P.Y); fe_1(P.Z); fe_0(P.T);
  ge_p1p1 Q;
  SV_NOUNROLL for (int w = W - 1; w >= 0; --w) {
    int32_t dA = sc_pop_top(D.dA, 4);
    int32_t dR = sc_pop_top(D.dR, 4);
    if (w == W - 1) {
      if (D.top8A) dA = 8;
      if (D.top8R) dR = 8;
    }
    if (D.rneg) dR = -dR;
    int32_t dB0, dB1;
    const bool bwin = sv_lat_bdigits(D, w, dB0, dB1);
    const int nsteps = bwin ? 8 : 6;
    const int s0 = (w == W - 1) ? 4 : 0;
    SV_NOUNROLL for (int s = s0; s < nsteps; ++s) {
      if (s < 4) {
        ge_dbl(Q, P.X, P.Y, P.Z);
      } else {
        fe qa, qb, qz, qt;
        bool neg;
        const bool zone = s >= 6;
        if (!zone) {
          const int32_t d = s == 4 ? dA : dR;
          neg = d < 0;
          const sv_u4* e = (s == 4 ? tabA : tabR) + (neg ? -d : d) * SV_LTAB_QUADS;
          sv_load_lentry(qa, qb, qz, qt, e, 1, neg);
        } else {
          const int32_t d = s == 6 ? dB0 : dB1;
          neg = d < 0;
          fe_1(qz);
          const sv_u4* e = (s == 6 ? btab0 : btab1) + (neg ? -d : d) * SV_BTAB_QUADS;
          sv_load_fe3(qa, e + (neg ? 3 : 0), 1);
          sv_load_fe3(qb, e + (neg ? 0 : 3), 1);
          sv_load_fe3(qt, e + 6, 1);
        }
        ge_add_preswapped(Q, P, qa, qb, qz, qt, neg, zone);
      }
      ge_p1p1_to_p3_opt(P, Q, s + 1 >= 4 && s + 1 < nsteps);
    }
  }
}

// P' == identity: X == 0 and Y == Z (mod p)
SV_HD bool sv_is_identity(const ge_p3& P) {
  fe d;
  fe_sub(d, P.Y, P.Z);
  return fe_iszero(P.X) && fe_iszero(d);
}

// Steps (1)-(5) of libsodium plus the decode of R (lattice.h), the Euclid
// reduction and the table build.  Returns the pre-verdict and the lane's
// window count in *W_lane; the caller picks the wave's W >= every W_lane.
// a_status >= 0: A's checks and decode are already known --
// a_status != 0 iff A is canonical, not of small order and decodes (the
// per-key tables of the throughput path, sv_kernels.hip) -- and table_A is
// not built (the caller reads the key's cached table instead).
SV_COLD bool sv_lat_pre(sv_lat& lat, const uint32_t A[8], const uint32_t R[8], const uint32_t S[8],
                        const uint32_t hram[16], sv_u4* tabA, sv_u4* tabR, bool trivial = false,
                        int a_status = -1) {
  bool ok = sc_is_canonical(S) && !sv_small_order(R) && sv_point_canonical(R) &&
            (a_status >= 0 ? a_status != 0 : (sv_point_canonical(A) && !sv_small_order(A)));
  // one point live at a time: h first (hram dies), then decode + table of -A,
  // of -R, then the Euclid reduction with no point live
  uint32_t h[8];
  sc_reduce512(h, hram);
  if (a_status < 0) {
    ge_p3 negA;
    ok = ge_frombytes(negA, A, true) && ok;
    sv_build_ltab(tabA, negA);
  }
  {
    ge_p3 negR;
    ok = ge_frombytes(negR, R, true) && ok;
    sv_build_ltab(tabR, negR);
  }
  sc_lattice_reduce(lat, h, trivial);
  return ok;
}
