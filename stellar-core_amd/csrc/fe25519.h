// GF(2^255 - 19) arithmetic for one lane, written for gfx950 VALU issue.
//
// Representation: 10 unsigned limbs held in 32-bit VGPRs, radix 2^25.5
// (limb i has weight 2^ceil(25.5 i): offsets 0,26,51,77,102,128,153,179,204,230;
// even limbs 26 bits, odd limbs 25 bits when carried).
//
// Why this and not 8 x 32-bit limbs: on gfx950 v_mad_u64_u32 issues at the
// same rate as the carry-propagating v_add_co_u32 / v_addc_co_u32 (4.8 SIMD
// cycles per wave-instruction at 2 waves/SIMD, profiles/r02/ubench_valu_rates.txt),
// so cost = instruction count.  With 25.5-bit limbs
// every product-accumulate is ONE v_mad_u64_u32 into a carry-free 64-bit column
// sum (no per-product carry flags, no realignment of 64-bit register pairs),
// followed by a single carry chain per multiply.
//
// Bounds vocabulary ("M" = limb bound in units of 2^26 for even / 2^25 for odd
// limbs):  R  = output of mul/sq/carry (M ~ 1),  fe_add(R,R) -> M2,
// fe_sub(R,R) -> M3.  fe_mul/fe_sq accept inputs up to M3 (19 * 3 * 2^26 <
// 2^32 for the premultiplied operand; column sums < 2^62.8).  Callers that
// form 3-term expressions re-carry with fe_weak() (see ge25519.h).
//
// Reference semantics restated: libsodium 1.0.18 fe25519_* as used by
// crypto_sign_verify_detached (called from stellar-core
// src/crypto/SecretKey.cpp:461-463).  Only the mathematical result (values
// mod p and the canonical encoding) is relied on, never the internal layout.
#pragma once

#include "sv_common.h"

#if defined(SV_HOST_FE51) && !defined(__HIPCC__)
// host CPU path: radix 2^51 (fe51_host.h), same interface and bound contract
#include "fe51_host.h"
#else

struct fe {
  uint32_t v[10];
};
// 19 g[1..9] of a product's g operand, computed once when two products share
// g (fe_mul_g19)
struct fe19 {
  uint32_t v[9];
};

#define SV_M26 0x3ffffffu
#define SV_M25 0x1ffffffu

SV_HD uint32_t fe_mask(int i) { return (i & 1) ? SV_M25 : SV_M26; }
SV_HD int fe_width(int i) { return (i & 1) ? 25 : 26; }
SV_HD int fe_off(int i) { return 26 * ((i + 1) / 2) + 25 * (i / 2); }

SV_HD void fe_0(fe& h) {
  SV_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = 0;
}
SV_HD void fe_1(fe& h) {
  fe_0(h);
  h.v[0] = 1;
}

// h = f + g
SV_HD void fe_add(fe& h, const fe& f, const fe& g) {
  SV_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}

// h = f - g + 2p; requires g <= R (limbs within 2p's limbs)
SV_HD void fe_sub(fe& h, const fe& f, const fe& g) {
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    const uint32_t b = (i == 0) ? 0x7ffffdau : ((i & 1) ? 0x3fffffeu : 0x7fffffeu);
    h.v[i] = f.v[i] + b - g.v[i];
  }
}

// h = f - g + 4p; requires g <= M3
SV_HD void fe_sub4(fe& h, const fe& f, const fe& g) {
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    const uint32_t b = (i == 0) ? 0xfffffb4u : ((i & 1) ? 0x7fffffcu : 0xffffffcu);
    h.v[i] = f.v[i] + b - g.v[i];
  }
}

// h = -f (= 2p - f); requires f <= R
SV_HD void fe_neg(fe& h, const fe& f) {
  fe z;
  fe_0(z);
  fe_sub(h, z, f);
}

// Parallel one-round carry: every limb keeps its low width bits and receives
// the carry of its neighbour (limb 0 receives 19 * carry of limb 9).  For
// inputs with limbs < 2^31 the output is R+ (limbs <= 2^26 + 2^6 / 2^25 + 2^6,
// limb 0 <= 2^26 + 19 * 2^6): accepted wherever R is.
SV_HD void fe_weak(fe& h) {
  uint32_t c[10];
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    c[i] = h.v[i] >> fe_width(i);
    h.v[i] &= fe_mask(i);
  }
  h.v[0] += 19u * c[9];
  SV_UNROLL for (int i = 1; i < 10; ++i) h.v[i] += c[i - 1];
}

// Carry of the even limbs 2, 4, 6, 8 only (into 3, 5, 7, 9): enough to use an
// M5 value as a product's g operand.  g's limbs 1..9 are pre-multiplied by 19
// (19 g_j < 2^32 needs g_even <= 3.37 2^26, g_odd <= 6.7 2^25; limb 0 never is),
// so after this even limbs are R and odd ones <= 5 2^25 + 5; the column sums
// stay < 2^63 with an M5 f operand (tests/test_host_arith.py fuzzes it).
SV_HD void fe_weak_even(fe& h) {
  SV_UNROLL for (int i = 2; i < 10; i += 2) {
    const uint32_t c = h.v[i] >> 26;
    h.v[i] &= SV_M26;
    h.v[i + 1] += c;
  }
}

// One 32x32->64 multiply-accumulate = one v_mad_u64_u32.  Written as inline
// asm so the multiplicands are guaranteed 32-bit VGPRs: with plain C, LLVM
// promotes limbs merged across branches to i64 and the backend then emits
// 64x32-bit products (2 v_mad_u64_u32 + 2 v_mov each).  The carry-out SGPR
// pair is architecturally required on gfx950 (no `null` sdst); vcc is used
// and never read.
// Carry-out SGPR pairs the inline-asm mads rotate over (SV_MAD_PAIRS):
// a VALU write of the SAME SGPR pair by consecutive mads serialises them
// (tools/ubench_valu.hip: 9.5 vs 6.4 cycles per wave-instruction at one wave
// per SIMD), so product k writes pair k mod SV_MAD_PAIRS from the top of the
// SGPR file (never read; declared clobbered so the allocator avoids them).
#ifndef SV_MAD_PAIRS
#define SV_MAD_PAIRS 4
#endif
// (k must fold to a constant: every caller is a fully unrolled loop)
#define SV_MAD_I(L, H) \
  asm("v_mad_u64_u32 %0, s[" #L ":" #H "], %1, %2, 0" : "=v"(acc) : "v"(a), "v"(b) : "s" #L, "s" #H)
#define SV_MAD_A(L, H) \
  asm("v_mad_u64_u32 %0, s[" #L ":" #H "], %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "s" #L, "s" #H)
#define SV_MAD_SWITCH(M)      \
  switch (k % SV_MAD_PAIRS) { \
    case 0: M(94, 95); break; \
    case 1: M(92, 93); break; \
    case 2: M(90, 91); break; \
    case 3: M(88, 89); break; \
    case 4: M(86, 87); break; \
    case 5: M(84, 85); break; \
    case 6: M(82, 83); break; \
    default: M(80, 81); break; \
  }
SV_HD void sv_mad_init_k(uint64_t& acc, uint32_t a, uint32_t b, int k) {
#if defined(__HIP_DEVICE_COMPILE__)
  SV_MAD_SWITCH(SV_MAD_I)
#else
  (void)k;
  acc = (uint64_t)a * b;
#endif
}
SV_HD void sv_mad_k(uint64_t& acc, uint32_t a, uint32_t b, int k) {
#if defined(__HIP_DEVICE_COMPILE__)
  SV_MAD_SWITCH(SV_MAD_A)
#else
  (void)k;
  acc += (uint64_t)a * b;
#endif
}
SV_HD void sv_mad_init(uint64_t& acc, uint32_t a, uint32_t b) { sv_mad_init_k(acc, a, b, 0); }
SV_HD void sv_mad(uint64_t& acc, uint32_t a, uint32_t b) { sv_mad_k(acc, a, b, 0); }

// Column-major forms with the carry chain folded into the multiply-adds:
// column k (terms i + j = k and i + j = k + 10) is opened by a mad whose
// addend is the carry out of column k - 1, so each carry step is one 64-bit
// shift and one mask, and no separate 64-bit add per column (9 fewer per
// product than summing the columns first and carrying after).  The price is one dependent chain per product instead of
// ten interleaved accumulators.  Bounds: the carry (< 2^38) adds nothing
// measurable to a column sum (< 2^62.8), and the output is R as above.
// One column as ONE inline-asm statement (z: the first mad opens with 0, a:
// with acc).  Per-mad statements cost an s_nop between every two dependent
// ones: LLVM's gfx950 hazard recognizer assumes any inline asm may carry the
// dst-sel forwarding hazard (16-bit SDWA / op_sel destinations), which
// v_mad_u64_u32 does not have, and pads a consumer statement by one wait
// state.  Inside one statement the mads issue back to back; a dependent chain
// costs nothing extra on gfx950 (tools/ubench_valu_rates: dependency distance
// 1, 2 and 4 issue at the independent rate).
#if defined(__HIP_DEVICE_COMPILE__)
SV_HD void sv_col10_z(uint64_t& acc, const uint32_t a[10], const uint32_t b[10]) {
  asm(
      "v_mad_u64_u32 %0, s[94:95], %1, %11, 0\n"
      "v_mad_u64_u32 %0, s[92:93], %2, %12, %0\n"
      "v_mad_u64_u32 %0, s[90:91], %3, %13, %0\n"
      "v_mad_u64_u32 %0, s[88:89], %4, %14, %0\n"
      "v_mad_u64_u32 %0, s[94:95], %5, %15, %0\n"
      "v_mad_u64_u32 %0, s[92:93], %6, %16, %0\n"
      "v_mad_u64_u32 %0, s[90:91], %7, %17, %0\n"
      "v_mad_u64_u32 %0, s[88:89], %8, %18, %0\n"
      "v_mad_u64_u32 %0, s[94:95], %9, %19, %0\n"
      "v_mad_u64_u32 %0, s[92:93], %10, %20, %0\n"
      : "=&v"(acc)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]), "v"(b[8]), "v"(b[9])
      : "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95");
}
SV_HD void sv_col10_a(uint64_t& acc, const uint32_t a[10], const uint32_t b[10]) {
  asm(
      "v_mad_u64_u32 %0, s[94:95], %1, %11, %0\n"
      "v_mad_u64_u32 %0, s[92:93], %2, %12, %0\n"
      "v_mad_u64_u32 %0, s[90:91], %3, %13, %0\n"
      "v_mad_u64_u32 %0, s[88:89], %4, %14, %0\n"
      "v_mad_u64_u32 %0, s[94:95], %5, %15, %0\n"
      "v_mad_u64_u32 %0, s[92:93], %6, %16, %0\n"
      "v_mad_u64_u32 %0, s[90:91], %7, %17, %0\n"
      "v_mad_u64_u32 %0, s[88:89], %8, %18, %0\n"
      "v_mad_u64_u32 %0, s[94:95], %9, %19, %0\n"
      "v_mad_u64_u32 %0, s[92:93], %10, %20, %0\n"
      : "+v"(acc)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]), "v"(b[8]), "v"(b[9])
      : "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95");
}
SV_HD void sv_col6_z(uint64_t& acc, const uint32_t a[6], const uint32_t b[6]) {
  asm(
      "v_mad_u64_u32 %0, s[94:95], %1, %7, 0\n"
      "v_mad_u64_u32 %0, s[92:93], %2, %8, %0\n"
      "v_mad_u64_u32 %0, s[90:91], %3, %9, %0\n"
      "v_mad_u64_u32 %0, s[88:89], %4, %10, %0\n"
      "v_mad_u64_u32 %0, s[94:95], %5, %11, %0\n"
      "v_mad_u64_u32 %0, s[92:93], %6, %12, %0\n"
      : "=&v"(acc)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5])
      : "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95");
}
SV_HD void sv_col6_a(uint64_t& acc, const uint32_t a[6], const uint32_t b[6]) {
  asm(
      "v_mad_u64_u32 %0, s[94:95], %1, %7, %0\n"
      "v_mad_u64_u32 %0, s[92:93], %2, %8, %0\n"
      "v_mad_u64_u32 %0, s[90:91], %3, %9, %0\n"
      "v_mad_u64_u32 %0, s[88:89], %4, %10, %0\n"
      "v_mad_u64_u32 %0, s[94:95], %5, %11, %0\n"
      "v_mad_u64_u32 %0, s[92:93], %6, %12, %0\n"
      : "+v"(acc)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5])
      : "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95");
}
SV_HD void sv_col5_a(uint64_t& acc, const uint32_t a[5], const uint32_t b[5]) {
  asm(
      "v_mad_u64_u32 %0, s[94:95], %1, %6, %0\n"
      "v_mad_u64_u32 %0, s[92:93], %2, %7, %0\n"
      "v_mad_u64_u32 %0, s[90:91], %3, %8, %0\n"
      "v_mad_u64_u32 %0, s[88:89], %4, %9, %0\n"
      "v_mad_u64_u32 %0, s[94:95], %5, %10, %0\n"
      : "+v"(acc)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4])
      : "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95");
}
#endif

// 2x as v_add_u32 x, x: LLVM canonicalises x + x to a shift, and gfx950
// issues 32-bit shifts at half the rate of adds (tools/ubench_valu_rates:
// 4.5 vs 2.6 SIMD cycles per wave-instruction at 2 waves/SIMD).
SV_HD uint32_t sv_twice(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(x));
  return r;
#else
  return x << 1;
#endif
}

// limb 0 receives 19 * (carry out of limb 9), then one carry into limb 1
SV_HD void fe_carry_wrap(fe& out, uint64_t c9) {
  const uint64_t h0 = (uint64_t)out.v[0] + c9 * 19u;
  out.v[0] = (uint32_t)h0 & SV_M26;
  out.v[1] += (uint32_t)(h0 >> 26);
}
// opens column k: the carry of column k - 1 as the addend (k > 0)
SV_HD void sv_mad_open(uint64_t& acc, uint64_t c, uint32_t a, uint32_t b, int k, int n) {
  if (k == 0) {
    sv_mad_init_k(acc, a, b, n);
  } else {
    acc = c;
    sv_mad_k(acc, a, b, n);
  }
}
SV_HD void sv_col_close(fe& out, uint64_t& c, uint64_t acc, int k) {
  c = acc >> fe_width(k);
  out.v[k] = (uint32_t)acc & fe_mask(k);
}
// (out may alias f or g: the limbs are written to a local first)
template <bool DBL>
SV_HD void fe_mul_cm(fe& h, const fe& f, const fe& g) {
  fe out;
  uint32_t g19[10], fa[10], fb[10];
  SV_UNROLL for (int j = 0; j < 10; ++j) g19[j] = 19u * g.v[j];
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    fa[i] = DBL ? sv_twice(f.v[i]) : f.v[i];
    fb[i] = sv_twice(fa[i]);  // (odd i only; unused ones are dropped)
  }
  uint64_t acc = 0, c = 0;
  SV_UNROLL for (int k = 0; k < 10; ++k) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t A[10], B[10];
    SV_UNROLL for (int i = 0; i < 10; ++i) {
      const int j = (k - i + 10) % 10;
      A[i] = ((i & 1) && (j & 1)) ? fb[i] : fa[i];
      B[i] = (i + j >= 10) ? g19[j] : g.v[j];
    }
    if (k == 0) {
      sv_col10_z(acc, A, B);
    } else {
      acc = c;
      sv_col10_a(acc, A, B);
    }
#else
    SV_UNROLL for (int i = 0; i < 10; ++i) {
      const int j = (k - i + 10) % 10;
      const uint32_t a = ((i & 1) && (j & 1)) ? fb[i] : fa[i];
      const uint32_t b = (i + j >= 10) ? g19[j] : g.v[j];
      if (i == 0) sv_mad_open(acc, c, a, b, k, 10 * k + i);
      else sv_mad_k(acc, a, b, 10 * k + i);
    }
#endif
    sv_col_close(out, c, acc, k);
  }
  fe_carry_wrap(out, c);
  h = out;
}
template <bool DBL>
SV_HD void fe_sq_cm(fe& h, const fe& f) {
  fe out;
  uint64_t acc = 0, c = 0;
  int n = 0;
  uint32_t fm[4][10];  // f << 0..3, by additions
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    fm[0][i] = f.v[i];
    fm[1][i] = sv_twice(fm[0][i]);
    fm[2][i] = sv_twice(fm[1][i]);
    fm[3][i] = sv_twice(fm[2][i]);
  }
  SV_UNROLL for (int k = 0; k < 10; ++k) {
    bool first = true;
    uint32_t A[6], B[6];
    int t = 0;
    SV_UNROLL for (int i = 0; i < 10; ++i) {
      SV_UNROLL for (int j = i; j < 10; ++j) {
        if ((i + j) % 10 != k) continue;
        const int sh = (i != j ? 1 : 0) + (((i & 1) && (j & 1)) ? 1 : 0) + (DBL ? 1 : 0);
        const uint32_t a = fm[sh][i];
        const uint32_t b = (i + j >= 10) ? 19u * f.v[j] : f.v[j];
        A[t] = a;
        B[t] = b;
        ++t;
#if !defined(__HIP_DEVICE_COMPILE__)
        if (first) sv_mad_open(acc, c, a, b, k, n);
        else sv_mad_k(acc, a, b, n);
#endif
        first = false;
        ++n;
      }
    }
#if defined(__HIP_DEVICE_COMPILE__)
    // columns hold 6 terms (k even) or 5 (k odd)
    if (k == 0) {
      sv_col6_z(acc, A, B);
    } else {
      acc = c;
      if (k & 1) sv_col5_a(acc, A, B);
      else sv_col6_a(acc, A, B);
    }
#endif
    (void)first;
    (void)n;
    sv_col_close(out, c, acc, k);
  }
  fe_carry_wrap(out, c);
  h = out;
}

// Device: each product / square as one generated inline-asm
// statement (fe_asm_gen.h, tools/gen_fe_asm.py), same arithmetic as the
// column-major forms above.
// (-DSV_FE_ASM_ON=0: A/B builds only, the column-major forms on the device)
#if defined(__HIP_DEVICE_COMPILE__)
#ifndef SV_FE_ASM_ON
#define SV_FE_ASM_ON 1
#endif
#if SV_FE_ASM_ON
#include "fe_asm_gen.h"
#endif
#else
#undef SV_FE_ASM_ON
#define SV_FE_ASM_ON 0
#endif

// Measurement builds only (-DSV_MADCOUNT; tools/madcount.py): each field
// product adds its v_mad_u64_u32 count to a device counter once per wave (by
// the wave's first active lane), so the counter holds the multiply-adds the
// SIMDs issue.  Counts per generated statement (fe_asm_gen.h; checked by
// tests/test_host_arith.py): products 101 (100 + the x19 wrap of the top
// column), squarings 56.
#define SV_MADS_MUL 101
#define SV_MADS_SQ 56
#if defined(SV_MADCOUNT) && defined(__HIPCC__)
static __device__ unsigned long long sv_madcount[1];
#endif
#if defined(SV_MADCOUNT) && defined(__HIP_DEVICE_COMPILE__)
#define SV_MADS(k)                                                                    \
  do {                                                                                \
    if (__lane_id() == (uint32_t)__builtin_amdgcn_readfirstlane((int)__lane_id())) \
      atomicAdd(&sv_madcount[0], (unsigned long long)(k));                            \
  } while (0)
#else
#define SV_MADS(k) ((void)0)
#endif

SV_HD void fe_mul(fe& h, const fe& f, const fe& g) {
  SV_MADS(SV_MADS_MUL);
#if SV_FE_ASM_ON
  fe_mul_asm(h, f, g);
#else
  fe_mul_cm<false>(h, f, g);
#endif
  SV_FENCE();
}
SV_HD void fe_premul19(fe19& t, const fe& g) {
  SV_UNROLL for (int j = 1; j < 10; ++j) t.v[j - 1] = 19u * g.v[j];
}
// h = f g with t = fe_premul19(g) (same value and bounds as fe_mul)
SV_HD void fe_mul_g19(fe& h, const fe& f, const fe& g, const fe19& t) {
#if SV_FE_ASM_ON
  SV_MADS(SV_MADS_MUL);
  fe_mul_g19_asm(h, f, g, t);
#else
  (void)t;
  fe_mul(h, f, g);
  return;
#endif
  SV_FENCE();
}
// h = 2 f g (doubling folded into the operand; inputs must be <= R)
SV_HD void fe_mul2(fe& h, const fe& f, const fe& g) {
  SV_MADS(SV_MADS_MUL);
#if SV_FE_ASM_ON
  fe_mul2_asm(h, f, g);
#else
  fe_mul_cm<true>(h, f, g);
#endif
  SV_FENCE();
}
SV_HD void fe_sq(fe& h, const fe& f) {
  SV_MADS(SV_MADS_SQ);
#if SV_FE_ASM_ON
  fe_sq_asm(h, f);
#else
  fe_sq_cm<false>(h, f);
#endif
  SV_FENCE();
}
// h = 2 f^2 (input must be <= R)
SV_HD void fe_sq2(fe& h, const fe& f) {
  SV_MADS(SV_MADS_SQ);
#if SV_FE_ASM_ON
  fe_sq2_asm(h, f);
#else
  fe_sq_cm<true>(h, f);
#endif
  SV_FENCE();
}
// n successive squarings (rolled loop: keeps the code object small).  Two
// squarings per iteration (SV_SQN_PAIRS): a product's outputs are early-clobber
// registers distinct from its inputs, so a one-squaring loop copies its 10
// limbs back into the loop-carried registers every iteration (10 v_mov per
// squaring); with two the second squaring writes straight into them.
SV_HD void fe_sqn(fe& h, const fe& f, int n) {
  fe_sq(h, f);
  int i = 1;
  if ((n - 1) & 1) {  // (n is a constant at every call site: folded)
    fe_sq(h, h);
    ++i;
  }
  SV_NOUNROLL for (; i < n; i += 2) {
    fe t;
    fe_sq(t, h);
    fe_sq(h, t);
  }
}

// h = cond ? f : h  (per lane, branch-free)
SV_HD void fe_cmov(fe& h, const fe& f, bool cond) {
  SV_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = cond ? f.v[i] : h.v[i];
}

// 255-bit little-endian value (bit 255 ignored, value may be >= p) -> fe
SV_HD void fe_frombytes(fe& h, const uint32_t w[8]) {
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    const int o = fe_off(i), q = o >> 5, r = o & 31;
    uint32_t x = w[q] >> r;
    if (r + fe_width(i) > 32) x |= w[q + 1] << (32 - r);
    h.v[i] = x & fe_mask(i);
  }
}

// canonical little-endian encoding (value mod p, < p) as 8 words
SV_COLD void fe_tobytes(uint32_t out[8], const fe& f) {
  uint32_t h[10];
  SV_UNROLL for (int i = 0; i < 10; ++i) h[i] = f.v[i];
  // three sequential carry passes: limbs within width, value < 2^255
  SV_UNROLL for (int pass = 0; pass < 3; ++pass) {
    SV_UNROLL for (int i = 0; i < 9; ++i) {
      h[i + 1] += h[i] >> fe_width(i);
      h[i] &= fe_mask(i);
    }
    const uint32_t c = h[9] >> 25;
    h[9] &= SV_M25;
    h[0] += 19u * c;
  }
  // q = [value >= p] = [value + 19 >= 2^255]
  uint32_t q = (h[0] + 19u) >> 26;
  SV_UNROLL for (int i = 1; i < 10; ++i) q = (h[i] + q) >> fe_width(i);
  h[0] += 19u * q;
  SV_UNROLL for (int i = 0; i < 9; ++i) {
    h[i + 1] += h[i] >> fe_width(i);
    h[i] &= fe_mask(i);
  }
  h[9] &= SV_M25;  // drops 2^255 (i.e. subtracts p together with the +19)
  SV_UNROLL for (int w = 0; w < 8; ++w) out[w] = 0;
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    const int o = fe_off(i), q2 = o >> 5, r = o & 31;
    out[q2] |= h[i] << r;
    if (r + fe_width(i) > 32) out[q2 + 1] |= h[i] >> (32 - r);
  }
}

SV_HD bool fe_iszero(const fe& f) {
  uint32_t s[8];
  fe_tobytes(s, f);
  uint32_t acc = 0;
  SV_UNROLL for (int i = 0; i < 8; ++i) acc |= s[i];
  return acc == 0;
}
SV_HD uint32_t fe_isnegative(const fe& f) {
  uint32_t s[8];
  fe_tobytes(s, f);
  return s[0] & 1u;
}

// z^(2^250 - 1) and the two small powers the chains below need.
SV_COLD void fe_pow_2_250_1(fe& z250, fe& z11, const fe& z) {
  fe t0, t1, t2, z9, z_5_0, z_10_0, z_20_0, z_50_0, z_100_0;
  fe_sq(t0, z);              // z^2
  fe_sqn(t1, t0, 2);         // z^8
  fe_mul(z9, t1, z);         // z^9
  fe_mul(z11, z9, t0);       // z^11
  fe_sq(t2, z11);            // z^22
  fe_mul(z_5_0, t2, z9);     // z^31 = z^(2^5-1)
  fe_sqn(t0, z_5_0, 5);
  fe_mul(z_10_0, t0, z_5_0);   // 2^10-1
  fe_sqn(t0, z_10_0, 10);
  fe_mul(z_20_0, t0, z_10_0);  // 2^20-1
  fe_sqn(t0, z_20_0, 20);
  fe_mul(t0, t0, z_20_0);      // 2^40-1
  fe_sqn(t0, t0, 10);
  fe_mul(z_50_0, t0, z_10_0);  // 2^50-1
  fe_sqn(t0, z_50_0, 50);
  fe_mul(z_100_0, t0, z_50_0); // 2^100-1
  fe_sqn(t0, z_100_0, 100);
  fe_mul(t0, t0, z_100_0);     // 2^200-1
  fe_sqn(t0, t0, 50);
  fe_mul(z250, t0, z_50_0);    // 2^250-1
}

// z^((p-5)/8) = z^(2^252 - 3)
SV_COLD void fe_pow22523(fe& h, const fe& z) {
  fe z250, z11;
  fe_pow_2_250_1(z250, z11, z);
  fe_sqn(z250, z250, 2);
  fe_mul(h, z250, z);
}

// z^(p-2) = z^(2^255 - 21)
SV_COLD void fe_invert(fe& h, const fe& z) {
  fe z250, z11;
  fe_pow_2_250_1(z250, z11, z);
  fe_sqn(z250, z250, 5);
  fe_mul(h, z250, z11);
}

// curve constants (tools/gen_constants.py, radix 2^25.5)
SV_HD void fe_const_d(fe& h) {
  const uint32_t c[10] = {0x35978a3, 0x0d37284, 0x3156ebd, 0x06a0a0e, 0x001c029,
                          0x179e898, 0x3a03cbb, 0x1ce7198, 0x2e2b6ff, 0x1480db3};
  SV_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = c[i];
}
SV_HD void fe_const_2d(fe& h) {
  const uint32_t c[10] = {0x2b2f159, 0x1a6e509, 0x22add7a, 0x0d4141d, 0x0038052,
                          0x0f3d130, 0x3407977, 0x19ce331, 0x1c56dff, 0x0901b67};
  SV_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = c[i];
}
// 1/d (the main kernel's first window builds P = 2 Q from a cached entry:
// 2T = (2dT) / d)
SV_HD void fe_const_dinv(fe& h) {
  const uint32_t c[10] = {0x1c9f843, 0x03c9db3, 0x285c4bc, 0x0c213ca, 0x02d775a,
                          0x1b9cf66, 0x3108a66, 0x1c86562, 0x1214d5c, 0x10241fb};
  SV_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = c[i];
}
SV_HD void fe_const_sqrtm1(fe& h) {
  const uint32_t c[10] = {0x20ea0b0, 0x186c9d2, 0x08f189d, 0x035697f, 0x0bd0c60,
                          0x1fbd7a7, 0x2804c9e, 0x1e16569, 0x004fc1d, 0x0ae0c92};
  SV_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = c[i];
}

#endif  // SV_HOST_FE51
