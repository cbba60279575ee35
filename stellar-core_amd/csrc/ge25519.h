// Twisted Edwards (a = -1) point arithmetic on edwards25519 for one lane.
//
// Coordinates (x = X/Z, y = Y/Z unless noted):
//   ge_p2      (X:Y:Z)
//   ge_p3      (X:Y:Z:T), xy = T/Z
//   ge_p1p1    "completed": x = X/Z, y = Y/T (output of dbl/add; 3-4 muls
//              convert it to p2 or p3)
//   ge_cached  (Y+X, Y-X, Z, 2dT)  -- per-signature table entries of -A
//   ge_precomp (y+x, y-x, 2dxy)    -- affine base-point table entries (LDS)
//
// The addition law used is the complete extended-coordinate law for a = -1
// (d is a non-square, -1 a square mod p), so results are the exact group
// elements for every input on the curve, including small- and mixed-order
// points: encode([h](-A) + [S]B) does not depend on how the sum is scheduled.
// That is what lets this engine use a wave-uniform fixed-window schedule and
// still be bit-exact with libsodium's sliding-window
// ge25519_double_scalarmult_vartime (reference call site:
// stellar-core src/crypto/SecretKey.cpp:461-463).
//
// Limb-bound bookkeeping (see fe25519.h): every fe_mul/fe_sq input is <= M3,
// except the f operand of the p1p1 conversions after a doubling (<= M5).
#pragma once

#include "fe25519.h"


// p1p1 -> p3: Y is the g operand of both Y3 = Z Y and T3 = X Y, so its
// 19-multiples are computed once as well (9 v_mul_lo_u32 per conversion)

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z, T2d; };
struct ge_precomp { fe ypx, ymx, xy2d; };

SV_HD void ge_p2_identity(ge_p2& p) {
  fe_0(p.X);
  fe_1(p.Y);
  fe_1(p.Z);
}

// r = 2p.  Inputs R.  Outputs: X M5, Y M2, Z M3, T R+.
// X is left at M5 (one carry pass saved per doubling): the conversions only
// ever use p1p1 X as the f operand of fe_mul, which tolerates M5 (fe25519.h
// header; fuzzed at the bound in tests/test_host_arith.py), never as the
// 19-premultiplied g operand, which needs <= M3.
SV_HD void ge_dbl(ge_p1p1& r, const fe& X, const fe& Y, const fe& Z) {
  fe XX, YY, ZZ2, A, AA;
  fe_add(A, X, Y);
  fe_sq(AA, A);
  fe_sq(XX, X);
  fe_sq(YY, Y);
  fe_sq2(ZZ2, Z);
  fe_add(r.Y, YY, XX);    // y^2 + x^2            M2
  fe_sub(r.Z, YY, XX);    // y^2 - x^2            M3
  fe_sub4(r.X, AA, r.Y);  // 2xy = (x+y)^2 - ..  M5
  fe_sub4(r.T, ZZ2, r.Z); // 2z^2 - (y^2 - x^2)  M5
  fe_weak_even(r.T);      // T is only ever a conversion product's g operand
}

// p1p1 -> p3 (wantT) or -> p2 (T left stale).  r must not alias p.  Bounds:
// X (<= M5) and Z (<= M3) are only ever f operands; Y (<= M2) and T are the
// g operands whose 19-multiples are shared: Y by Z Y and X Y, T by X T and
// Z T.
SV_HD void ge_p1p1_convert(ge_p3& r, const ge_p1p1& p, bool wantT) {
  {
    fe19 y19;
    fe_premul19(y19, p.Y);
    if (wantT) fe_mul_g19(r.T, p.X, p.Y, y19);
    fe_mul_g19(r.Y, p.Z, p.Y, y19);
  }
  fe19 t19;
  fe_premul19(t19, p.T);
  fe_mul_g19(r.X, p.X, p.T, t19);
  fe_mul_g19(r.Z, p.Z, p.T, t19);
}

SV_HD void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
  ge_p3 t;
  ge_p1p1_convert(t, p, false);
  r.X = t.X;
  r.Y = t.Y;
  r.Z = t.Z;
}

SV_HD void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) { ge_p1p1_convert(r, p, true); }

// p1p1 -> p3 when the next step is an addition (wantT), else -> p2 (T left
// stale).  wantT is wave-uniform, so this is a scalar branch.
SV_HD void ge_p1p1_to_p3_opt(ge_p3& r, const ge_p1p1& p, bool wantT) { ge_p1p1_convert(r, p, wantT); }

// r = p + q where the caller has already swapped q's (Y+X, Y-X) pair for a
// negative digit (by choosing load addresses); neg then only swaps the final
// Z/T pair, i.e. negates 2dT.  zone: q is affine (Z = 1, base-point table), so
// 2 Z1 Z2 = 2 Z1 is an add + carry pass instead of a multiply (wave-uniform).
// Inputs: p R; qa, qb <= M3; qZ, qT2d <= R.  Outputs: X M3, Y M2, Z/T M2 or M3.
SV_HD void ge_add_preswapped(ge_p1p1& r, const ge_p3& p, const fe& qa, const fe& qb, const fe& qZ,
                             const fe& qT2d, bool neg, bool zone) {
  fe t0, t1, PP, MM, TT, ZZ2, zp, zm;
  fe_mul(TT, p.T, qT2d);
  if (zone) {
    fe_add(ZZ2, p.Z, p.Z);
    fe_weak(ZZ2);           // R+
  } else {
    fe_mul2(ZZ2, p.Z, qZ);  // 2 Z1 Z2, R
  }
  fe_add(t0, p.Y, p.X);   // M2
  fe_sub(t1, p.Y, p.X);   // M3
  fe_mul(PP, t0, qa);
  fe_mul(MM, t1, qb);
  fe_sub(r.X, PP, MM);    // M3
  fe_add(r.Y, PP, MM);    // M2
  fe_add(zp, ZZ2, TT);    // M2
  fe_sub(zm, ZZ2, TT);    // M3
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    r.Z.v[i] = neg ? zm.v[i] : zp.v[i];
    r.T.v[i] = neg ? zp.v[i] : zm.v[i];
  }
}

SV_HD void ge_p3_to_cached(ge_cached& c, const ge_p3& p) {
  fe d2;
  fe_const_2d(d2);
  fe_add(c.YpX, p.Y, p.X);  // M2
  fe_sub(c.YmX, p.Y, p.X);  // M3
  c.Z = p.Z;
  fe_mul(c.T2d, p.T, d2);
}

SV_HD void ge_cached_identity(ge_cached& c) {
  fe_1(c.YpX);
  fe_1(c.YmX);
  fe_1(c.Z);
  fe_0(c.T2d);
}

// Decompress a 32-byte encoding (bit 255 = sign of x) into -P (negate = true)
// or P (negate = false).  Restates libsodium 1.0.18
// ge25519_frombytes_negate_vartime: y is read mod 2^255 without reduction,
// x = u v^3 (u v^7)^((p-5)/8) with u = y^2 - 1, v = d y^2 + 1; if v x^2 = -u
// x is multiplied by sqrt(-1); if neither v x^2 = u nor = -u the point is
// rejected.  The sign test compares the parity of x (after the root choice)
// with bit 255, exactly as libsodium does (so x = 0 with bit 255 set passes
// here; such encodings are on the small-order blacklist anyway).
// Returns true on success.
// Tail of the decompression once x = u v^3 (u v^7)^((p-5)/8) is known.
SV_HD bool ge_frombytes_finish(ge_p3& h, const fe& u, const fe& v, const uint32_t w[8], bool negate) {
  fe vxx, chk, chk2, xs, sq;
  fe_sq(vxx, h.X);
  fe_mul(vxx, vxx, v);
  fe_sub(chk, vxx, u);
  fe_add(chk2, vxx, u);
  const bool m_ok = fe_iszero(chk);
  const bool p_ok = fe_iszero(chk2);
  fe_const_sqrtm1(sq);
  fe_mul(xs, h.X, sq);
  fe_cmov(h.X, xs, !m_ok);
  const uint32_t sign = w[7] >> 31;
  fe nx;
  fe_neg(nx, h.X);
  const bool flip = negate ? (fe_isnegative(h.X) == sign) : (fe_isnegative(h.X) != sign);
  fe_cmov(h.X, nx, flip);
  fe_weak(h.X);
  fe_mul(h.T, h.X, h.Y);
  return m_ok || p_ok;
}

SV_COLD bool ge_frombytes(ge_p3& h, const uint32_t w[8], bool negate) {
  fe u, v, v3, one, d;
  fe_1(one);
  fe_const_d(d);
  fe_frombytes(h.Y, w);
  fe_1(h.Z);
  fe_sq(u, h.Y);
  fe_mul(v, u, d);
  fe_sub(u, u, one);  // y^2 - 1
  fe_weak(u);
  fe_add(v, v, one);  // d y^2 + 1
  fe_weak(v);
  fe_sq(v3, v);
  fe_mul(v3, v3, v);  // v^3
  fe_sq(h.X, v3);
  fe_mul(h.X, h.X, v);
  fe_mul(h.X, h.X, u);  // u v^7
  fe_pow22523(h.X, h.X);
  fe_mul(h.X, h.X, v3);
  fe_mul(h.X, h.X, u);  // u v^3 (u v^7)^((p-5)/8)
  return ge_frombytes_finish(h, u, v, w, negate);
}

// canonical encoding of a projective point given 1/Z (8 little-endian words)
SV_COLD void ge_p2_tobytes_zinv(uint32_t out[8], const fe& X, const fe& Y, const fe& zi) {
  fe x, y;
  fe_mul(x, X, zi);
  fe_mul(y, Y, zi);
  fe_tobytes(out, y);
  out[7] ^= fe_isnegative(x) << 31;
}

// canonical encoding of a projective point (8 little-endian words)
SV_COLD void ge_p2_tobytes(uint32_t out[8], const fe& X, const fe& Y, const fe& Z) {
  fe zi;
  fe_invert(zi, Z);
  ge_p2_tobytes_zinv(out, X, Y, zi);
}
