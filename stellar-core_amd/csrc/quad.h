// Latency path: one signature per QUAD of lanes.
//
// The throughput kernels give each signature one lane, so a small batch (the
// SCP envelope flood of BASELINE config 4, 1k signatures) runs as a handful of
// waves whose latency is one lane's whole instruction stream.  Here the four
// lanes of a quad share a signature and split every point operation four ways:
//
//   doubling   the 4 squarings X^2, Y^2, 2Z^2, (X+Y)^2 -- one per lane -- then
//              the 3-4 products of the p1p1 -> p2/p3 conversion, one per lane
//   addition   the 4 products T*2dT', 2Z*Z', (Y+X)*(Y'+X'), (Y-X)*(Y'-X'),
//              then the 4 conversion products, one per lane
//
// with the results exchanged by DPP quad broadcasts (v_mov_b32 quad_perm), so
// every lane of the quad holds the whole point between operations.  The
// formulas, the limb bounds and the operation order are exactly those of
// ge_dbl / ge_add_preswapped / ge_p1p1_to_p3 (ge25519.h); only the assignment
// of field operations to lanes differs, so verdicts are the per-lane path's.
//
// Lane role r = lane & 3 selects the operand of its field operation.
#pragma once

#include "verify_core.h"

// value of lane K of this lane's quad (DPP quad_perm broadcast)
template <int K>
__device__ __forceinline__ uint32_t qd_from(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xf, 0xf, false);
#else
  return v;  // (host pass: never executed)
#endif
}
template <int K>
__device__ __forceinline__ void fe_from(fe& o, const fe& f) {
  SV_UNROLL for (int i = 0; i < 10; ++i) o.v[i] = qd_from<K>(f.v[i]);
}
// per-lane choice among four field elements by quad role
struct qd_role {
  bool r1, r2, r3;
};
__device__ __forceinline__ void fe_pick4(fe& o, const qd_role& q, const fe& a0, const fe& a1, const fe& a2,
                                         const fe& a3) {
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    const uint32_t x = q.r1 ? a1.v[i] : a0.v[i];
    const uint32_t y = q.r3 ? a3.v[i] : a2.v[i];
    o.v[i] = (q.r2 || q.r3) ? y : x;
  }
}

// The conversion products of a p1p1 point (X, Y, Z, T fields of Q): lane r
// computes product r of {X*T, Y*Z, Z*T, X*Y}; the quad then holds P = p3 (T
// valid only if wantT, i.e. every lane needs the 4th product).  Operand order
// as in ge_p1p1_to_p3_opt (p.X is always the f operand).
__device__ __forceinline__ void qd_p1p1_to_p3(ge_p3& P, const ge_p1p1& Q, const qd_role& q, bool wantT) {
  fe f, g, h;
  fe_pick4(f, q, Q.X, Q.Y, Q.Z, Q.X);
  fe_pick4(g, q, Q.T, Q.Z, Q.T, Q.Y);
  fe_mul(h, f, g);
  fe_from<0>(P.X, h);
  fe_from<1>(P.Y, h);
  fe_from<2>(P.Z, h);
  if (wantT) fe_from<3>(P.T, h);
}

// P = 2P (ge_dbl on the quad)
__device__ __forceinline__ void qd_dbl(ge_p3& P, const qd_role& q, bool wantT) {
  fe s, sq, XX, YY, ZZ2, AA, A;
  fe_add(A, P.X, P.Y);
  fe_pick4(s, q, P.X, P.Y, P.Z, A);
  fe_sq(sq, s);
  if (q.r2) fe_add(sq, sq, sq);  // 2 Z^2 (M2; the bound ge_dbl's fe_sub4 below accepts)
  fe_from<0>(XX, sq);
  fe_from<1>(YY, sq);
  fe_from<2>(ZZ2, sq);
  fe_from<3>(AA, sq);
  ge_p1p1 r;
  fe_add(r.Y, YY, XX);
  fe_sub(r.Z, YY, XX);
  fe_sub4(r.X, AA, r.Y);
  fe_sub4(r.T, ZZ2, r.Z);
#if SV_DBL_WEAK_EVEN
  fe_weak_even(r.T);  // (T: a conversion product's g operand only)
#else
  fe_weak(r.T);
#endif
  qd_p1p1_to_p3(P, r, q, wantT);
}

// P += entry (ge_add_preswapped on the quad).  `mine` is this lane's operand
// of the entry, already chosen by role and digit sign: role 0 the 2dT (2dxy)
// field, role 1 Z (1 for an affine entry), role 2 the (Y+X) side, role 3 the
// (Y-X) side of the pair after the sign swap.  neg swaps the final Z/T pair.
__device__ __forceinline__ void qd_add(ge_p3& P, const fe& mine, const qd_role& q, bool neg, bool wantT) {
  fe f, zz, ypx, ymx, h, TT, ZZ, PP, MM;
  fe_add(zz, P.Z, P.Z);
  fe_add(ypx, P.Y, P.X);
  fe_sub(ymx, P.Y, P.X);
  fe_pick4(f, q, P.T, zz, ypx, ymx);
  fe_mul(h, f, mine);
  fe_from<0>(TT, h);
  fe_from<1>(ZZ, h);
  fe_from<2>(PP, h);
  fe_from<3>(MM, h);
  ge_p1p1 r;
  fe zp, zm;
  fe_sub(r.X, PP, MM);
  fe_add(r.Y, PP, MM);
  fe_add(zp, ZZ, TT);
  fe_sub(zm, ZZ, TT);
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    r.Z.v[i] = neg ? zm.v[i] : zp.v[i];
    r.T.v[i] = neg ? zp.v[i] : zm.v[i];
  }
  qd_p1p1_to_p3(P, r, q, wantT);
}
