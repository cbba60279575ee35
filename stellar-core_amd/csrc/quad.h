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

// value of lane K of this lane's quad (DPP quad_perm broadcast; bound_ctrl
// set, which quad_perm never exercises, lets LLVM fold the move into a VOP2
// consumer such as the X + Y add of qo_dbl)
template <int K>
__device__ __forceinline__ uint32_t qd_from(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xf, 0xf, true);
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
  fe_weak_even(r.T);  // (T: a conversion product's g operand only)
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

// ---------------------------------------------------------------------------
// "Own form" (the latency kernels' scalar-multiplication loop): lane r of the
// quad holds ONLY coordinate r of P (0 X, 1 Y, 2 Z, 3 T) -- the product it
// computed last -- instead of the whole point.  Each step moves just the
// values its lanes need (DPP quad_perm with per-lane sources) instead of
// broadcasting every result to every lane and picking from four, and the
// conversion products keep a fixed lane map (X, Y, Z, T on lanes 0..3), so
// no step ever rebuilds the whole point until the end (qo_expand).  Same
// field operations, operand order and bounds as ge_dbl / ge_add_preswapped /
// ge_p1p1_to_p3 (ge25519.h), hence the same verdicts.

// value of lane P<r> of this lane's quad, for lane r
template <int P0, int P1, int P2, int P3>
__device__ __forceinline__ void fe_perm(fe& o, const fe& f) {
  SV_UNROLL for (int i = 0; i < 10; ++i) {
#if defined(__HIP_DEVICE_COMPILE__)
    o.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)f.v[i], P0 | (P1 << 2) | (P2 << 4) | (P3 << 6), 0xf,
                                                   0xf, true);
#else
    o.v[i] = f.v[i];
#endif
  }
}

// P = identity: (0 : 1 : 1 : 0)
__device__ __forceinline__ void qo_identity(fe& h, const qd_role& q) {
  if (q.r1 || q.r2) fe_1(h);
  else fe_0(h);
}

// the whole point on every lane of the quad
__device__ __forceinline__ void qo_expand(ge_p3& P, const fe& h) {
  fe_from<0>(P.X, h);
  fe_from<1>(P.Y, h);
  fe_from<2>(P.Z, h);
  fe_from<3>(P.T, h);
}

// P = 2P: lanes 0, 1, 2 square their own coordinate (lane 2 doubles it),
// lane 3 squares X + Y; the conversion products X'T', Y'Z', Z'T', X'Y' land
// on lanes 0..3 again.
__device__ __forceinline__ void qo_dbl(fe& h, const qd_role& q) {
  fe x, y, s, sq;
  fe_from<0>(x, h);
  fe_from<1>(y, h);
  fe_add(s, x, y);  // X + Y (M2)
  SV_UNROLL for (int i = 0; i < 10; ++i) s.v[i] = q.r3 ? s.v[i] : h.v[i];
  fe_sq(sq, s);
  if (q.r2) fe_add(sq, sq, sq);  // 2 Z^2 (M2; the bound ge_dbl's fe_sub4 below accepts)
  fe XX, YY, u, w;
  fe_from<0>(XX, sq);
  fe_from<1>(YY, sq);
  fe_perm<3, 1, 2, 3>(u, sq);  // lanes 0, 3: (X+Y)^2
  fe_perm<2, 1, 2, 3>(w, sq);  // lanes 0, 2: 2 Z^2
  fe Yp, Zp, Xp, Tp;
  fe_add(Yp, YY, XX);   // y^2 + x^2            M2
  fe_sub(Zp, YY, XX);   // y^2 - x^2            M3
  fe_sub4(Xp, u, Yp);   // 2xy (lanes 0, 3)     M5
  fe_sub4(Tp, w, Zp);   // (lanes 0, 2)         M5
  fe_weak_even(Tp);  // (T: a conversion product's g operand only)
  // lane 0 X'T', 1 Y'Z', 2 Z'T', 3 X'Y' (p1p1 X is always the f operand)
  fe f, g;
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    f.v[i] = q.r1 ? Yp.v[i] : (q.r2 ? Zp.v[i] : Xp.v[i]);
    g.v[i] = q.r3 ? Yp.v[i] : (q.r1 ? Zp.v[i] : Tp.v[i]);
  }
  fe_mul(h, f, g);
}

// this lane's operand of cached entry `ent` (LDS; YpX, YmX, Z, T2d x 10
// dwords) in own-form roles: lane 0 the (Y+X) side, lane 1 the (Y-X) side
// (swapped when neg), lane 2 Z, lane 3 2dT
__device__ __forceinline__ void qo_load_cached(fe& o, const uint32_t* ent, uint32_t role, bool neg) {
  const uint32_t comp = role >= 2 ? role : ((role == 0) != neg ? 0u : 1u);
  const uint32_t* src = ent + 10 * comp;
  SV_UNROLL for (int k = 0; k < 10; ++k) o.v[k] = src[k];
}
// the same for an affine base-point entry (global; y+x, y-x, 2dxy as 3 quads
// each): lane 2 the constant 1 (Z)
__device__ __forceinline__ void qo_load_affine(fe& o, const sv_u4* ent, uint32_t role, bool neg) {
  const uint32_t comp = role == 3 ? 2u : role == 2 ? 0u : ((role == 0) != neg ? 0u : 1u);
  const sv_u4* src = ent + 3 * comp;
  const sv_u4 a = src[0], b = src[1], c = src[2];
  o.v[0] = a.x; o.v[1] = a.y; o.v[2] = a.z; o.v[3] = a.w;
  o.v[4] = b.x; o.v[5] = b.y; o.v[6] = b.z; o.v[7] = b.w;
  o.v[8] = c.x; o.v[9] = c.y;
  if (role == 2) fe_1(o);
}

// P += entry: lane 0 (Y+X)(Y'+X'), 1 (Y-X)(Y'-X'), 2 2Z Z', 3 T 2dT', then
// the conversion products as in qo_dbl.  neg swaps the final Z/T pair.
__device__ __forceinline__ void qo_add(fe& h, const fe& mine, const qd_role& q, bool neg) {
  fe r, a, b, f, pr;
  fe_perm<1, 0, 2, 3>(r, h);  // lane 0 <- Y, 1 <- X, 2 and 3 their own
  fe_add(a, h, r);            // lane 0 X + Y, lane 2 2Z   M2
  fe_sub(b, h, r);            // lane 1 Y - X              M3
  SV_UNROLL for (int i = 0; i < 10; ++i) f.v[i] = q.r1 ? b.v[i] : (q.r3 ? h.v[i] : a.v[i]);
  fe_mul(pr, f, mine);
  fe PP, MM, ZZ, TT;
  fe_from<0>(PP, pr);
  fe_from<1>(MM, pr);
  fe_from<2>(ZZ, pr);
  fe_from<3>(TT, pr);
  fe X1, Y1, zp, zm;
  fe_sub(X1, PP, MM);  // M3
  fe_add(Y1, PP, MM);  // M2
  fe_add(zp, ZZ, TT);  // M2
  fe_sub(zm, ZZ, TT);  // M3
  fe g;
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    const uint32_t z1 = neg ? zm.v[i] : zp.v[i], t1 = neg ? zp.v[i] : zm.v[i];
    f.v[i] = q.r1 ? Y1.v[i] : (q.r2 ? z1 : X1.v[i]);
    g.v[i] = q.r3 ? Y1.v[i] : (q.r1 ? z1 : t1);
  }
  fe_mul(h, f, g);
}
