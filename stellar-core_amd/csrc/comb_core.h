// Per-lane pieces of the warm-key latency path (comb.h) shared by the device
// kernels (sv_comb.hip) and the host test build (tests/native/host_core.cpp):
// the entry format and the base-point table entries.
#pragma once

#include "comb.h"
#include "verify_core.h"

// one coordinate of an entry (10 carried limbs + 2 pad dwords)
SV_HD void sv_ce_put_coord(uint32_t* ent, int k, const fe& f) {
  fe w = f;
  fe_weak(w);
  SV_UNROLL for (int i = 0; i < 10; ++i) ent[12 * k + i] = w.v[i];
  ent[12 * k + 10] = 0;
  ent[12 * k + 11] = 0;
}
SV_HD void sv_ce_put(uint32_t* ent, const ge_cached& c) {
  sv_ce_put_coord(ent, 0, c.YpX);
  sv_ce_put_coord(ent, 1, c.YmX);
  sv_ce_put_coord(ent, 2, c.Z);
  sv_ce_put_coord(ent, 3, c.T2d);
}
// the entry with a digit's sign applied: (Y+X, Y-X) swapped for neg (the
// caller negates 2dT through ge_add_preswapped's neg)
SV_HD void sv_ce_get(ge_cached& c, const uint32_t* ent, bool neg) {
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    c.YpX.v[i] = ent[(neg ? 12 : 0) + i];
    c.YmX.v[i] = ent[(neg ? 0 : 12) + i];
    c.Z.v[i] = ent[24 + i];
    c.T2d.v[i] = ent[36 + i];
  }
}

// Entry (pos, e) of the base-point tables: e * 256^pos * B in cached form.
SV_COLD void sv_comb_bentry(uint32_t* ent, int pos, int e) {
  const uint32_t benc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                            0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  ge_p3 B, acc;
  ge_frombytes(B, benc, false);
  ge_p1p1 Q;
  for (int i = 0; i < 8 * pos; ++i) {
    ge_dbl(Q, B.X, B.Y, B.Z);
    ge_p1p1_to_p3(B, Q);
  }
  ge_cached bc;
  ge_p3_to_cached(bc, B);
  fe_0(acc.X); fe_1(acc.Y); fe_1(acc.Z); fe_0(acc.T);
  for (int bit = 7; bit >= 0; --bit) {
    ge_dbl(Q, acc.X, acc.Y, acc.Z);
    ge_p1p1_to_p3(acc, Q);
    if ((e >> bit) & 1) {
      ge_add_preswapped(Q, acc, bc.YpX, bc.YmX, bc.Z, bc.T2d, false, false);
      ge_p1p1_to_p3(acc, Q);
    }
  }
  ge_cached ce;
  ge_p3_to_cached(ce, acc);
  sv_ce_put(ent, ce);
}
