// gfx950 kernels of the warm-key latency path (layout: comb.h).
//
// Per signature, libsodium 1.0.18 crypto_sign_verify_detached (the call
// stellar-core makes at /root/reference/src/crypto/SecretKey.cpp:461-463)
// accepts iff
//   (1) S < L, (2) R not small-order, (3)-(5) A canonical, not small-order and
//   decodable, and (8) encode([S]B - [h]A) == R, h = SHA-512(R||A||M) mod L.
// This path evaluates exactly that:
//   * (3)-(5) are a property of the key: the key-table build records them as
//     the slot status (SV_KEY_BAD: every signature under the key rejects);
//   * (8): encode() is injective and always emits a canonical y, so
//     encode(Q) == R  iff  R is canonical, decodes to a point R_pt with
//     encode(R_pt) == R, and Q == R_pt (x = 0 encodings with the sign bit set
//     have no such point; they are also on (2)'s blacklist).  Q == R_pt is
//     tested projectively, X == x_R Z and Y == y_R Z, so no inversion;
//   * Q = [S]B + [h](-A) is a sum of 96 table entries (comb.h).  The complete
//     addition law makes the sum exact for every A, including mixed-order keys,
//     in any order.
//
// Kernel geometry (sv_comb_kernel): 4 waves per workgroup, one per SIMD.
//   wave 0  decodes R of the workgroup's signatures (one lane each: the
//           square-root exponentiation, 57 us at 1k) and hands (x_R, y_R,
//           ok) over in LDS;
//   waves 1-3 ("chain waves") each verify SPW signatures: every lane hashes
//           its signature (SHA-512 over the message's LDS window, mod L,
//           signed digits), then the 16/SPW lane quads of a signature each
//           load their share of the 96 entries (B, then -A) and add them with
//           every point addition split over the quad's four lanes (own form,
//           quad.h), and the quads' partial sums meet in a tree (DPP /
//           ds_bpermute).  After one barrier the root quad tests Q == R_pt.
//           (62 us at 1k: the longer half, since the lane's image is read
//           from host memory; profiles/r04/lane_msg_lds/.)
// A 1000-signature batch with SPW = 2 is 167 workgroups: at most one per CU,
// every wave alone on its SIMD.
#include <hip/hip_runtime.h>

#include "comb_core.h"
#include "quad.h"
#include "sv_kparams.h"

struct sv_comb_params {
  sv_kparams k;           // inputs and verdicts (ws / btab / bitmap unused)
  const uint32_t* kslot;  // n: key-cache slot of each signature's key
  const uint32_t* ktab;   // slots x SV_KEY_SLOT_DW: tables of -A
  const uint32_t* kstat;  // slots: SV_KEY_OK / SV_KEY_BAD
  const uint32_t* ctab;   // SV_CB_DW: tables of B
};

// this lane's coordinate of cached entry `ent` for a digit of sign `neg`
// (own-form operand roles, quad.h qo_load_cached): lane 0 the (Y+X) side,
// lane 1 the (Y-X) side -- swapped when neg --, lane 2 Z, lane 3 2dT
__device__ __forceinline__ void ce_load(fe& o, const uint32_t* ent, uint32_t role, bool neg) {
  const uint32_t comp = role >= 2 ? role : ((role == 0) != neg ? 0u : 1u);
  const sv_u4* s = (const sv_u4*)(ent + 12 * comp);
  const sv_u4 a = s[0], b = s[1], c = s[2];
  o.v[0] = a.x; o.v[1] = a.y; o.v[2] = a.z; o.v[3] = a.w;
  o.v[4] = b.x; o.v[5] = b.y; o.v[6] = b.z; o.v[7] = b.w;
  o.v[8] = c.x; o.v[9] = c.y;
}
// writes this lane's coordinate (role) of an entry
__device__ __forceinline__ void ce_store(uint32_t* ent, uint32_t role, const fe& f) {
  sv_u4* d = (sv_u4*)(ent + 12 * role);
  d[0] = sv_u4{f.v[0], f.v[1], f.v[2], f.v[3]};
  d[1] = sv_u4{f.v[4], f.v[5], f.v[6], f.v[7]};
  d[2] = sv_u4{f.v[8], f.v[9], 0u, 0u};
}

// own form (quad.h) of the point of a cached entry, scaled by 2:
// (2X, 2Y, 2Z, 2T) = ((Y+X)-(Y-X), (Y+X)+(Y-X), 2Z, (2dT)/d), negated (X, T)
// for a negative digit (whose (Y+X, Y-X) pair ce_load already swapped)
__device__ __forceinline__ void qo_from_cached(fe& h, const fe& mine, const qd_role& q, bool neg) {
  fe o, d, s, z, t, nt, dinv;
  fe_perm<1, 0, 2, 3>(o, mine);  // lane 0 <- lane 1's side, lane 1 <- lane 0's
  fe_sub(d, mine, o);            // lane 0: a - b   (b <= R+)
  fe_add(s, o, mine);            // lane 1: a + b
  fe_add(z, mine, mine);         // lane 2: 2Z
  fe_const_dinv(dinv);
  fe_mul(t, mine, dinv);         // lane 3: 2T
  fe_neg(nt, t);
  SV_UNROLL for (int i = 0; i < 10; ++i) {
    const uint32_t t3 = neg ? nt.v[i] : t.v[i];
    h.v[i] = q.r1 ? s.v[i] : (q.r2 ? z.v[i] : (q.r3 ? t3 : d.v[i]));
  }
  fe_weak(h);  // R+ (own-form coordinates enter qo_add / qo_dbl at <= R)
}

// own form -> this lane's cached operand of the same point (lane 0 Y+X,
// 1 Y-X, 2 Z, 3 2dT: the qo_add operand roles); c is the own form (<= R)
__device__ __forceinline__ void qo_to_cached(fe& mine, const fe& c, const qd_role& q) {
  fe o, s, d, t, d2;
  fe_perm<1, 0, 2, 3>(o, c);  // lane 0: Y (lane 1's), lane 1: X (lane 0's)
  fe_add(s, o, c);            // lane 0: Y + X      M2
  fe_sub(d, c, o);            // lane 1: Y - X      M3
  fe_const_2d(d2);
  fe_mul(t, c, d2);           // lane 3: 2d T       R
  SV_UNROLL for (int i = 0; i < 10; ++i) mine.v[i] = q.r1 ? d.v[i] : (q.r2 ? c.v[i] : (q.r3 ? t.v[i] : s.v[i]));
}

// value of lane + D (D = 4, 8: DPP row shift inside a row of 16; 16, 32:
// ds_bpermute).  Lanes whose source is out of range read garbage, which only
// quads that are not tree receivers ever consume.
template <int D>
__device__ __forceinline__ uint32_t sv_lane_down(uint32_t v) {
  if (D == 4) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x104, 0xf, 0xf, false);
  if (D == 8) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x108, 0xf, 0xf, false);
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((__lane_id() + D) & 63u) << 2), (int)v);
}
template <int D>
__device__ __forceinline__ void fe_lane_down(fe& o, const fe& f) {
  SV_UNROLL for (int i = 0; i < 10; ++i) o.v[i] = sv_lane_down<D>(f.v[i]);
}

// word i of w[8] for a per-lane index (select chain, no scratch)
__device__ __forceinline__ uint32_t sv_pick8(const uint32_t w[8], uint32_t i) {
  uint32_t r = w[0];
  SV_UNROLL for (int k = 1; k < 8; ++k) r = i == (uint32_t)k ? w[k] : r;
  return r;
}
// signed 4-bit digit k (0..7) / signed 8-bit digit k (0..3) of a packed word
__device__ __forceinline__ int32_t sv_snib(uint32_t w, uint32_t k) { return (int32_t)(w << (28u - 4u * k)) >> 28; }
__device__ __forceinline__ int32_t sv_sbyte(uint32_t w, uint32_t k) { return (int32_t)(w << (24u - 8u * k)) >> 24; }

// One signature per SPW-th of a chain wave; see the file header.
template <int MODE, int SPW>
__global__ __launch_bounds__(256, 1) void sv_comb_kernel(sv_comb_params c) {
  // Latency class: these waves win the SIMD's issue arbitration over a
  // throughput kernel's waves sharing the CU (shared mode, sv_kernels.hip).
  __builtin_amdgcn_s_setprio(3);
  constexpr int NS = SV_COMB_CHAIN_WAVES * SPW;  // signatures per workgroup
  constexpr int LPS = 64 / SPW;                  // lanes per signature
  constexpr int QPS = LPS / 4;                   // quads per signature
  constexpr int PA = SV_KA_POS / QPS;            // -A positions per quad
  constexpr int PB = SV_CB_POS / QPS;            // B positions per quad
  static_assert(PB >= 2 && PA % 4 == 0, "geometry");
  const sv_kparams& p = c.k;
  __shared__ uint32_t s_r[NS][20];  // x_R, y_R (10 limbs each)
  __shared__ uint32_t s_rok[NS];
  __shared__ sv_u4 s_msg[SV_COMB_CHAIN_WAVES][SPW * (SV_MSG_CAP / 16)];  // message windows
  const uint32_t lane = __lane_id();
  const uint64_t gbase = (uint64_t)blockIdx.x * NS;
  // wave-uniform, visibly so (a scalar branch around the barrier)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave == 0) {
    // decode wave: R_pt with encode(R_pt) == R, or ok = false
    if (lane < (uint32_t)NS) {
      const uint64_t g = gbase + lane;
      const uint64_t gi = g < p.n ? g : p.n - 1;
      uint32_t R[8];
      sv_unpack2(R, p.sig + 4 * gi);
      bool ok = !sv_small_order(R) && sv_point_canonical(R);
      ge_p3 Rp;
      ok = ge_frombytes(Rp, R, false) && ok;
      SV_UNROLL for (int i = 0; i < 10; ++i) {
        s_r[lane][i] = Rp.X.v[i];
        s_r[lane][10 + i] = Rp.Y.v[i];
      }
      s_rok[lane] = ok ? 1u : 0u;
    }
    __syncthreads();
    return;
  }
  const uint32_t sw = lane / LPS;            // signature within the wave
  const uint32_t quad = (lane % LPS) >> 2;   // quad within the signature
  const uint32_t role = lane & 3u;
  const qd_role q{role == 1, role == 2, role == 3};
  const uint32_t ls = (wave - 1) * SPW + sw;  // signature within the workgroup
  const uint64_t g = gbase + ls;
  const bool active = g < p.n;
  const uint64_t gi = active ? g : p.n - 1;  // idle tail signatures redo the last item

  // Hash first (the message through its LDS window, sv_load_and_hash_lds),
  // then the quad's entries in two groups, B then -A: fewer entries live at
  // once than loading all of them together (SPW = 4: 256 -> 229 VGPRs, 4096
  // warm 0.216 -> 0.199 ms in A/B, profiles/r04/lane_msg_lds/).
  uint32_t A[8], S[8], hram[16];
  sv_load_and_hash_lds<MODE, LPS>(p, gi, lane % LPS, s_msg[wave - 1] + sw * (SV_MSG_CAP / 16), A, S, hram);
  const uint32_t ks = c.kslot[gi];
  const uint32_t kst = c.kstat[ks];
  const bool s_ok = sc_is_canonical(S);
  // a lane with S >= L is rejected by (1); clearing bits 253..255 keeps its
  // radix-256 digits inside the table (top digit <= 32); every S < 2^253,
  // so every S < L, is left unchanged
  S[7] &= 0x1fffffffu;
  uint32_t dB[8];
  sc_digits_r256(dB, S);
  // this quad's entries: B positions quad*PB + t, -A positions quad*PA + t
  fe entB[PB];
  bool negB[PB];
  {
    constexpr int WB = PB >= 4 ? PB / 4 : 1;
    uint32_t wb[WB];
    SV_UNROLL for (int u = 0; u < WB; ++u) wb[u] = sv_pick8(dB, ((quad * PB) >> 2) + u);
    SV_UNROLL for (int t = 0; t < PB; ++t) {
      const uint32_t k = PB >= 4 ? (uint32_t)(t & 3) : ((quad * PB) & 3) + t;
      const int32_t e = sv_sbyte(wb[PB >= 4 ? t >> 2 : 0], k);
      negB[t] = e < 0;
      const uint32_t pos = quad * PB + t;
      ce_load(entB[t], c.ctab + (pos * SV_CB_ENT + (uint32_t)(e < 0 ? -e : e)) * SV_CE_DW, role, e < 0);
    }
  }
  // the quad's partial sum, B half
  fe P;
  qo_from_cached(P, entB[0], q, negB[0]);
  SV_UNROLL for (int t = 1; t < PB; ++t) qo_add(P, entB[t], q, negB[t]);
  uint32_t h[8], dA[8];
  sc_reduce512(h, hram);
  sc_digits_r16(dA, h);
  // -A half
  const uint32_t* ka = c.ktab + (size_t)ks * SV_KEY_SLOT_DW;
  {
    constexpr int WA = PA >= 8 ? PA / 8 : 1;
    uint32_t wa[WA];
    SV_UNROLL for (int u = 0; u < WA; ++u) wa[u] = sv_pick8(dA, ((quad * PA) >> 3) + u);
    fe ent[PA];
    bool eneg[PA];
    SV_UNROLL for (int t = 0; t < PA; ++t) {
      const uint32_t k = PA >= 8 ? (uint32_t)(t & 7) : ((quad * PA) & 7) + t;
      const int32_t d = sv_snib(wa[PA >= 8 ? t >> 3 : 0], k);
      eneg[t] = d < 0;
      const uint32_t pos = quad * PA + t;
      ce_load(ent[t], ka + (pos * SV_KA_ENT + (uint32_t)(d < 0 ? -d : d)) * SV_CE_DW, role, d < 0);
    }
    SV_UNROLL for (int t = 0; t < PA; ++t) qo_add(P, ent[t], q, eneg[t]);
  }
  // tree over the signature's quads: quad k (k % 2s == 0) adds quad k + s
  SV_UNROLL for (int s = 1; s < QPS; s *= 2) {
    fe cp, mine;
    if (s == 1) fe_lane_down<4>(cp, P);
    else if (s == 2) fe_lane_down<8>(cp, P);
    else if (s == 4) fe_lane_down<16>(cp, P);
    else fe_lane_down<32>(cp, P);
    qo_to_cached(mine, cp, q);
    qo_add(P, mine, q, false);
  }

  __syncthreads();  // x_R, y_R from the decode wave
  // root quad: Q == R_pt  <=>  X == x_R Z and Y == y_R Z
  fe z, rc, t, dd;
  fe_from<2>(z, P);
  SV_UNROLL for (int i = 0; i < 10; ++i) rc.v[i] = s_r[ls][(role == 1 ? 10 : 0) + i];
  fe_mul(t, rc, z);
  fe_sub(dd, P, t);  // lane 0: X - x_R Z, lane 1: Y - y_R Z
  const uint32_t zr = fe_iszero(dd) ? 1u : 0u;
  const uint32_t eq = qd_from<0>(zr) & qd_from<1>(zr);
  const bool ok = eq != 0 && s_rok[ls] != 0 && s_ok && kst == SV_KEY_OK;
  if (active && quad == 0 && role == 0) p.verdict[g] = ok ? 1 : 0;
}

// Tables of -A for one key per wave (blockIdx.x = key): status, then
// entries d * 16^j (-A), d = 0..8, for j = 0..63.  Quad k owns positions
// 4k..4k+3: every quad runs the same doubling chain P_j = 16^j (-A) (in
// lockstep; the chain is serial anyway) and keeps the four points it owns,
// then builds their entries by repeated addition.  Entries are carried (R+).
__global__ __launch_bounds__(64, 1) void sv_keytab_kernel(const uint32_t* pks, const uint32_t* slots, uint32_t* ktab,
                                                          uint32_t* kstat) {
  const uint32_t key = blockIdx.x;
  const uint32_t lane = __lane_id();
  const uint32_t quad = lane >> 2, role = lane & 3u;
  const qd_role q{role == 1, role == 2, role == 3};
  uint32_t A[8];
  SV_UNROLL for (int i = 0; i < 8; ++i) A[i] = pks[8 * key + i];
  bool ok = sv_point_canonical(A) && !sv_small_order(A);
  ge_p3 nA;
  ok = ge_frombytes(nA, A, true) && ok;
  fe P;
  SV_UNROLL for (int i = 0; i < 10; ++i)
    P.v[i] = q.r1 ? nA.Y.v[i] : (q.r2 ? nA.Z.v[i] : (q.r3 ? nA.T.v[i] : nA.X.v[i]));
  fe own[4];
  SV_NOUNROLL for (int j = 0; j < SV_KA_POS; ++j) {
    const bool mine = (uint32_t)(j >> 2) == quad;
    SV_UNROLL for (int u = 0; u < 4; ++u)
      if ((j & 3) == u) fe_cmov(own[u], P, mine);
    if (j + 1 < SV_KA_POS) {
      SV_NOUNROLL for (int k = 0; k < 4; ++k) qo_dbl(P, q);
    }
  }
  const uint32_t slot = slots[key];
  uint32_t* base = ktab + (size_t)slot * SV_KEY_SLOT_DW;
  fe one;
  fe_1(one);
  fe idc;  // cached identity (1, 1, 1, 0)
  SV_UNROLL for (int i = 0; i < 10; ++i) idc.v[i] = q.r3 ? 0u : one.v[i];
  SV_UNROLL for (int u = 0; u < 4; ++u) {
    uint32_t* pe = base + (quad * 4 + u) * SV_KA_ENT * SV_CE_DW;
    ce_store(pe, role, idc);
    fe c1, w;
    qo_to_cached(c1, own[u], q);
    w = c1;
    fe_weak(w);
    ce_store(pe + SV_CE_DW, role, w);
    fe acc = own[u];
    SV_NOUNROLL for (int e = 2; e < SV_KA_ENT; ++e) {
      qo_add(acc, c1, q, false);
      qo_to_cached(w, acc, q);
      fe_weak(w);
      ce_store(pe + e * SV_CE_DW, role, w);
    }
  }
  if (lane == 0) kstat[slot] = ok ? SV_KEY_OK : SV_KEY_BAD;
}

// Tables of B: entry (j, e) = e * 256^j B, one lane each (init, once per device).
__global__ __launch_bounds__(128) void sv_comb_btab_kernel(uint32_t* ctab) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= SV_CB_POS * SV_CB_ENT) return;
  sv_comb_bentry(ctab + (size_t)id * SV_CE_DW, id / SV_CB_ENT, id % SV_CB_ENT);
}

// ------------------------------------------------------------ launchers
extern "C" {

size_t sv_comb_btab_bytes(void) { return (size_t)SV_CB_DW * 4; }
size_t sv_key_slot_bytes(void) { return (size_t)SV_KEY_SLOT_DW * 4; }

hipError_t sv_launch_comb_btab(uint32_t* d_ctab, hipStream_t s) {
  hipLaunchKernelGGL(sv_comb_btab_kernel, dim3((SV_CB_POS * SV_CB_ENT + 127) / 128), dim3(128), 0, s, d_ctab);
  return hipGetLastError();
}

// nkeys keys (pks: nkeys x 32 B, device) into the given slots
hipError_t sv_launch_keytab(const void* d_pks, const uint32_t* d_slots, uint32_t nkeys, uint32_t* d_ktab,
                            uint32_t* d_kstat, hipStream_t s) {
  if (nkeys == 0) return hipSuccess;
  hipLaunchKernelGGL(sv_keytab_kernel, dim3(nkeys), dim3(64), 0, s, (const uint32_t*)d_pks, d_slots, d_ktab, d_kstat);
  return hipGetLastError();
}

// signatures per chain wave for a batch of n (every workgroup alone on its CU
// while the batch fits the device's CUs)
int sv_comb_spw(uint64_t n, int cus) {
  const uint64_t wg1 = (n + 3 * 1 - 1) / (3 * 1), wg2 = (n + 3 * 2 - 1) / (3 * 2);
  if (wg1 <= (uint64_t)cus) return 1;
  if (wg2 <= (uint64_t)cus) return 2;
  return 4;
}

hipError_t sv_launch_comb(int mode, int spw, const void* pk, const void* sig, const void* msg, const uint64_t* off,
                          const uint32_t* len, uint32_t fixed_len, uint64_t n, void* verdict, const uint32_t* kslot,
                          const uint32_t* ktab, const uint32_t* kstat, const uint32_t* ctab, hipStream_t s) {
  if (n == 0) return hipSuccess;
  sv_comb_params c;
  c.k.pk = (const sv_u4*)pk;
  c.k.sig = (const sv_u4*)sig;
  c.k.msg = (const uint8_t*)msg;
  c.k.msg_off = off;
  c.k.msg_len = len;
  c.k.n = n;
  c.k.fixed_len = fixed_len;
  c.k.verdict = (uint8_t*)verdict;
  c.k.bitmap = nullptr;
  c.k.ws = nullptr;
  c.k.btab = nullptr;
  c.k.dbg = 0;
  c.k.status = nullptr;
  c.kslot = kslot;
  c.ktab = ktab;
  c.kstat = kstat;
  c.ctab = ctab;
  const uint64_t per = (uint64_t)SV_COMB_CHAIN_WAVES * (uint64_t)spw;
  const dim3 grid((unsigned)((n + per - 1) / per)), block(256);
#define SV_COMB_LAUNCH(M, W) hipLaunchKernelGGL((sv_comb_kernel<M, W>), grid, block, 0, s, c)
#define SV_COMB_MODES(W)                  \
  if (mode == 0) SV_COMB_LAUNCH(0, W);    \
  else if (mode == 1) SV_COMB_LAUNCH(1, W); \
  else SV_COMB_LAUNCH(2, W);
  if (spw == 1) {
    SV_COMB_MODES(1)
  } else if (spw == 2) {
    SV_COMB_MODES(2)
  } else {
    SV_COMB_MODES(4)
  }
#undef SV_COMB_MODES
#undef SV_COMB_LAUNCH
  return hipGetLastError();
}

}  // extern "C"
