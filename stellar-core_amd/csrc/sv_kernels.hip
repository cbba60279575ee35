// gfx950 kernels of the batched ed25519 verification engine.
//
//   sv_prep_kernel / sv_main_kernel  the throughput path: one lane per
//       signature, the half-size equation of lattice.h, per chunk a prep
//       kernel (hash, checks, decompression, Euclid, tables of -A / -R and
//       digit records into the chunk workspace) and a persistent main kernel
//       (the windowed double-scalar multiplication, table entries by LDS-DMA)
//   sv_octet_kernel  the latency path for keys not in the key cache: one
//       signature per octet of lanes, every point operation split over a quad
//       (quad.h); the warm-key kernel is sv_comb.hip
//   sv_btab_init_kernel  the base-point tables (device init)
//   sv_sign_kernel   the RFC 8032 signer (benchmark datasets)
// Retired kernel forms (the direct 253-bit ladder, the unsplit verify kernel,
// the one-quad latency kernel) and the compile-time switches that selected
// them were removed in round 4 (tools/unifdef.py; the shipped code objects
// were unchanged, tools/codeobj_digest.sh); they are in the git history.
#include <hip/hip_runtime.h>

#include <atomic>

#include "verify_core.h"
#include "quad.h"
#include "sv_kparams.h"
#include "keytab.h"

#define SV_BLOCK 256
#define SV_WAVES_PER_SIMD 2
// sv_main_kernel runs at 3 waves/SIMD (168 VGPRs): with its digits streamed
// from the record and one base address per staged entry it fits without
// spills in the loop; measured 1-1.5 % faster than 2 waves
// (profiles/r02/ab_main_waves.txt)
#ifndef SV_QUAD_WAVES
#define SV_QUAD_WAVES 3  // sv_quad_kernel (medium batches), waves per SIMD
#endif
#ifndef SV_MAIN_WAVES
#define SV_MAIN_WAVES 3
#endif
// base-point tables in the device buffer: e·B, then e·(2^128 B) (lattice.h)

// test knobs (include/stellar_sigverify.h sv_set_debug_flags)
#define SV_DBG_TRIVIAL_PAIR 1u  // every lane takes the fallback pair (h, 1)
#define SV_DBG_MAX_WINDOWS 2u   // every wave runs 64 windows
#define SV_DBG_PREP_ONLY 8u     // split path: prep kernel only (profiling; no verdicts)
#define SV_DBG_KEY_COLLIDE 16u  // per-key tables: every key gets the same fingerprint (collision path)
#define SV_DBG_DROP_HANDOVER 0x80u  // three-wave octet: the tables' hand-over flag is never raised (fail-closed test)
__device__ __forceinline__ int sv_wave_windows(int wl, uint32_t dbg) {
  int W = (dbg & SV_DBG_MAX_WINDOWS) ? 64 : SV_LAT_MIN_WINDOWS;
  while (__ballot(wl > W) != 0) ++W;
  return __builtin_amdgcn_readfirstlane(W);
}

__device__ __forceinline__ void sv_load_btab_lds(sv_u4* s_btab, const sv_u4* g_btab) {
  for (int i = threadIdx.x; i < SV_BTAB_ENTRIES * (SV_BTAB_STRIDE / 4); i += blockDim.x) s_btab[i] = g_btab[i];
  __syncthreads();
}

#ifdef SV_PHASE_PROF
__device__ unsigned long long sv_phase_cycles[8];
#define SV_PHASE(k)                                              \
  do {                                                           \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();  \
    if (lane == 0) atomicAdd(&sv_phase_cycles[k], t_ - t_prev);  \
    t_prev = t_;                                                 \
  } while (0)
#else
#define SV_PHASE(k) ((void)0)
#endif

// ---------------------------------------------- throughput path: prep + main
// The per-signature phases (SHA-512, checks, decompression, mod L, Euclid,
// tables, digits) and the scalar multiplication run as two kernels over a
// chunk of up to SV_CHUNK signatures:
//   sv_prep_kernel  one lane per signature, SV_PREP_WAVES waves/SIMD (the
//                   phases are serial chains that need the extra waves to
//                   hide their latency); writes the signature's tables and a
//                   7-quad digit record into the chunk workspace, and each
//                   wave's window count W into wmax[group].
//   sv_main_kernel  the hot loop only, SV_MAIN_WAVES (3) waves/SIMD, persistent.
// SV_PREP_WAVES = 3 (168 VGPRs, 128 B of scratch in the table build) measured
// 1.7-4.2 % faster prep than 2 (199 VGPRs, no scratch) in three A/B runs
// (profiles/r02/ab_prep_waves*.txt): the extra wave hides more issue latency
// than the spills cost.
// Workspace per signature of the chunk: SV_SLOT_QUADS_L quads of tables, then
// (separate array) SV_REC_QUADS quads of digits/flags.
#ifndef SV_PREP_WAVES
#define SV_PREP_WAVES 3
#endif
#ifndef SV_CHUNK
#define SV_CHUNK (1u << 20)
#endif
#define SV_REC_QUADS ((16 + 2 * SV_LB_DIGITS + 1 + 3) / 4)
// record: dA[8] dR[8] dB0[SV_LB_DIGITS] dB1[SV_LB_DIGITS] flags (9 quads at radix 2^16)
static_assert(16 + 2 * SV_LB_DIGITS + 2 <= 4 * SV_REC_QUADS, "digit record size");
// record flags
#define SV_REC_RNEG 1u
#define SV_REC_TOP8A 2u
#define SV_REC_TOP8R 4u
#define SV_REC_OK 8u

// ------------------------------------- per-key tables (throughput path)
// Catchup checkpoints, tx sets and SCP traffic sign with far fewer keys than
// signatures (a checkpoint: ~16 signatures per account).  With per-key tables
// on, each chunk first maps every signature's key to a slot of a persistent
// device table (sv_keyslot_kernel: one claim word per slot, compare-and-swap
// on a salted 64-bit fingerprint of the key); the first signature to claim a
// slot queues it, and sv_keybuild_kernel decodes each queued key ONCE
// (compacted: one lane per new key) into its entry: the key's 9 cached
// multiples of -A and a status bit (A canonical, not small-order, decodes).
// The prep kernel then skips A's square root and table build for a wave
// whose 64 keys all have a built entry with exactly their 32 bytes (a
// fingerprint collision or a full probe run leaves the lane's key uncached:
// the wave decodes inline as without tables), and the main kernel reads
// table_A from the entry.  Decoding is deterministic, so verdicts do not
// depend on the tables.  Entries are never modified after their build; the
// host clears the claim words when the claims reach `limit` (sv_api.cpp).
static_assert(SV_KT_TQUADS == SV_ATAB_ENTRIES * SV_LTAB_QUADS, "key-table entry layout");

struct sv_cparams {
  sv_kparams k;
  uint64_t start;  // first signature of the chunk
  uint64_t cnt;    // signatures in the chunk (<= SV_CHUNK)
  sv_u4* rec;      // SV_CHUNK x SV_REC_QUADS
  uint32_t* wmax;  // SV_CHUNK / 64
  sv_ktparams kt;
};

__device__ __forceinline__ unsigned long long sv_kt_fp(const uint32_t A[8], uint64_t salt, uint32_t dbg) {
  if (dbg & SV_DBG_KEY_COLLIDE) return 1ull;
  uint64_t h = salt;
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    h = (h ^ A[i]) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
  }
  return h | 1ull;
}

// Slot of every signature's key (one lane per signature of the chunk).
__global__ __launch_bounds__(SV_BLOCK) void sv_keyslot_kernel(sv_cparams c) {
  const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= c.cnt) return;
  const sv_ktparams& t = c.kt;
  uint32_t A[8];
  sv_unpack2(A, c.k.pk + 2 * (c.start + li));
  const unsigned long long fp = sv_kt_fp(A, t.salt, c.k.dbg);
  uint32_t ks = SV_KT_NONE;
  for (int q = 0; q < SV_KT_PROBES; ++q) {
    const uint64_t s = ((fp >> 17) + (uint64_t)q) & t.mask;
    unsigned long long w = __hip_atomic_load(&t.index[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w == 0ull) {
      if (__hip_atomic_load(&t.count[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= t.limit) break;
      w = atomicCAS(&t.index[s], 0ull, fp);
      if (w == 0ull) {  // claimed: sv_keybuild_kernel decodes this key into slot s
        sv_u4* e = t.store + s * SV_KT_QUADS + SV_KT_TQUADS;
        e[0] = sv_u4{A[0], A[1], A[2], A[3]};
        e[1] = sv_u4{A[4], A[5], A[6], A[7]};
        t.builders[atomicAdd(&t.count[0], 1u)] = (uint32_t)s;
        atomicAdd(&t.count[1], 1u);
        ks = (uint32_t)s;
        break;
      }
    }
    if (w == fp) {  // (the prep kernel compares the entry's 32 bytes)
      ks = (uint32_t)s;
      break;
    }
  }
  t.kslot[li] = ks;
}

// Decodes the keys claimed in this chunk, one lane per key.
__global__ __launch_bounds__(SV_BLOCK, SV_PREP_WAVES) void sv_keybuild_kernel(sv_cparams c) {
  const sv_ktparams& t = c.kt;
  const uint32_t nb = t.count[0];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  if (i - lane >= nb) return;  // (wave-uniform)
  const bool active = i < nb;
  const uint32_t s = t.builders[active ? i : nb - 1];  // (idle tail lanes redo the last key: same bytes)
  sv_u4* e = t.store + (uint64_t)s * SV_KT_QUADS;
  uint32_t A[8];
  sv_unpack2(A, e + SV_KT_TQUADS);
  bool ok = sv_point_canonical(A) && !sv_small_order(A);
  ge_p3 negA;
  ok = ge_frombytes(negA, A, true) && ok;
  sv_build_ltab(e, negA);
  if (active) e[SV_KT_TQUADS + 2] = sv_u4{ok ? 1u : 0u, 0u, 0u, 0u};
}

// KT: per-key tables on (a separate instantiation, so the tables-off path
// carries none of their code).  DF (decode first; launches whose inputs are
// read in place from mapped host memory, SV_KP_IN_PLACE): a lane loads A and
// R, decodes both and builds their tables -- 60 % of the kernel -- and only
// then loads S and the message and hashes: the half of each row the decode
// needs crosses PCIe first, and the rest arrives while the decodes run,
// instead of every wave waiting out its whole row first (the quad kernel's
// order).  The same checks, combined as one conjunction,
// so the verdicts are unchanged.  Not with KT (a table-backed A skips its
// decode) and not for device-resident inputs (the headline path keeps its
// measured order).
template <int MODE, bool KT, bool DF = false>
__global__ __launch_bounds__(SV_BLOCK, SV_PREP_WAVES) void sv_prep_kernel(sv_cparams c) {
  static_assert(!(KT && DF), "decode-first runs without per-key tables");
  const sv_kparams& p = c.k;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // index in the chunk
  if (li - lane >= c.cnt) return;                                        // (wave-uniform)
  const bool active = li < c.cnt;
  const uint64_t ii = c.start + (active ? li : c.cnt - 1);  // idle tail lanes redo the last item
#ifdef SV_DIAG_PREP_ALIAS  // (diagnostic builds only: table writes into a small region)
  sv_u4* tabA = p.ws + (li & (uint64_t)(SV_DIAG_PREP_ALIAS - 1)) * SV_SLOT_QUADS_L;
#else
  sv_u4* tabA = p.ws + li * SV_SLOT_QUADS_L;
#endif
  sv_u4* tabR = tabA + SV_ATAB_ENTRIES * SV_LTAB_QUADS;
#ifdef SV_PHASE_PROF
  unsigned long long t_prev = __builtin_amdgcn_s_memtime();
#endif
  uint32_t A[8], S[8], hram[16], R[8];
  sv_lat lat;
  bool ok;
  uint32_t ks = SV_KT_NONE;
  if (DF) {
    sv_unpack2(A, p.pk + 2 * ii);
    sv_unpack2(R, p.sig + 4 * ii);
    bool dok;
    {
      ge_p3 negA;
      dok = ge_frombytes(negA, A, true);
      sv_build_ltab(tabA, negA);
    }
    {
      ge_p3 negR;
      dok = ge_frombytes(negR, R, true) && dok;
      sv_build_ltab(tabR, negR);
    }
    sv_load_rest_and_hash<MODE>(p, ii, A, R, S, hram);
    ok = sc_is_canonical(S) && !sv_small_order(R) && sv_point_canonical(R) && sv_point_canonical(A) &&
         !sv_small_order(A) && dok;
    uint32_t h[8];
    sc_reduce512(h, hram);
    sc_lattice_reduce(lat, h, (p.dbg & SV_DBG_TRIVIAL_PAIR) != 0);
  } else {
#ifdef SV_PHASE_PROF
  {
    uint32_t M[8];
    sv_unpack2(A, p.pk + 2 * ii);
    sv_unpack2(R, p.sig + 4 * ii);
    sv_unpack2(S, p.sig + 4 * ii + 2);
    sv_unpack2(M, (const sv_u4*)(p.msg) + 2 * ii);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    SV_PHASE(5);
    sha512_ram32(hram, R, A, M);
  }
#else
  sv_load_and_hash<MODE>(p, ii, A, S, hram);
  sv_unpack2(R, p.sig + 4 * ii);
#endif
  SV_PHASE(0);
  // per-key tables: skip A for a wave whose keys all have a built entry
  int a_status = -1;
  if (KT) {
    ks = c.kt.kslot[active ? li : c.cnt - 1];
    bool hit = false;
    uint32_t st = 0;
    if (ks != SV_KT_NONE) {
      const sv_u4* e = c.kt.store + (uint64_t)ks * SV_KT_QUADS + SV_KT_TQUADS;
      const sv_u4 k0 = e[0], k1 = e[1], k2 = e[2];
      hit = k0.x == A[0] && k0.y == A[1] && k0.z == A[2] && k0.w == A[3] && k1.x == A[4] && k1.y == A[5] &&
            k1.z == A[6] && k1.w == A[7];
      st = k2.x;
    }
    if (__ballot(!hit) == 0) a_status = (int)(st & 1u);
    else ks = SV_KT_NONE;
  }
#ifdef SV_PHASE_PROF
  ok = sc_is_canonical(S) && !sv_small_order(R) && sv_point_canonical(A) && !sv_small_order(A) &&
            sv_point_canonical(R);
  ge_p3 negA, negR;
  ok = ge_frombytes(negA, A, true) && ok;
  ok = ge_frombytes(negR, R, true) && ok;
  SV_PHASE(1);
  {
    uint32_t h[8];
    sc_reduce512(h, hram);
    sc_lattice_reduce(lat, h, (p.dbg & SV_DBG_TRIVIAL_PAIR) != 0);
  }
  SV_PHASE(2);
  sv_build_ltab(tabA, negA);
  sv_build_ltab(tabR, negR);
  SV_PHASE(3);
#else
  ok = sv_lat_pre(lat, A, R, S, hram, tabA, tabR, (p.dbg & SV_DBG_TRIVIAL_PAIR) != 0, a_status);
#endif
  }
  const int W = sv_wave_windows(sv_lat_windows(lat.bits), p.dbg);
  sv_lat_digits D;
  sv_lat_prepare(D, lat, S, W);
  const uint32_t flags = (D.rneg ? SV_REC_RNEG : 0u) | (D.top8A ? SV_REC_TOP8A : 0u) |
                         (D.top8R ? SV_REC_TOP8R : 0u) | (ok ? SV_REC_OK : 0u);
  uint32_t rw[4 * SV_REC_QUADS];
  SV_UNROLL for (int k = 0; k < 4 * SV_REC_QUADS; ++k) rw[k] = 0u;
  SV_UNROLL for (int k = 0; k < 8; ++k) {
    rw[k] = D.dA[k];
    rw[8 + k] = D.dR[k];
  }
  SV_UNROLL for (int k = 0; k < SV_LB_DIGITS; ++k) {
    rw[16 + k] = (uint32_t)D.dB0[k];
    rw[16 + SV_LB_DIGITS + k] = (uint32_t)D.dB1[k];
  }
  rw[16 + 2 * SV_LB_DIGITS] = flags;
  rw[16 + 2 * SV_LB_DIGITS + 1] = ks;  // table_A: key entry ks, or (SV_KT_NONE) the lane's slot
  sv_u4* r = c.rec + li * SV_REC_QUADS;
  SV_UNROLL for (int k = 0; k < SV_REC_QUADS; ++k) r[k] = sv_u4{rw[4 * k], rw[4 * k + 1], rw[4 * k + 2], rw[4 * k + 3]};
  if (lane == 0) c.wmax[li >> 6] = (uint32_t)W;
  SV_PHASE(4);
}

// The main kernel's scalar multiplication: the step machine of
// sv_lat_scalarmult (verify_core.h, STAGED with one stage region) with the
// digits streamed from the signature's record instead of held in registers
// (33 VGPRs -> 7: what lets the kernel run at 3 waves/SIMD without spills).
// Record words (sv_prep_kernel): dA[0..7], dR[8..15] = the radix-16 digit
// strings after sv_lat_prepare's shift, so window w's digit is nibble
// p = w + 64 - W; dB0[16..23], dB1[24..31] = base-point digits j (window 4j).
__device__ __forceinline__ int32_t sv_nibble(uint32_t word, int p) {
  return (int32_t)__builtin_amdgcn_sbfe((int)word, (unsigned)(4 * (p & 7)), 4u);
}
// The identity entry of every -A / -R table (digit 0), one copy per device:
// the prep kernel does not write each signature's entry 0 (verify_core.h
// sv_build_ltab) and the main kernel stages digit-0 additions from here (an
// L2-resident line).
__device__ sv_u4 sv_ident_lentry[SV_LTAB_QUADS] = {{1u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 1u, 0u},
                                                    {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {1u, 0u, 0u, 0u},
                                                    {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u},
                                                    {0u, 0u, 0u, 0u}};
__device__ __forceinline__ const sv_u4* sv_lentry_at(const sv_u4* tab, int32_t d) {
  if (d == 0) return sv_ident_lentry;
  return tab + (d < 0 ? -d : d) * SV_LTAB_QUADS;
}
__device__ __forceinline__ void sv_main_scalarmult(ge_p3& P, const uint32_t* rw, uint32_t flags, int W,
                                                   const sv_u4* tabA, const sv_u4* tabR, const sv_u4* btab0,
                                                   const sv_u4* btab1, sv_u4* stage) {
#if defined(__HIP_DEVICE_COMPILE__)
  const bool top8A = (flags & SV_REC_TOP8A) != 0, top8R = (flags & SV_REC_TOP8R) != 0;
  const bool rneg = (flags & SV_REC_RNEG) != 0;
  // current and next digit words (the word changes every 8 windows)
  uint32_t curA = rw[7], curR = rw[15], nxtA = rw[6], nxtR = rw[14];
  ge_p1p1 Q;
  {
    // Window W-1 (no doublings; above every base-point window), peeled: P is
    // the identity, so P + Q_A = Q_A is taken straight from the (pre-swapped)
    // cached entry as (2X : 2Y : 2Z : 2T) -- (Y+X) - (Y-X), (Y+X) + (Y-X), 2Z
    // and 2T = (2dT) / d, negated for a negative digit -- instead of a full
    // addition and conversion (8 products -> 1); then the R entry is added.
    int32_t dA = top8A ? 8 : sv_nibble(curA, 63), dR = top8R ? 8 : sv_nibble(curR, 63);
    if (rneg) dR = -dR;
    fe qa, qb, qz, qt;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sv_stage_lentry(stage, sv_lentry_at(tabA, dA));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sv_load_lentry(qa, qb, qz, qt, stage + __lane_id(), 64, dA < 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sv_stage_lentry(stage, sv_lentry_at(tabR, dR));
    fe_sub(P.X, qa, qb);
    fe_add(P.Y, qa, qb);
    fe_add(P.Z, qz, qz);
    fe di, nt;
    fe_const_dinv(di);
    fe_mul(P.T, qt, di);
    fe_neg(nt, P.T);
    SV_UNROLL for (int i = 0; i < 10; ++i) P.T.v[i] = dA < 0 ? nt.v[i] : P.T.v[i];
    fe_weak(P.X);  // (the addition below takes p at R)
    fe_weak(P.Y);
    fe_weak(P.Z);
    fe_weak(P.T);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sv_load_lentry(qa, qb, qz, qt, stage + __lane_id(), 64, dR < 0);
    ge_add_preswapped(Q, P, qa, qb, qz, qt, dR < 0, false);
    ge_p1p1_to_p3_opt(P, Q, false);  // (a doubling comes next)
  }
  SV_NOUNROLL for (int w = W - 2; w >= 0; --w) {
    const int pos = w + 64 - W;  // (wave-uniform)
    if ((pos & 7) == 7 && w != W - 1) {
      curA = nxtA;
      curR = nxtR;
      const int k = (pos >> 3) - 1;
      if (k >= 0) {
        nxtA = rw[k];
        nxtR = rw[8 + k];
      }
    }
    int32_t dA = sv_nibble(curA, pos), dR = sv_nibble(curR, pos);
    if (w == W - 1) {
      if (top8A) dA = 8;
      if (top8R) dR = 8;
    }
    if (rneg) dR = -dR;
    const bool bwin = w % SV_LB_WIN == 0 && w / SV_LB_WIN < SV_LB_DIGITS;
    int32_t dB0 = 0, dB1 = 0;
    if (bwin) {
      dB0 = (int32_t)rw[16 + w / SV_LB_WIN];
      dB1 = (int32_t)rw[16 + SV_LB_DIGITS + w / SV_LB_WIN];
#ifdef SV_DIAG_BTAB_ALIAS  // (diagnostic builds only: wrong verdicts; base-point entries from a small range)
      dB0 %= SV_DIAG_BTAB_ALIAS;
      dB1 %= SV_DIAG_BTAB_ALIAS;
#endif
    }
    const int nsteps = bwin ? 8 : 6;
    const int s0 = (w == W - 1) ? 4 : 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sv_stage_lentry(stage, sv_lentry_at(tabA, dA));
    SV_NOUNROLL for (int s = s0; s < nsteps; ++s) {
      if (s < 4) {
        ge_dbl(Q, P.X, P.Y, P.Z);
      } else {
        fe qa, qb, qz, qt;
        bool neg;
        const bool zone = s >= 6;
        // the entry DMA'd for this step (and any digit load) has landed; once
        // the entry is read, the stage receives the next addition's entry
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!zone) {
          neg = (s == 4 ? dA : dR) < 0;
          sv_load_lentry(qa, qb, qz, qt, stage + __lane_id(), 64, neg);
          if (s == 4 || bwin) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (s == 4) sv_stage_lentry(stage, sv_lentry_at(tabR, dR));
            else sv_stage_bentry(stage, btab0, dB0);
          }
        } else {
          neg = (s == 6 ? dB0 : dB1) < 0;
          fe_1(qz);
          const sv_u4* st = stage + __lane_id();
          sv_load_fe3(qa, st, 64);
          sv_load_fe3(qb, st + 3 * 64, 64);
          sv_load_fe3(qt, st + 6 * 64, 64);
          if (s == 6) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            sv_stage_bentry(stage, btab1, dB1);
          }
        }
        ge_add_preswapped(Q, P, qa, qb, qz, qt, neg, zone);
      }
      ge_p1p1_to_p3_opt(P, Q, s + 1 >= 4 && s + 1 < nsteps);
    }
  }
#endif
}

template <bool KT>
__global__ __launch_bounds__(SV_BLOCK, SV_MAIN_WAVES) void sv_main_kernel(sv_cparams c) {
  const sv_kparams& p = c.k;
  __shared__ sv_u4 s_stage[SV_BLOCK / 64][SV_LTAB_QUADS * 64];  // per-wave entry stage
  const uint32_t lane = threadIdx.x & 63u;
  sv_u4* stage = s_stage[threadIdx.x >> 6];
  const uint64_t gtid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const sv_u4* btab0 = p.btab;
  const sv_u4* btab1 = p.btab + SV_LBTAB_ENTRIES * SV_BTAB_QUADS;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = gtid - lane; base < c.cnt; base += stride) {
    const uint64_t li = base + lane;  // (slots exist up to the chunk's last full wave)
    const bool active = li < c.cnt;
#ifdef SV_DIAG_TAB_ALIAS  // (diagnostic builds only: wrong verdicts; table reads from a small region)
    const sv_u4* slot = p.ws + (li & (uint64_t)(SV_DIAG_TAB_ALIAS - 1)) * SV_SLOT_QUADS_L;
#else
    const sv_u4* slot = p.ws + li * SV_SLOT_QUADS_L;
#endif
    const sv_u4* tabR = slot + SV_ATAB_ENTRIES * SV_LTAB_QUADS;
    const uint32_t* rw = (const uint32_t*)(c.rec + li * SV_REC_QUADS);
    const uint32_t flags = rw[16 + 2 * SV_LB_DIGITS];
    const sv_u4* tabA = slot;
    if (KT) {
      const uint32_t ks = rw[16 + 2 * SV_LB_DIGITS + 1];
      if (ks != SV_KT_NONE) tabA = c.kt.store + (uint64_t)ks * SV_KT_QUADS;
    }
    const bool pre_ok = (flags & SV_REC_OK) != 0;
    const int W = (int)__builtin_amdgcn_readfirstlane(c.wmax[li >> 6]);
    ge_p3 P;
    sv_main_scalarmult(P, rw, flags, W, tabA, tabR, btab0, btab1, stage);
    const bool ok = pre_ok && sv_is_identity(P) && active;
    if (active) p.verdict[c.start + li] = ok ? 1 : 0;
    const uint64_t mask = __ballot(ok);
    if (p.bitmap != nullptr && lane == 0) p.bitmap[(c.start + base) >> 6] = mask;
  }
}

// ------------------------------------------- latency path (quad.h)
// Helpers of the octet kernel below (every point operation split over a quad
// of lanes).
#define SV_QENT_DW 40  // cached entry: YpX, YmX, Z, T2d x 10 dwords

// this lane's operand of cached entry e (LDS): role 0 T2d, role 1 Z, roles
// 2 / 3 the (Y+X, Y-X) pair swapped when neg
__device__ __forceinline__ void qd_load_cached(fe& o, const uint32_t* ent, uint32_t role, bool neg) {
  const uint32_t comp = role == 0 ? 3u : role == 1 ? 2u : ((role == 2) != neg ? 0u : 1u);
  const uint32_t* src = ent + 10 * comp;
  SV_UNROLL for (int k = 0; k < 10; ++k) o.v[k] = src[k];
}
// this lane's operand of affine base-point entry e (global): role 0 2dxy,
// role 1 the constant 1 (Z), roles 2 / 3 the (y+x, y-x) pair swapped when neg
__device__ __forceinline__ void qd_load_affine(fe& o, const sv_u4* ent, uint32_t role, bool neg) {
  const uint32_t comp = role == 0 ? 2u : ((role == 2) != neg ? 0u : 1u);
  const sv_u4* src = ent + 3 * comp;
  const sv_u4 a = src[0], b = src[1], c = src[2];
  o.v[0] = a.x; o.v[1] = a.y; o.v[2] = a.z; o.v[3] = a.w;
  o.v[4] = b.x; o.v[5] = b.y; o.v[6] = b.z; o.v[7] = b.w;
  o.v[8] = c.x; o.v[9] = c.y;
  if (role == 1) fe_1(o);
}

// ------------------------------------------- latency path, two quads per signature
// One signature per OCTET of lanes: the two quads of
// the octet evaluate the two halves of (*) in lattice.h in parallel,
//   quad 0:  P_A = [c0](-A) + [s_lo] B           (table_A, e B)
//   quad 1:  P_R = [c1](-R) + [s_hi] 2^128 B     (table_R, e 2^128 B)
// over the same W windows (each quad: 4 doublings, ONE table addition and, on
// base windows, ONE base-point addition per window, every point operation
// split over its 4 lanes as in quad.h), then quad 0 adds P_R (fetched from
// lanes + 4 by DPP row_shl:4) and tests P_A + P_R for the identity.  Against
// one quad per signature this removes one variable and one base addition per
// window from the serial chain; quad 0 decompresses A and quad 1 R, as the
// even / odd lanes of a quad did before.  8 signatures per single-wave
// workgroup.
#define SV_OSIGS 8

// value of lane + 4 (row_shl:4 within each row of 16: lanes 0-3 <- 4-7 and
// 8-11 <- 12-15, i.e. quad 0 of every octet reads quad 1)
__device__ __forceinline__ uint32_t oc_from_hi(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x104, 0xf, 0xf, false);
}
__device__ __forceinline__ void fe_from_hi(fe& o, const fe& f) {
  SV_UNROLL for (int i = 0; i < 10; ++i) o.v[i] = oc_from_hi(f.v[i]);
}

// Two waves per 8 signatures.  The base-point part [s]B of (*) (lattice.h)
// runs on wave 1 after its table build (its own 112 doublings, 8 additions
// per half) while wave 0 runs the -A / -R chains without base additions;
// wave 0 adds the result at the end (second LDS handoff).
#define SV_OCTET_BLOCK 128
// HI (cold batches while no bulk work runs, sv_launch_verify): a third wave
// per workgroup runs the top windows of the -A / -R chains.  It starts as soon
// as the decode wave has the decoded points (before their tables), doubles
// them 4 Wlo times (Q = 16^Wlo P), builds Q's tables in LDS and runs windows
// W-1 .. Wlo; wave 0 runs Wlo-1 .. 0 and adds the high part at the end.  The
// third wave repeats the doublings, so what it saves is the additions of its
// windows, plus the head start it gets on wave 0, which waits for the tables:
// balanced at about W / SV_OCT_HI_DIV of them, W / SV_OCT_HI_DIV_WIDE for
// launches the host marks SV_KP_OCT_HI_WIDE (more workgroups than CUs, where
// wave 0 shares its SIMD more often).
// The waves of a HI workgroup hand over through LDS flags, not barriers (a
// barrier would hold the third wave until the table build is done): one
// barrier at entry clears the flags, each hand-over is data, a release fence
// and a flag store, and each wait an acquire after the flag is seen.
#define SV_OCTET_BLOCK_HI 192
#ifndef SV_OCT_HI_DIV
#define SV_OCT_HI_DIV 6
#endif
#ifndef SV_OCT_HI_DIV_WIDE
#define SV_OCT_HI_DIV_WIDE 4
#endif
// windows the third wave doubles through before it needs W (wave 0's lattice
// reduction); a split that would leave wave 0 fewer is not made (tiny W: the
// high part is then the identity)
#define SV_OCT_HI_PRE 20
__device__ __forceinline__ int sv_oct_hi_windows(int W, uint32_t dbg) {
  const int div = (dbg & SV_KP_OCT_HI_WIDE) ? SV_OCT_HI_DIV_WIDE : SV_OCT_HI_DIV;
  int h = (W + div / 2) / div;
  h = h < 1 ? 1 : (h > W ? W : h);
  return W - h < SV_OCT_HI_PRE ? 0 : h;
}
enum { SV_OF_PT = 0, SV_OF_TAB, SV_OF_DIG, SV_OF_PB, SV_OF_PHI, SV_OF_N };
// hand-over: this wave's LDS writes before the flag; good = false marks
// data computed after a wait of this wave that timed out
__device__ __forceinline__ void sv_oflag_set(uint32_t* f, bool good = true) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63u) == 0) __hip_atomic_store(f, good ? 1u : 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wait for a hand-over; true if it came and was good.  Bounded (~0.5 s): a
// lost flag must not hang the kernel.  Wave 0 rejects the workgroup's
// signatures unless every hand-over it used was good (fail closed).
__device__ __forceinline__ bool sv_oflag_wait(uint32_t* f) {
  uint32_t v = 0;
  for (uint32_t it = 0; it < (1u << 24); ++it) {
    v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    if (v != 0) break;
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return v == 1;
}

// The tables (23 KB) are dynamic LDS, placed after the static arrays below:
// measured 2.2 us faster per cold 1k batch than the same tables as the first
// static array (0.2428 -> 0.2406 ms, 8 of 8 rounds, profiles/r04/ab_octlds/).
#define SV_OCTET_TAB_BYTES (SV_OSIGS * 2 * SV_ATAB_ENTRIES * SV_QENT_DW * 4)
// + the hash wave's message windows (sv_load_and_hash_lds), after the tables.
// MSG: launches of at most one workgroup per CU (n <= 8 per CU) only; larger
// ones read the message from memory (the extra 4 KB would cost a
// workgroup slot per CU: 12288 cold 0.58 -> 0.80 ms).
#define SV_OCTET_LDS_BYTES(MSG, HI) (((HI) ? 2 : 1) * SV_OCTET_TAB_BYTES + ((MSG) ? SV_OSIGS * SV_MSG_CAP : 0))
// (cached-form table of 0..8 multiples of P, whole on every lane of the quad,
// into `tab` by the quad's role-0 lane: the decode wave's build, and HI's)
__device__ __forceinline__ void sv_oct_build_table(uint32_t* tab, const ge_p3& Pt, const qd_role& q, uint32_t role) {
  ge_cached c1, ce;
  ge_p3_to_cached(c1, Pt);
  ge_cached_identity(ce);
  const bool store = role == 0;
  if (store) sv_store_lentry((sv_u4*)tab, ce);
  if (store) sv_store_lentry((sv_u4*)(tab + SV_QENT_DW), c1);
  // entries 2..8 by repeated addition of P, each addition split over the
  // quad (qd_add: one product per lane and stage) instead of one lane's
  // serial 8 products
  fe mine;
  fe_pick4(mine, q, c1.T2d, c1.Z, c1.YpX, c1.YmX);
  ge_p3 P3 = Pt;
  SV_NOUNROLL for (int e = 2; e < SV_ATAB_ENTRIES; ++e) {
    qd_add(P3, mine, q, false, true);
    ge_p3_to_cached(ce, P3);
    if (store) sv_store_lentry((sv_u4*)(tab + e * SV_QENT_DW), ce);
  }
}
template <int MODE, bool MSG, bool HI>
__global__ __launch_bounds__(HI ? SV_OCTET_BLOCK_HI : SV_OCTET_BLOCK, 1) void sv_octet_kernel(sv_kparams p) {
  // (16-byte aligned: the tables and the message windows are read as sv_u4)
  extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
  static_assert(SV_OCTET_TAB_BYTES % 16 == 0, "the message windows follow the tables at a 16-byte boundary");
  uint32_t(*s_tab)[2][SV_ATAB_ENTRIES][SV_QENT_DW] = (uint32_t(*)[2][SV_ATAB_ENTRIES][SV_QENT_DW])s_dyn;
  // (HI: the tables of Q = 16^Wlo P after them)
  uint32_t(*s_tabh)[2][SV_ATAB_ENTRIES][SV_QENT_DW] =
      (uint32_t(*)[2][SV_ATAB_ENTRIES][SV_QENT_DW])(s_dyn + SV_OCTET_TAB_BYTES / 4);
  __builtin_amdgcn_s_setprio(3);  // latency class (as sv_comb_kernel)
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t role = lane & 3u, half = (lane >> 2) & 1u, sl = lane >> 3;
  const qd_role q{role == 1, role == 2, role == 3};
  const uint64_t i = (uint64_t)blockIdx.x * SV_OSIGS + sl;
  const bool active = i < p.n;
  const uint64_t ii = active ? i : p.n - 1;  // idle tail octets redo the last item
  // Two waves per workgroup, same lane -> (signature, quad, role) map.  The
  // decompressions and table builds (wave 1) do not depend on the hash, the
  // scalar reduction and the Euclid reduction (wave 0), so the two chains run
  // side by side on two SIMDs instead of one after the other; wave 1 hands
  // over the tables in LDS (as before) and its decode verdicts in s_dok.
  __shared__ uint32_t s_dok[SV_OSIGS];
  // wave-uniform, and visibly so to the compiler (a scalar branch): a
  // divergent-looking branch would be structurized with EXEC masking and
  // both waves would then execute both barriers
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool dec_wave = wv == 1;
  const bool hi_wave = HI && wv == 2;
  // HI: the decoded points (decode wave -> high wave), the digit strings and
  // the window split (wave 0 -> high wave), the high part (high wave -> wave 0)
  __shared__ uint32_t s_pt[HI ? SV_OSIGS : 1][2][40];
  __shared__ uint32_t s_hd[HI ? SV_OSIGS : 1][2][9];  // dg[8], flags (1 top8, 2 flip)
  __shared__ int32_t s_win[2];                         // W, Wlo
  __shared__ uint32_t s_phi[HI ? SV_OSIGS : 1][2][SV_QENT_DW];
  __shared__ uint32_t s_oflag[HI ? SV_OF_N : 1];
  if (HI) {
    if (threadIdx.x < SV_OF_N) s_oflag[threadIdx.x] = 0;
    __syncthreads();  // (the only barrier of a HI workgroup)
  }
  if (hi_wave) {
    bool good = sv_oflag_wait(&s_oflag[SV_OF_PT]);  // the decoded points
    fe h;
    {
      const uint32_t* src = &s_pt[sl][half][10 * role];  // own form: lane r holds coordinate r
      SV_UNROLL for (int k = 0; k < 10; ++k) h.v[k] = src[k];
    }
    SV_NOUNROLL for (int k = 0; k < 4 * SV_OCT_HI_PRE; ++k) qo_dbl(h, q);
    good = sv_oflag_wait(&s_oflag[SV_OF_DIG]) && good;  // the digits and the split
    const int W = s_win[0], Wlo = s_win[1];
    if (Wlo < W) {  // (Wlo >= SV_OCT_HI_PRE then, sv_oct_hi_windows)
      SV_NOUNROLL for (int k = 4 * SV_OCT_HI_PRE; k < 4 * Wlo; ++k) qo_dbl(h, q);
      ge_p3 Q;
      qo_expand(Q, h);
      uint32_t* tabh = &s_tabh[sl][half][0][0];
      sv_oct_build_table(tabh, Q, q, role);
      // (this wave reads back what its role-0 lanes stored: LDS is in order
      // within a wave)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      uint32_t dg[8];
      SV_UNROLL for (int k = 0; k < 8; ++k) dg[k] = s_hd[sl][half][k];
      const uint32_t fl = s_hd[sl][half][8];
      const bool top8 = (fl & 1u) != 0, flip = (fl & 2u) != 0;
      qo_identity(h, q);
      SV_NOUNROLL for (int w = W - 1; w >= Wlo; --w) {
        int32_t d = sc_pop_top(dg, 4);
        if (w == W - 1 && top8) d = 8;
        if (flip) d = -d;
        if (w != W - 1) {
          SV_NOUNROLL for (int k = 0; k < 4; ++k) qo_dbl(h, q);
        }
        fe m;
        qo_load_cached(m, tabh + (d < 0 ? -d : d) * SV_QENT_DW, role, d < 0);
        qo_add(h, m, q, d < 0);
      }
    } else {
      qo_identity(h, q);  // (no high windows: the identity)
    }
    ge_p3 PH;
    qo_expand(PH, h);
    ge_cached ch;
    ge_p3_to_cached(ch, PH);
    if (role == 0) sv_store_lentry((sv_u4*)&s_phi[sl][half][0], ch);
    sv_oflag_set(&s_oflag[SV_OF_PHI], good);  // the high parts written
    return;
  }
  uint32_t A[8], S[8], hram[16], R[8];
  if (dec_wave) {
    sv_unpack2(A, p.pk + 2 * ii);
    sv_unpack2(R, p.sig + 4 * ii);
  } else {
    if (MSG) {
      sv_u4* s_msg = (sv_u4*)(s_dyn + (HI ? 2 : 1) * SV_OCTET_TAB_BYTES / 4);
      sv_load_and_hash_lds<MODE, 8>(p, ii, lane & 7u, s_msg + sl * (SV_MSG_CAP / 16), A, S, hram);
    } else {
      sv_load_and_hash<MODE>(p, ii, A, S, hram);
    }
    sv_unpack2(R, p.sig + 4 * ii);
  }
  bool ok = true;
  if (dec_wave) {
    // decompress: quad 0 -A, quad 1 -R; role 0 of each quad stores its table
    uint32_t E[8];
    SV_UNROLL for (int k = 0; k < 8; ++k) E[k] = half ? R[k] : A[k];
    ge_p3 Pt;
    const uint32_t dok = ge_frombytes(Pt, E, true) ? 1u : 0u;
    // (the DPP read outside the branch: a lane disabled by EXEC is no source)
    const uint32_t both = dok & oc_from_hi(dok);
    if (half == 0 && role == 0) s_dok[sl] = both;
    if (HI && role == 0) {  // (the high wave's starting point)
      SV_UNROLL for (int k = 0; k < 10; ++k) {
        s_pt[sl][half][k] = Pt.X.v[k];
        s_pt[sl][half][10 + k] = Pt.Y.v[k];
        s_pt[sl][half][20 + k] = Pt.Z.v[k];
        s_pt[sl][half][30 + k] = Pt.T.v[k];
      }
    }
    if (HI) sv_oflag_set(&s_oflag[SV_OF_PT]);
    ge_cached c1, ce;
    ge_p3_to_cached(c1, Pt);
    ge_cached_identity(ce);
    uint32_t* tab = &s_tab[sl][half][0][0];
    const bool store = role == 0;
    if (store) sv_store_lentry((sv_u4*)tab, ce);
    if (store) sv_store_lentry((sv_u4*)(tab + SV_QENT_DW), c1);
    // entries 2..8 by repeated addition of P, each addition split over the
    // quad (qd_add: one product per lane and stage) instead of one lane's
    // serial 8 products
    fe mine;
    fe_pick4(mine, q, c1.T2d, c1.Z, c1.YpX, c1.YmX);
    ge_p3 P3 = Pt;
    SV_NOUNROLL for (int e = 2; e < SV_ATAB_ENTRIES; ++e) {
      qd_add(P3, mine, q, false, true);
      ge_p3_to_cached(ce, P3);
      if (store) sv_store_lentry((sv_u4*)(tab + e * SV_QENT_DW), ce);
    }
  }
  __shared__ int32_t s_bd[SV_OSIGS][2][SV_LB_DIGITS];  // base-point digits (wave 0 -> 1)
  __shared__ uint32_t s_pb[SV_OSIGS][SV_QENT_DW];       // [s]B, cached form (wave 1 -> 0)
  if (dec_wave) {
    bool dig_good = true;
    if (HI) {
      if (!(p.dbg & SV_DBG_DROP_HANDOVER)) sv_oflag_set(&s_oflag[SV_OF_TAB]);  // tables and s_dok written
      dig_good = sv_oflag_wait(&s_oflag[SV_OF_DIG]);  // s_bd
    } else {
      __syncthreads();  // tables and s_dok written; s_bd read below
    }
    {
      // quad 0: [s_lo] B from e B, quad 1: [s_hi] 2^128 B from e 2^128 B;
      // digit j carries weight 2^(16 j) (Horner: 16 doublings between digits)
      int32_t bd[SV_LB_DIGITS];
      SV_UNROLL for (int j = 0; j < SV_LB_DIGITS; ++j) bd[j] = s_bd[sl][half][j];
      const sv_u4* btab = p.btab + (half ? SV_LBTAB_ENTRIES * SV_BTAB_QUADS : 0);
      fe h;
      qo_identity(h, q);
      SV_NOUNROLL for (int j = SV_LB_DIGITS - 1; j >= 0; --j) {
        int32_t dB = bd[SV_LB_DIGITS - 1];
        SV_UNROLL for (int k = SV_LB_DIGITS - 1; k > 0; --k) bd[k] = bd[k - 1];
        fe b;
        qo_load_affine(b, btab + (dB < 0 ? -dB : dB) * SV_BTAB_QUADS, role, dB < 0);  // lands during the doublings
        if (j != SV_LB_DIGITS - 1) {
          SV_NOUNROLL for (int k = 0; k < 4 * SV_LB_WIN; ++k) qo_dbl(h, q);
        }
        qo_add(h, b, q, dB < 0);
      }
      ge_p3 PB;
      qo_expand(PB, h);
      // quad 0: + quad 1's half (lanes + 4), then the sum in cached form
      ge_p3 P1;
      fe_from_hi(P1.X, PB.X);
      fe_from_hi(P1.Y, PB.Y);
      fe_from_hi(P1.Z, PB.Z);
      fe_from_hi(P1.T, PB.T);
      ge_cached c1;
      ge_p3_to_cached(c1, P1);
      fe mine;
      fe_pick4(mine, q, c1.T2d, c1.Z, c1.YpX, c1.YmX);  // qd_add's operand order
      qd_add(PB, mine, q, false, true);
      ge_p3_to_cached(c1, PB);
      if (half == 0 && role == 0) sv_store_lentry((sv_u4*)&s_pb[sl][0], c1);
    }
    if (HI) sv_oflag_set(&s_oflag[SV_OF_PB], dig_good);
    else __syncthreads();  // s_pb written
    return;
  }
  ok = sc_is_canonical(S) && !sv_small_order(R) && sv_point_canonical(A) && !sv_small_order(A) &&
       sv_point_canonical(R);
  sv_lat lat;
  {
    uint32_t h[8];
    sc_reduce512(h, hram);
    sc_lattice_reduce(lat, h, (p.dbg & SV_DBG_TRIVIAL_PAIR) != 0);
  }
  const int W = sv_wave_windows(sv_lat_windows(lat.bits), p.dbg);
  sv_lat_digits D;
  sv_lat_prepare(D, lat, S, W);
  // (HI: this wave runs windows Wlo-1 .. 0, the high wave the rest)
  const int Wlo = HI ? W - sv_oct_hi_windows(W, p.dbg) : W;
  if (role == 0) {
    SV_UNROLL for (int j = 0; j < SV_LB_DIGITS; ++j) s_bd[sl][half][j] = half ? D.dB1[j] : D.dB0[j];
    if (HI) {
      SV_UNROLL for (int k = 0; k < 8; ++k) s_hd[sl][half][k] = half ? D.dR[k] : D.dA[k];
      s_hd[sl][half][8] = ((half ? D.top8R : D.top8A) ? 1u : 0u) | ((half && D.rneg) ? 2u : 0u);
    }
  }
  if (HI && lane == 0) {
    s_win[0] = W;
    s_win[1] = Wlo;
  }
  bool handed = true;  // (HI: every hand-over wave 0 waits for arrived)
  if (HI) {
    sv_oflag_set(&s_oflag[SV_OF_DIG]);             // digits and the split
    handed = sv_oflag_wait(&s_oflag[SV_OF_TAB]);  // the tables
  } else {
    __syncthreads();  // tables visible to the whole quad
  }
  ok = ok && s_dok[sl] != 0;

  const uint32_t* tab = &s_tab[sl][half][0][0];
  // this quad's digit string and its top-digit carry
  uint32_t dg[8];
  SV_UNROLL for (int k = 0; k < 8; ++k) dg[k] = half ? D.dR[k] : D.dA[k];
  const bool top8 = half ? D.top8R : D.top8A;
  const bool flip = half && D.rneg;
  // own form (quad.h): lane r holds coordinate r of P until the end
  fe h;
  qo_identity(h, q);
  SV_NOUNROLL for (int k = 0; k < W - Wlo; ++k) (void)sc_pop_top(dg, 4);  // (the high wave's digits)
  SV_NOUNROLL for (int w = Wlo - 1; w >= 0; --w) {
    int32_t d = sc_pop_top(dg, 4);
    if (w == W - 1 && top8) d = 8;
    if (flip) d = -d;
    const bool bwin = false;  // (the base part runs on wave 1)
    const int32_t dB = 0;
    fe b;
    if (w != Wlo - 1) {
      SV_NOUNROLL for (int k = 0; k < 4; ++k) qo_dbl(h, q);
    }
    fe m;
    qo_load_cached(m, tab + (d < 0 ? -d : d) * SV_QENT_DW, role, d < 0);
    qo_add(h, m, q, d < 0);
    if (bwin) qo_add(h, b, q, dB < 0);
  }
  ge_p3 P;
  qo_expand(P, h);
  // quad 0: P_A + P_R, P_R in cached form from quad 1
  {
    if (HI) {
      handed = sv_oflag_wait(&s_oflag[SV_OF_PHI]) && handed;  // the high parts from wave 2
      fe mh;
      qd_load_cached(mh, &s_phi[sl][half][0], role, false);
      qd_add(P, mh, q, false, true);  // this quad's low + high part
    }
    ge_p3 PR;
    fe_from_hi(PR.X, P.X);
    fe_from_hi(PR.Y, P.Y);
    fe_from_hi(PR.Z, P.Z);
    fe_from_hi(PR.T, P.T);
    fe d2, t2d, ypx, ymx, mine;
    fe_const_2d(d2);
    fe_mul(t2d, PR.T, d2);
    fe_add(ypx, PR.Y, PR.X);
    fe_sub(ymx, PR.Y, PR.X);
    fe_pick4(mine, q, t2d, PR.Z, ypx, ymx);  // role 0 2dT, 1 Z, 2 Y+X, 3 Y-X (qd_add's operand order)
    qd_add(P, mine, q, false, true);
    if (HI) handed = sv_oflag_wait(&s_oflag[SV_OF_PB]) && handed;  // [s]B from wave 1
    else __syncthreads();
    qd_load_cached(mine, &s_pb[sl][0], role, false);
    qd_add(P, mine, q, false, false);
  }
  ok = ok && handed && sv_is_identity(P);
  // a lost hand-over: the rejects below are fail-closed placeholders, and the
  // launch's failure word tells the host so (one plain store per workgroup;
  // every writer stores the same code)
  if (HI && !handed && p.status != nullptr && lane == 0) *(volatile uint32_t*)p.status = SV_KFAIL_HANDOVER;
  const bool owner = half == 0 && role == 0;
  if (active && owner) p.verdict[i] = ok ? 1 : 0;
  const uint64_t bal = __ballot(ok && active && owner);
  if (p.bitmap != nullptr && lane == 0) {
    uint8_t m8 = 0;
    SV_UNROLL for (int k = 0; k < SV_OSIGS; ++k) m8 |= (uint8_t)(((bal >> (8 * k)) & 1u) << k);
    ((uint8_t*)p.bitmap)[blockIdx.x] = m8;
    // the last workgroup clears the rest of the final 64-bit word, as the
    // throughput path's whole-word ballots do (bits past n read as 0)
    if (blockIdx.x == gridDim.x - 1)
      for (uint32_t b = blockIdx.x + 1; b % 8 != 0; ++b) ((uint8_t*)p.bitmap)[b] = 0;
  }
}

// ------------------------------------------- medium batches: one signature per quad
// Between the latency path and full throughput, a batch of n signatures gives
// the one-lane kernels n / 64 waves: under one per SIMD up to 64k signatures,
// each at a lone wave's serial latency (the one-lane prep + main stream of a
// wave is ~0.3M instructions).  Here a QUAD of lanes evaluates one
// signature's whole half-size equation (*) (lattice.h), 16 signatures per
// wave and 4x the waves, each with a ~3x shorter instruction stream:
//   * all four lanes load, hash, check and run the Euclid reduction (one
//     instruction stream whatever the number of lanes: free in latency);
//   * lanes 0 / 2 decode -A while lanes 1 / 3 decode -R (the same code);
//   * the quad builds both 9-entry tables with quad-split additions (qd_add)
//     into the chunk workspace, each lane storing (and later reading) only
//     its own operands;
//   * the throughput path's joint chain (4 doublings, the -A and -R entries,
//     on base windows the e B and e 2^128 B entries) runs in own form
//     (quad.h), each window's entries loaded before its doublings.
// Same field operations, bounds and decisions as the one-lane path, so the
// verdicts are identical (every fixture class is GPU-tested on it).
#define SV_QSIGS 16
// A table entry holds each lane's operands in a region of its own, so every
// lane only ever reads back what it wrote itself (no cross-lane memory
// ordering inside the wave): lane 0 (Y+X, Y-X), lane 1 (Y-X, Y+X) -- the pair
// read straight or swapped by a digit's sign, qo_load_cached's roles -- lane 2
// Z, lane 3 2dT.  60 dwords per entry, 2 x 9 entries per signature.
#define SV_QENT 60
#define SV_QSLOT_QUADS (2 * SV_ATAB_ENTRIES * SV_QENT / 4)
__device__ __forceinline__ uint32_t qd_swap1(uint32_t v) {  // lane r ^ 1 of the quad
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t sv_qoff(uint32_t role) { return role < 2 ? 20u * role : 40u + 10u * (role - 2); }
__device__ __forceinline__ void sv_qst10(uint32_t* d, const fe& x) {
  uint2* p = (uint2*)d;
  SV_UNROLL for (int k = 0; k < 5; ++k) p[k] = uint2{x.v[2 * k], x.v[2 * k + 1]};
}
// this lane's operands of cached entry c into table entry `ent`
__device__ __forceinline__ void sv_qstore(uint32_t* ent, const ge_cached& c, const qd_role& q, uint32_t role) {
  fe x, y;
  fe_pick4(x, q, c.YpX, c.YmX, c.Z, c.T2d);  // the operand read straight ...
  fe_pick4(y, q, c.YmX, c.YpX, c.Z, c.T2d);  // ... and swapped (roles 0, 1)
  uint32_t* d = ent + sv_qoff(role);
  sv_qst10(d, x);
  if (role < 2) sv_qst10(d + 10, y);
}
// this lane's operand of entry `ent` with a digit's sign (qo_load_cached's)
__device__ __forceinline__ void sv_qload(fe& o, const uint32_t* ent, uint32_t role, bool neg) {
  const uint2* p = (const uint2*)(ent + sv_qoff(role) + (role < 2 && neg ? 10u : 0u));
  SV_UNROLL for (int k = 0; k < 5; ++k) {
    const uint2 v = p[k];
    o.v[2 * k] = v.x;
    o.v[2 * k + 1] = v.y;
  }
}
// {0..8}(P) in cached form, P affine (ge_frombytes) and whole on every lane
__device__ __forceinline__ void sv_qbuild(uint32_t* tab, const ge_p3& P, const qd_role& q, uint32_t role) {
  ge_cached c1, ce;
  ge_p3_to_cached(c1, P);
  ge_cached_identity(ce);
  sv_qstore(tab, ce, q, role);
  sv_qstore(tab + SV_QENT, c1, q, role);
  fe mine;
  fe_pick4(mine, q, c1.T2d, c1.Z, c1.YpX, c1.YmX);  // (qd_add's operand order)
  ge_p3 P3 = P;
  SV_NOUNROLL for (int e = 2; e < SV_ATAB_ENTRIES; ++e) {
    qd_add(P3, mine, q, false, true);
    ge_p3_to_cached(ce, P3);
    sv_qstore(tab + e * SV_QENT, ce, q, role);
  }
}
template <int MODE, bool MSG>
__global__ __launch_bounds__(64, SV_QUAD_WAVES) void sv_quad_kernel(sv_kparams p) {
  __shared__ sv_u4 s_msg[MSG ? SV_QSIGS * (SV_MSG_CAP / 16) : 1];
  if (p.dbg & SV_KP_LAT) __builtin_amdgcn_s_setprio(3);  // (on the latency lane: as the octet / comb kernels)
  const uint32_t lane = threadIdx.x;
  const uint32_t role = lane & 3u, sq = lane >> 2;
  const qd_role q{role == 1, role == 2, role == 3};
  const uint64_t i = (uint64_t)blockIdx.x * SV_QSIGS + sq;
  const bool active = i < p.n;
  const uint64_t ii = active ? i : p.n - 1;  // idle tail quads redo the last item (own slots)
  uint32_t A[8], S[8], hram[16], R[8];
  bool ok = true;
  sv_lat lat;
  sv_lat_digits D;
  int W = 0;
  // checks, scalar and lattice reduction, digits (after the hash)
  auto prologue = [&]() {
    ok = ok && sc_is_canonical(S) && !sv_small_order(R) && sv_point_canonical(A) && !sv_small_order(A) &&
         sv_point_canonical(R);
    {
      uint32_t h[8];
      sc_reduce512(h, hram);
      sc_lattice_reduce(lat, h, (p.dbg & SV_DBG_TRIVIAL_PAIR) != 0);
    }
    W = sv_wave_windows(sv_lat_windows(lat.bits), p.dbg);
    sv_lat_prepare(D, lat, S, W);
  };
  if (MSG) {
    sv_load_and_hash_lds<MODE, 4>(p, ii, role, s_msg + sq * (SV_MSG_CAP / 16), A, S, hram);
    sv_unpack2(R, p.sig + 4 * ii);
    prologue();
  } else {
    // A and R only: the decode below needs nothing else, so a batch read in
    // place from host memory starts computing once half of its bytes are
    // across PCIe; S and the message follow after the decode, with the hash
    sv_unpack2(A, p.pk + 2 * ii);
    sv_unpack2(R, p.sig + 4 * ii);
  }
  // decode: lanes 0, 2 -A, lanes 1, 3 -R; then both tables on the whole quad
  uint32_t* tabA = (uint32_t*)(p.ws + i * SV_QSLOT_QUADS);
  uint32_t* tabR = tabA + SV_ATAB_ENTRIES * SV_QENT;
  {
    uint32_t E[8];
    SV_UNROLL for (int k = 0; k < 8; ++k) E[k] = (role & 1u) ? R[k] : A[k];
    ge_p3 Pt;
    const uint32_t dk = ge_frombytes(Pt, E, true) ? 1u : 0u;
    ok = ok && (dk & qd_swap1(dk)) != 0;
    ge_p3 Pq;
    fe_from<0>(Pq.X, Pt.X);
    fe_from<0>(Pq.Y, Pt.Y);
    fe_from<0>(Pq.Z, Pt.Z);
    fe_from<0>(Pq.T, Pt.T);
    sv_qbuild(tabA, Pq, q, role);
    fe_from<1>(Pq.X, Pt.X);
    fe_from<1>(Pq.Y, Pt.Y);
    fe_from<1>(Pq.Z, Pt.Z);
    fe_from<1>(Pq.T, Pt.T);
    sv_qbuild(tabR, Pq, q, role);
  }
  if (!MSG) {
    sv_unpack2(S, p.sig + 4 * ii + 2);
    if (MODE == 0) {
      uint32_t M[8];
      sv_unpack2(M, (const sv_u4*)(p.msg) + 2 * ii);
      sha512_ram32(hram, R, A, M);
    } else if (MODE == 1) {
      sha512_ram_var(hram, R, A, p.msg + p.msg_off[ii], p.msg_len[ii]);
    } else {
      sha512_ram_var(hram, R, A, p.msg + ii * (uint64_t)p.fixed_len, p.fixed_len);
    }
    prologue();
  }
  const sv_u4* btab0 = p.btab;
  const sv_u4* btab1 = p.btab + SV_LBTAB_ENTRIES * SV_BTAB_QUADS;
  fe h;
  qo_identity(h, q);
  SV_NOUNROLL for (int w = W - 1; w >= 0; --w) {
    int32_t dA = sc_pop_top(D.dA, 4), dR = sc_pop_top(D.dR, 4);
    if (w == W - 1) {
      if (D.top8A) dA = 8;
      if (D.top8R) dR = 8;
    }
    if (D.rneg) dR = -dR;
    int32_t dB0, dB1;
    const bool bwin = sv_lat_bdigits(D, w, dB0, dB1);
    // the window's entries, loaded before its doublings
    fe ma, mr, m0;
    sv_qload(ma, tabA + (dA < 0 ? -dA : dA) * SV_QENT, role, dA < 0);
    sv_qload(mr, tabR + (dR < 0 ? -dR : dR) * SV_QENT, role, dR < 0);
    if (bwin) qo_load_affine(m0, btab0 + (dB0 < 0 ? -dB0 : dB0) * SV_BTAB_QUADS, role, dB0 < 0);
    if (w != W - 1) {
      SV_NOUNROLL for (int k = 0; k < 4; ++k) qo_dbl(h, q);
    }
    qo_add(h, ma, q, dA < 0);
    if (bwin) qo_load_affine(ma, btab1 + (dB1 < 0 ? -dB1 : dB1) * SV_BTAB_QUADS, role, dB1 < 0);
    qo_add(h, mr, q, dR < 0);
    if (bwin) {
      qo_add(h, m0, q, dB0 < 0);
      qo_add(h, ma, q, dB1 < 0);
    }
  }
  ge_p3 P;
  qo_expand(P, h);
  ok = ok && sv_is_identity(P);
  const bool owner = role == 0;
  if (active && owner) p.verdict[i] = ok ? 1 : 0;
  const uint64_t bal = __ballot(ok && active && owner);
  if (p.bitmap != nullptr && lane == 0) {
    uint32_t m16 = 0;
    SV_UNROLL for (int k = 0; k < SV_QSIGS; ++k) m16 |= (uint32_t)((bal >> (4 * k)) & 1u) << k;
    ((uint16_t*)p.bitmap)[blockIdx.x] = (uint16_t)m16;
    // the last workgroup clears the rest of the final 64-bit word (bits past n read as 0)
    if (blockIdx.x == gridDim.x - 1)
      for (uint32_t b = blockIdx.x + 1; b % 4 != 0; ++b) ((uint16_t*)p.bitmap)[b] = 0;
  }
}

__global__ __launch_bounds__(192) void sv_btab_init_kernel(uint32_t* btab) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  // table 0: e B (also the signer's table: it reads entries <= 2^(SV_B_BITS-1));
  // table 1: e 2^128 B
  if (e < SV_LBTAB_ENTRIES) sv_btab_entry_shift(btab + e * SV_BTAB_STRIDE, e, 0);
  else if (e < 2 * SV_LBTAB_ENTRIES)
    sv_btab_entry_shift(btab + e * SV_BTAB_STRIDE, e - SV_LBTAB_ENTRIES, 128);
}

struct sv_sparams {
  const sv_u4* seed;  // n x 32 B
  const sv_u4* msg;   // n x 32 B
  uint64_t n;
  sv_u4* pk;          // n x 32 B out
  sv_u4* sig;         // n x 64 B out
  sv_u4* ws;
  const sv_u4* btab;
};

__global__ __launch_bounds__(SV_BLOCK, SV_WAVES_PER_SIMD) void sv_sign_kernel(sv_sparams p) {
  const sv_u4* s_btab = p.btab;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t gtid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  sv_u4* slot = p.ws + gtid * SV_SLOT_QUADS;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = gtid - lane; base < p.n; base += stride) {
    const uint64_t i = base + lane;
    const bool active = i < p.n;
    const uint64_t ii = active ? i : p.n - 1;
    uint32_t seed[8], M[8], pk[8], sig[16];
    sv_unpack2(seed, p.seed + 2 * ii);
    sv_unpack2(M, p.msg + 2 * ii);
    sv_sign_lane(pk, sig, seed, M, slot, 1, s_btab);
    if (active) {
      p.pk[2 * i] = sv_u4{pk[0], pk[1], pk[2], pk[3]};
      p.pk[2 * i + 1] = sv_u4{pk[4], pk[5], pk[6], pk[7]};
      SV_UNROLL for (int q = 0; q < 4; ++q)
        p.sig[4 * i + q] = sv_u4{sig[4 * q], sig[4 * q + 1], sig[4 * q + 2], sig[4 * q + 3]};
    }
  }
}

// ------------------------------------------------------------ launchers
extern "C" {

#ifdef SV_PHASE_PROF
int sv_debug_phase_cycles(unsigned long long out[8], int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sv_phase_cycles), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(sv_phase_cycles), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

#ifdef SV_MADCOUNT
// (measurement builds: the field-product multiply-adds issued since the last reset)
int sv_debug_madcount(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sv_madcount), sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(sv_madcount), &z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

size_t sv_ws_bytes_per_block(void) { return (size_t)SV_BLOCK * SV_SLOT_QUADS * sizeof(sv_u4); }

// ------------------------------------------------- chunk planner (split path)
// sv_main_kernel is persistent: Cm = CUs x blocks/CU x 4 resident waves, each
// walking 64-signature groups with stride Cm, so a chunk of g groups runs
// floor(g / Cm) full rounds and a last round of g mod Cm waves, dispatched one
// block per CU first: d = ceil((g mod Cm) / SIMDs) waves per SIMD.  A SIMD
// with fewer waves issues less per cycle (a wave's dependent issue leaves
// gaps), measured on MI355X (profiles/r02/ab_chunk.txt): relative throughput
// 0.55 with one wave, 0.97 with two, against the main kernel's three.  So a
// 2^20 batch in one chunk (16384 groups = 5 rounds + a last round of one wave
// per SIMD) loses ~4 % against two chunks of 8192 (2 rounds + two waves per
// SIMD each).  The planner splits a launch into k equal chunks (k from the
// workspace bound up) minimising the modelled time of both kernels.
static double sv_rounds(uint64_t g, uint64_t simds, int wps) {
  const uint64_t C = simds * (uint64_t)wps;
  const uint64_t full = g / C, rem = g % C;
  double t = (double)full;
  if (rem) {
    const uint64_t d = (rem + simds - 1) / simds;  // waves per SIMD in the last round
    const double eff = d >= (uint64_t)wps ? 1.0 : (d == 1 ? 0.55 : 0.97);
    t += (double)d / ((double)wps * eff);
  }
  return t;
}
// resident waves per SIMD of a kernel (occupancy API; cached, benign races)
static int sv_wps(const void* kernel, std::atomic<int>& cache) {
  int w = cache.load(std::memory_order_relaxed);
  if (w == 0) {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, SV_BLOCK, 0) != hipSuccess || b < 1) b = 1;
    w = b * (SV_BLOCK / 64) / 4;
    if (w < 1) w = 1;
    cache.store(w, std::memory_order_relaxed);
  }
  return w;
}
static std::atomic<int> g_main_wps{0}, g_prep_wps{0};
static int sv_main_wps(void) { return sv_wps((const void*)sv_main_kernel<false>, g_main_wps); }
static int sv_prep_wps(void) { return sv_wps((const void*)sv_prep_kernel<0, false, false>, g_prep_wps); }
// Shared mode (sv_launch_verify `share`): while latency-class batches are
// live on the device, the throughput kernels leave one workgroup slot per CU
// free for them -- the persistent main kernel runs one block per CU fewer
// (the caller's grid) and each prep launch asks for enough dynamic LDS that
// one block fewer fits per CU -- so a latency kernel (sv_comb_kernel<.,1>:
// 146 VGPRs, 17 KB LDS; sv_octet_kernel: 166 VGPRs, 25 KB) is dispatched as
// soon as it is queued instead of after a whole bulk chunk.
static int sv_share_wps(int w) { return w > 1 ? w - 1 : 1; }
static std::atomic<int> g_lds_cu{0};
static size_t sv_prep_share_lds(void) {
  int v = g_lds_cu.load(std::memory_order_relaxed);
  if (v == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess || v < 1)
      v = 160 * 1024;
    g_lds_cu.store(v, std::memory_order_relaxed);
  }
  const int w = sv_share_wps(sv_prep_wps());  // blocks per CU wanted
  size_t b = (size_t)v / (size_t)(w + 1) + 256;  // w + 1 blocks no longer fit
  b = (b + 255) & ~(size_t)255;
  return b > 65536 ? 65536 : b;
}
// Shared mode for the quad kernel (one-wave workgroups, SV_QUAD_WAVES per
// SIMD): dynamic LDS such that at most 4 (SV_QUAD_WAVES - 1) fit per CU and
// 32 KiB of LDS stay free, which leaves a latency workgroup room on each CU.
static size_t sv_quad_share_lds(void) {
  int v = g_lds_cu.load(std::memory_order_relaxed);
  if (v == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess || v < 1)
      v = 160 * 1024;
    g_lds_cu.store(v, std::memory_order_relaxed);
  }
  const int blocks = 4 * (SV_QUAD_WAVES > 1 ? SV_QUAD_WAVES - 1 : 1);
  size_t b = ((size_t)v - 32 * 1024) / (size_t)blocks;
  b &= ~(size_t)255;
  return b > 65536 ? 65536 : b;
}
// SIMDs of the current device (4 per CU)
static std::atomic<int> g_cus[64];
static uint64_t sv_device_simds(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  int c = g_cus[dev].load(std::memory_order_relaxed);
  if (c == 0) {
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1) return 0;
    g_cus[dev].store(c, std::memory_order_relaxed);
  }
  return 4u * (uint64_t)c;
}
// Signatures per chunk for a throughput-path launch of n on the current
// device (every chunk but the last has exactly this many; a multiple of 64,
// at most SV_CHUNK).
uint64_t sv_plan_chunk(uint64_t n, int share) {
  const uint64_t G = (n + 63) / 64;
  const uint64_t capG = SV_CHUNK / 64;
  const int mw = share ? sv_share_wps(sv_main_wps()) : sv_main_wps();
  const int pw = share ? sv_share_wps(sv_prep_wps()) : sv_prep_wps();
  const uint64_t simds = sv_device_simds();
  if (G == 0 || simds == 0) return SV_CHUNK;
  const uint64_t kmin = (G + capG - 1) / capG;
  // per-group costs: main round of Cm groups vs prep round of Cp groups, in
  // main-group units (MI355X: 0.45 us vs 0.17 us per group); launch pair ~ 20
  const double kPrep = 0.38, kLaunch = 20.0;
  uint64_t best_k = kmin;
  double best = 0.0;
  for (uint64_t k = kmin; k <= 2 * kmin + 4 && k <= G; ++k) {
    const uint64_t g = (G + k - 1) / k, last = G - (k - 1) * g;
    if (last == 0 || last > g) continue;
    const double one = sv_rounds(g, simds, mw) * (double)(simds * mw) +
                       kPrep * sv_rounds(g, simds, pw) * (double)(simds * pw);
    const double tail = sv_rounds(last, simds, mw) * (double)(simds * mw) +
                        kPrep * sv_rounds(last, simds, pw) * (double)(simds * pw);
    const double t = (double)(k - 1) * one + tail + kLaunch * (double)k;
    if (k == kmin || t < best * 0.999) {
      best = t;
      best_k = k;
    }
  }
  const uint64_t g = (G + best_k - 1) / best_k;
  return g * 64 < SV_CHUNK ? g * 64 : SV_CHUNK;
}

// Signatures one throughput-path launch sequence processes per prep/main
// chunk (sv_plan_chunk): the workspace of a batch of n holds ws_cap(n) of them,
// rounded up to whole workgroups.
uint64_t sv_ws_cap(uint64_t n) {
  const uint64_t p0 = sv_plan_chunk(n, 0), p1 = sv_plan_chunk(n, 1);
  const uint64_t p = p0 > p1 ? p0 : p1;  // (either mode may run on one workspace)
  const uint64_t c = n < p ? n : p;
  return (c + SV_BLOCK - 1) / SV_BLOCK * SV_BLOCK;
}
// Device workspace for `grid` persistent workgroups (fused verify kernel,
// signer: per-lane slots) and, split, a chunk of `cap` signatures (tables +
// digit records + window counts).  The latency kernel needs none.
size_t sv_ws_bytes(unsigned grid, uint64_t cap) {
  size_t b = (size_t)grid * sv_ws_bytes_per_block();
  const size_t s = (size_t)cap * (SV_SLOT_QUADS_L + SV_REC_QUADS) * sizeof(sv_u4) + (cap / 64) * 4;
  if (s > b) b = s;
  return b;
}
// workspace a verify launch of n signatures on `path` needs
size_t sv_verify_ws_bytes(int path, unsigned grid, uint64_t n) {
  if (path == 2) return 0;
  (void)grid;
  if (path == 3) return (size_t)((n + SV_QSIGS - 1) / SV_QSIGS * SV_QSIGS) * SV_QSLOT_QUADS * sizeof(sv_u4);
  return sv_ws_bytes(0, sv_ws_cap(n));
}
#define SV_BTAB_TOTAL (2 * SV_LBTAB_ENTRIES)
size_t sv_btab_bytes(void) { return (size_t)SV_BTAB_TOTAL * SV_BTAB_STRIDE * 4; }
int sv_block_threads(void) { return SV_BLOCK; }

hipError_t sv_launch_btab_init(uint32_t* d_btab, hipStream_t s) {
  hipLaunchKernelGGL(sv_btab_init_kernel, dim3((SV_BTAB_TOTAL + 191) / 192), dim3(192), 0, s, d_btab);
  return hipGetLastError();
}

int sv_occupancy_blocks_per_cu(void) {
  int b0 = 0, b1 = 0, b2 = 0, b3 = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b0, sv_main_kernel<false>, SV_BLOCK, 0) != hipSuccess) b0 = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b3, sv_sign_kernel, SV_BLOCK, 0) != hipSuccess) b3 = 1;
  const int ms = b0 > b3 ? b0 : b3;
  (void)b1;
  (void)b2;
  return ms < 1 ? 1 : ms;
}

size_t sv_key_table_entry_bytes(void) { return (size_t)SV_KT_QUADS * sizeof(sv_u4); }
uint64_t sv_plan_chunk_max(uint64_t n) { return sv_ws_cap(n); }

// Blocks per CU of the persistent main kernel in shared mode.
int sv_share_blocks_per_cu(void) { return sv_share_wps(sv_main_wps()) * 4 / (SV_BLOCK / 64); }

// ws must hold sv_verify_ws_bytes(path, grid, n) bytes.  share: shared mode
// (above); the caller's grid is then CUs x sv_share_blocks_per_cu().  kt
// (optional): per-key tables (above); kt->kslot / kt->builders hold
// sv_plan_chunk(n) entries, kt->count 2.
hipError_t sv_launch_verify(int mode, int path, unsigned grid, const void* pk, const void* sig, const void* msg,
                            const uint64_t* off, const uint32_t* len, uint32_t fixed_len, uint64_t n,
                            void* verdict, void* bitmap, void* ws, const void* btab, uint32_t dbg, int share,
                            const sv_ktparams* kt, uint32_t* status, hipStream_t s) {
  sv_kparams p;
  p.status = status;
  p.pk = (const sv_u4*)pk;
  p.sig = (const sv_u4*)sig;
  p.msg = (const uint8_t*)msg;
  p.msg_off = off;
  p.msg_len = len;
  p.n = n;
  p.fixed_len = fixed_len;
  p.verdict = (uint8_t*)verdict;
  p.bitmap = (uint64_t*)bitmap;
  p.ws = (sv_u4*)ws;
  p.btab = (const sv_u4*)btab;
  p.dbg = dbg;
  if (path == 2) {  // SV_PATH_LATENCY
    const unsigned og = (unsigned)((n + SV_OSIGS - 1) / SV_OSIGS);
    const bool msg = og <= sv_device_simds() / 4;
    const bool hi = (dbg & SV_KP_OCT_HI) != 0;
#define SV_OCTET_LAUNCH(M, G, H)                                                                            \
  hipLaunchKernelGGL((sv_octet_kernel<M, G, H>), dim3(og), dim3((H) ? SV_OCTET_BLOCK_HI : SV_OCTET_BLOCK), \
                     SV_OCTET_LDS_BYTES(G, H), s, p)
#define SV_OCTET_LAUNCH2(M, G) \
  do {                          \
    if (hi) SV_OCTET_LAUNCH(M, G, true); \
    else SV_OCTET_LAUNCH(M, G, false);   \
  } while (0)
    if (mode == 0) SV_OCTET_LAUNCH2(0, false);  // (32-byte messages: no window)
    else if (mode == 1 && msg) SV_OCTET_LAUNCH2(1, true);
    else if (mode == 1) SV_OCTET_LAUNCH2(1, false);
    else if (msg) SV_OCTET_LAUNCH2(2, true);
    else SV_OCTET_LAUNCH2(2, false);
#undef SV_OCTET_LAUNCH2
#undef SV_OCTET_LAUNCH
    return hipGetLastError();
  }
  if (path == 3) {  // the throughput path's medium-batch geometry (sv_quad_kernel)
    const unsigned qg = (unsigned)((n + SV_QSIGS - 1) / SV_QSIGS);
    const bool msg = mode != 0;
    const size_t qlds = share ? sv_quad_share_lds() : 0;
#define SV_QUAD_LAUNCH(M, G) hipLaunchKernelGGL((sv_quad_kernel<M, G>), dim3(qg), dim3(64), qlds, s, p)
    if (mode == 0) SV_QUAD_LAUNCH(0, false);
    else if (mode == 1 && msg) SV_QUAD_LAUNCH(1, true);
    else SV_QUAD_LAUNCH(2, true);
#undef SV_QUAD_LAUNCH
    return hipGetLastError();
  }
  const uint64_t cap = sv_ws_cap(n);
  const uint64_t chunk = sv_plan_chunk(n, share);
  const size_t plds = share ? sv_prep_share_lds() : 0;
  sv_u4* rec = p.ws + (size_t)cap * SV_SLOT_QUADS_L;
  uint32_t* wmax = (uint32_t*)(rec + (size_t)cap * SV_REC_QUADS);
  for (uint64_t start = 0; start < n; start += chunk) {
    sv_cparams c;
    c.k = p;
    c.start = start;
    c.cnt = n - start < chunk ? n - start : chunk;
    c.rec = rec;
    c.wmax = wmax;
    c.kt = kt ? *kt : sv_ktparams{};
    const unsigned pg = (unsigned)((c.cnt + SV_BLOCK - 1) / SV_BLOCK);
    if (kt) {
      const hipError_t e = hipMemsetAsync(kt->count, 0, sizeof(uint32_t), s);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(sv_keyslot_kernel, dim3(pg), dim3(SV_BLOCK), 0, s, c);
      hipLaunchKernelGGL(sv_keybuild_kernel, dim3(pg), dim3(SV_BLOCK), 0, s, c);
    }
#define SV_PREP_LAUNCH(M, K, F) hipLaunchKernelGGL((sv_prep_kernel<M, K, F>), dim3(pg), dim3(SV_BLOCK), plds, s, c)
    if (kt) {
      if (mode == 0) SV_PREP_LAUNCH(0, true, false);
      else if (mode == 1) SV_PREP_LAUNCH(1, true, false);
      else SV_PREP_LAUNCH(2, true, false);
    } else if (dbg & SV_KP_IN_PLACE) {
      if (mode == 0) SV_PREP_LAUNCH(0, false, true);
      else if (mode == 1) SV_PREP_LAUNCH(1, false, true);
      else SV_PREP_LAUNCH(2, false, true);
    } else {
      if (mode == 0) SV_PREP_LAUNCH(0, false, false);
      else if (mode == 1) SV_PREP_LAUNCH(1, false, false);
      else SV_PREP_LAUNCH(2, false, false);
    }
#undef SV_PREP_LAUNCH
    if (!(dbg & SV_DBG_PREP_ONLY)) {
      const dim3 mg(grid < pg ? grid : pg);
      if (kt) hipLaunchKernelGGL(sv_main_kernel<true>, mg, dim3(SV_BLOCK), 0, s, c);
      else hipLaunchKernelGGL(sv_main_kernel<false>, mg, dim3(SV_BLOCK), 0, s, c);
    }
  }
  return hipGetLastError();
}

hipError_t sv_launch_sign(unsigned grid, const void* seed, const void* msg, uint64_t n, void* pk, void* sig,
                          void* ws, const void* btab, hipStream_t s) {
  sv_sparams p;
  p.seed = (const sv_u4*)seed;
  p.msg = (const sv_u4*)msg;
  p.n = n;
  p.pk = (sv_u4*)pk;
  p.sig = (sv_u4*)sig;
  p.ws = (sv_u4*)ws;
  p.btab = (const sv_u4*)btab;
  hipLaunchKernelGGL(sv_sign_kernel, dim3(grid), dim3(SV_BLOCK), 0, s, p);
  return hipGetLastError();
}

}  // extern "C"
