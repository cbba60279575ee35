// Verify-launch parameters and the per-signature input loader shared by the
// kernel translation units (sv_kernels.hip, sv_comb.hip).
#pragma once

#include "keytab.h"
#include "verify_core.h"

struct sv_kparams {
  const sv_u4* pk;        // n x 32 B (2 quads)
  const sv_u4* sig;       // n x 64 B (4 quads)
  const uint8_t* msg;     // fixed: n x fixed_len ; var: msg bytes
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  uint64_t n;
  uint32_t fixed_len;     // 0 = variable-length
  uint8_t* verdict;       // n bytes
  uint64_t* bitmap;       // optional, ceil(n/64) words
  sv_u4* ws;              // workspace: grid threads x SV_SLOT_QUADS (lane-major)
  const sv_u4* btab;      // SV_BTAB_ENTRIES x 9 quads (global copy)
  uint32_t dbg;           // SV_DBG_* test knobs (sv_set_debug_flags), 0 in production; + SV_KP_LAT (keytab.h)
  // optional (nullptr: none): the launch's failure word.  A kernel that cannot
  // stand behind its verdicts (the three-wave octet kernel after a hand-over
  // wait ran out) writes a nonzero SV_KFAIL_* code here; the host, which zeroed
  // it before the launch, then returns an error for the whole batch instead of
  // the (fail-closed) rejects: an error is never a reject
  // (include/stellar_sigverify.h; /root/reference/src/crypto/SecretKey.cpp:461-466
  // caches every verdict it is given).
  uint32_t* status;
};
#define SV_KFAIL_HANDOVER 1u  // sv_octet_kernel<., ., HI>: a hand-over flag never came

__device__ __forceinline__ void sv_unpack2(uint32_t w[8], const sv_u4* p) {
  const sv_u4 a = p[0], b = p[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// Loads one signature's inputs and hashes R || A || M (step (6)).
// MODE 0: fixed 32-byte messages, 1: variable length, 2: fixed other length.
template <int MODE>
__device__ __forceinline__ void sv_load_and_hash(const sv_kparams& p, uint64_t ii, uint32_t A[8], uint32_t S[8],
                                                 uint32_t hram[16]) {
  uint32_t R[8];
  sv_unpack2(A, p.pk + 2 * ii);
  sv_unpack2(R, p.sig + 4 * ii);
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
}

// The rest of a signature's inputs once A and R are loaded (the decode-first
// order of sv_prep_kernel<., ., DF>): S, then the message, and R || A || M
// hashed.
template <int MODE>
__device__ __forceinline__ void sv_load_rest_and_hash(const sv_kparams& p, uint64_t ii, const uint32_t A[8],
                                                      const uint32_t R[8], uint32_t S[8], uint32_t hram[16]) {
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
}

// The latency kernels' loader (sv_comb_kernel chain waves, sv_octet_kernel
// hash wave).  Their input image lives in mapped host memory (the lane reads
// it in place), where every dependent round trip costs ~2 us: a message read
// word by word inside the SHA-512 blocks pays one per block.  Here the LPS
// lanes of a signature first copy the 16-byte-aligned window holding its
// message into LDS (lbuf, SV_MSG_CAP bytes; one 16-byte load per lane per
// LPS * 16 bytes), so the message costs one round trip after the offset's,
// and the hash reads LDS.  A longer message is hashed from memory as before.
#define SV_MSG_CAP 512
template <int MODE, int LPS>
__device__ __forceinline__ void sv_load_and_hash_lds(const sv_kparams& p, uint64_t ii, uint32_t li, sv_u4* lbuf,
                                                     uint32_t A[8], uint32_t S[8], uint32_t hram[16]) {
  if (MODE == 0) {  // (32-byte messages come with R, A and S in one round trip)
    sv_load_and_hash<0>(p, ii, A, S, hram);
    return;
  }
  uint32_t R[8];
  sv_unpack2(A, p.pk + 2 * ii);
  sv_unpack2(R, p.sig + 4 * ii);
  sv_unpack2(S, p.sig + 4 * ii + 2);
  const uint8_t* mp = MODE == 1 ? p.msg + p.msg_off[ii] : p.msg + ii * (uint64_t)p.fixed_len;
  const uint32_t mlen = MODE == 1 ? p.msg_len[ii] : p.fixed_len;
  // (an aligned 16-byte block never crosses a page: reading the whole first
  // and last block of the message stays inside mapped memory)
  const uint32_t lead = (uint32_t)((uintptr_t)mp & 15u);
  const uint32_t nq = (lead + mlen + 15u) >> 4;
  const bool fits = nq <= SV_MSG_CAP / 16;
  if (fits && nq > 0) {
    // every load of the window first (unpredicated: an index past the window
    // re-reads its last quad), then the LDS writes: a load-then-write loop
    // waits out one round trip per iteration (up to SV_MSG_CAP / 16 / LPS of
    // them, ~2 us each from mapped host memory)
    const sv_u4* src = (const sv_u4*)(mp - lead);
    constexpr int kIt = (SV_MSG_CAP / 16 + LPS - 1) / LPS;
    sv_u4 t[kIt];
    SV_UNROLL for (int k = 0; k < kIt; ++k) {
      const uint32_t c = li + (uint32_t)(k * LPS);
      t[k] = src[c < nq ? c : nq - 1];
    }
    // (pins the loads here: LLVM would otherwise sink each one into its
    // predicated LDS write below, one round trip apiece again)
    SV_UNROLL for (int k = 0; k < kIt; ++k) asm volatile("" : "+v"(t[k].x), "+v"(t[k].y), "+v"(t[k].z), "+v"(t[k].w));
    SV_UNROLL for (int k = 0; k < kIt; ++k) {
      const uint32_t c = li + (uint32_t)(k * LPS);
      if (c < nq) lbuf[c] = t[k];
    }
  }
  // (the lanes of one wave: LDS is in order within the wave)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  sha512_ram_var(hram, R, A, fits ? (const uint8_t*)lbuf + lead : mp, mlen);
}
