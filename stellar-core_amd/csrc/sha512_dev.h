// SHA-512 (FIPS 180-4) for one lane, 64-bit words emulated on 32-bit VALU
// (rotates become v_alignbit_b32 pairs, adds v_add_co/v_addc pairs).
//
// Used for h = SHA-512(R || A || M), step (6) of libsodium 1.0.18
// crypto_sign_verify_detached as called by stellar-core
// src/crypto/SecretKey.cpp:461-463.  Round constants are derived in
// tools/gen_constants.py from their FIPS definition.
#pragma once

#include "sv_common.h"

SV_CONST uint64_t SV_SHA512_K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

// 64-bit rotate (n a compile-time constant, 0 < n < 64).  Device: two
// v_alignbit_b32 on the 32-bit halves (LLVM otherwise expands it into two
// 64-bit shifts and two ORs).
SV_HD uint64_t sv_rotr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t rlo, rhi;
  if (n < 32) {
    rlo = __builtin_amdgcn_alignbit(hi, lo, n);
    rhi = __builtin_amdgcn_alignbit(lo, hi, n);
  } else if (n == 32) {
    rlo = hi;
    rhi = lo;
  } else {
    rlo = __builtin_amdgcn_alignbit(lo, hi, n - 32);
    rhi = __builtin_amdgcn_alignbit(hi, lo, n - 32);
  }
  return sv_pack64(rlo, rhi);
#else
  return (x >> n) | (x << (64 - n));
#endif
}
SV_HD uint32_t sv_bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}
// big-endian 64-bit word from 8 little-endian-packed bytes held as two u32
SV_HD uint64_t sv_be64(uint32_t lo_bytes, uint32_t hi_bytes) {
  return sv_pack64(sv_bswap32(hi_bytes), sv_bswap32(lo_bytes));
}

SV_HD void sha512_init(uint64_t st[8]) {
  st[0] = 0x6a09e667f3bcc908ULL; st[1] = 0xbb67ae8584caa73bULL;
  st[2] = 0x3c6ef372fe94f82bULL; st[3] = 0xa54ff53a5f1d36f1ULL;
  st[4] = 0x510e527fade682d1ULL; st[5] = 0x9b05688c2b3e6c1fULL;
  st[6] = 0x1f83d9abfb41bd6bULL; st[7] = 0x5be0cd19137e2179ULL;
}

// One compression, inlined into its caller so the state and the message
// schedule live in registers (as an out-of-line function with array
// arguments the schedule went through memory every round).  Rounds 0-15 run
// unrolled without the schedule update; rounds 16-79 as 4 rolled passes of 16
// unrolled rounds (static register indices, uniform round-constant loads).
#define SV_SHA512_ROUND(Wi, Ki)                                                       \
  do {                                                                               \
    const uint64_t S1 = sv_xor3_64(sv_rotr64(e, 14), sv_rotr64(e, 18), sv_rotr64(e, 41)); \
    const uint64_t ch = (e & f) ^ (~e & g);                                           \
    const uint64_t t1 = h + S1 + ch + (Ki) + (Wi);                                    \
    const uint64_t S0 = sv_xor3_64(sv_rotr64(a, 28), sv_rotr64(a, 34), sv_rotr64(a, 39)); \
    const uint64_t mj = sv_maj64(a, b, c);                                            \
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;           \
  } while (0)
SV_HD void sha512_compress(uint64_t st[8], uint64_t w[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  SV_UNROLL for (int i = 0; i < 16; ++i) SV_SHA512_ROUND(w[i], SV_SHA512_K[i]);
  SV_NOUNROLL for (int pass = 1; pass < 5; ++pass) {
    SV_UNROLL for (int i = 0; i < 16; ++i) {
      const uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint64_t s0 = sv_xor3_64(sv_rotr64(w15, 1), sv_rotr64(w15, 8), w15 >> 7);
      const uint64_t s1 = sv_xor3_64(sv_rotr64(w2, 19), sv_rotr64(w2, 61), w2 >> 6);
      w[i] = w[i] + s0 + w[(i + 9) & 15] + s1;
      SV_SHA512_ROUND(w[i], SV_SHA512_K[16 * pass + i]);
    }
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// digest as a little-endian 512-bit integer in 16 u32 words
SV_HD void sha512_digest_le(uint32_t out[16], const uint64_t st[8]) {
  SV_UNROLL for (int i = 0; i < 8; ++i) {
    out[2 * i] = sv_bswap32((uint32_t)(st[i] >> 32));
    out[2 * i + 1] = sv_bswap32((uint32_t)st[i]);
  }
}

// SHA-512(R || A || M) for a 32-byte M: exactly one block.
SV_HD void sha512_ram32(uint32_t out[16], const uint32_t R[8], const uint32_t A[8], const uint32_t M[8]) {
  uint64_t st[8], w[16];
  sha512_init(st);
  SV_UNROLL for (int t = 0; t < 4; ++t) {
    w[t] = sv_be64(R[2 * t], R[2 * t + 1]);
    w[4 + t] = sv_be64(A[2 * t], A[2 * t + 1]);
    w[8 + t] = sv_be64(M[2 * t], M[2 * t + 1]);
  }
  w[12] = 0x8000000000000000ULL;
  w[13] = 0;
  w[14] = 0;
  w[15] = 96 * 8;
  sha512_compress(st, w);
  sha512_digest_le(out, st);
}

// Message bytes m[mi, mi + 8) as a big-endian SHA-512 word, bytes at or past
// mlen replaced by the padding (0x80 at mlen, zeros after).  Reads aligned
// dwords only, and only those holding at least one message byte (so never
// past the message's last dword), then funnel-shifts them into place.
SV_HD uint64_t sv_msg_word(const uint8_t* m, uint32_t mlen, uint32_t mi) {
  const uintptr_t a = (uintptr_t)(m + mi), end = (uintptr_t)(m + mlen);
  const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  const uint32_t d0 = (uintptr_t)q < end ? q[0] : 0u;
  const uint32_t d1 = (uintptr_t)(q + 1) < end ? q[1] : 0u;
  const uint32_t d2 = (uintptr_t)(q + 2) < end ? q[2] : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = __builtin_amdgcn_alignbit(d1, d0, sh);
  const uint32_t hi = __builtin_amdgcn_alignbit(d2, d1, sh);
#else
  const uint32_t lo = sh ? (d0 >> sh) | (d1 << (32 - sh)) : d0;
  const uint32_t hi = sh ? (d1 >> sh) | (d2 << (32 - sh)) : d1;
#endif
  uint64_t v = sv_pack64(lo, hi);  // byte j of the word at bits 8j
  if (mlen < mi + 8) {
    const uint32_t valid = mlen > mi ? mlen - mi : 0u;  // < 8
    v &= (1ull << (8 * valid)) - 1;
    if (mlen >= mi) v |= 0x80ull << (8 * (mlen - mi));
  }
  return sv_be64((uint32_t)v, (uint32_t)(v >> 32));
}

// SHA-512(R || A || M) for an arbitrary-length M in memory (any alignment).
// Stream: R (32 B) || A (32 B) fill words 0-7 of block 0; message byte j is at
// stream offset 64 + j, so every other word is 8 consecutive message bytes
// (sv_msg_word); word 15 of the last block is the bit length (< 2^64).
SV_HD void sha512_ram_var(uint32_t out[16], const uint32_t R[8], const uint32_t A[8], const uint8_t* m,
                          uint32_t mlen) {
  uint64_t st[8], w[16];
  sha512_init(st);
  const uint32_t nblocks = (64u + mlen + 16u + 1u + 127u) / 128u;
  SV_NOUNROLL for (uint32_t blk = 0; blk < nblocks; ++blk) {
    SV_UNROLL for (int t = 0; t < 16; ++t) {
      uint64_t v;
      if (t < 8 && blk == 0) {
        v = t < 4 ? sv_be64(R[2 * t], R[2 * t + 1]) : sv_be64(A[2 * t - 8], A[2 * t - 7]);
      } else {
        v = sv_msg_word(m, mlen, 128u * blk + 8u * (uint32_t)t - 64u);
      }
      if (t == 15 && blk == nblocks - 1) v = (uint64_t)(64u + mlen) * 8u;
      w[t] = v;
    }
    sha512_compress(st, w);
  }
  sha512_digest_le(out, st);
}
