// BLAKE2b-256 (RFC 7693) and SHA-256 (FIPS 180-4) for one lane.
//
// What they replace in the reference:
//   * verify-cache key  BLAKE2b-256(pk || sig || msg)  per signature,
//     /root/reference/src/crypto/SecretKey.cpp:50-61 (verifySigCacheKey), hashed
//     on the host before every cache lookup;
//   * transaction contents hash  SHA-256(networkID || envelope type || tx XDR),
//     /root/reference/src/transactions/TransactionFrame.cpp:90-117, the 32-byte
//     message every transaction signature is verified over.
// Computing them in the same device pass removes the remaining per-signature
// host cost (~1 us of BLAKE2b against ~14 ns of GPU verification).
//
// Input bytes are read as aligned dwords plus a funnel shift: an aligned dword
// never crosses a page, so reading the whole dword that holds the last valid
// byte is always safe; bytes past the end are masked to zero.
#pragma once

#include "sv_common.h"

// Little-endian 32-bit word of the bytes p[0..3], zero-filled past `avail`
// valid bytes (avail <= 0 gives 0).  p may have any alignment.
SV_HD uint32_t sv_ld32(const uint8_t* p, int64_t avail) {
  if (avail <= 0) return 0u;
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3u);
  uint32_t v = w[0] >> (8u * sh);
  if (sh != 0 && avail > (int64_t)(4 - sh)) v |= w[1] << (32u - 8u * sh);
  if (avail < 4) v &= (1u << (8u * (uint32_t)avail)) - 1u;
  return v;
}

SV_HD uint32_t sv_rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// 64-bit rotate (n a compile-time constant, 0 < n < 64): on the device two
// v_alignbit_b32 on the halves, or a swap for n = 32 (LLVM otherwise emits
// two 64-bit shifts and two ORs)
SV_HD uint64_t sv_rotr64b(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n == 32) return sv_pack64(hi, lo);
  if (n < 32) return sv_pack64(__builtin_amdgcn_alignbit(hi, lo, n), __builtin_amdgcn_alignbit(lo, hi, n));
  return sv_pack64(__builtin_amdgcn_alignbit(lo, hi, n - 32), __builtin_amdgcn_alignbit(hi, lo, n - 32));
#else
  return (x >> n) | (x << (64 - n));
#endif
}
SV_HD uint32_t sv_bswap32b(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// ------------------------------------------------------------------ BLAKE2b
SV_HD void blake2b_compress(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
  constexpr uint8_t SIG[12][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
  constexpr uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                              0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                              0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  uint64_t v[16];
  SV_UNROLL for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = IV[i]; }
  v[12] ^= t;  // byte counter (< 2^64 here, so the high counter word stays 0)
  if (last) v[14] = ~v[14];
#define SV_B2G(a, b, c, d, x, y)          \
  v[a] = v[a] + v[b] + (x);               \
  v[d] = sv_rotr64b(v[d] ^ v[a], 32);     \
  v[c] = v[c] + v[d];                     \
  v[b] = sv_rotr64b(v[b] ^ v[c], 24);     \
  v[a] = v[a] + v[b] + (y);               \
  v[d] = sv_rotr64b(v[d] ^ v[a], 16);     \
  v[c] = v[c] + v[d];                     \
  v[b] = sv_rotr64b(v[b] ^ v[c], 63);
  SV_UNROLL for (int r = 0; r < 12; ++r) {
    SV_B2G(0, 4, 8, 12, m[SIG[r][0]], m[SIG[r][1]]);
    SV_B2G(1, 5, 9, 13, m[SIG[r][2]], m[SIG[r][3]]);
    SV_B2G(2, 6, 10, 14, m[SIG[r][4]], m[SIG[r][5]]);
    SV_B2G(3, 7, 11, 15, m[SIG[r][6]], m[SIG[r][7]]);
    SV_B2G(0, 5, 10, 15, m[SIG[r][8]], m[SIG[r][9]]);
    SV_B2G(1, 6, 11, 12, m[SIG[r][10]], m[SIG[r][11]]);
    SV_B2G(2, 7, 8, 13, m[SIG[r][12]], m[SIG[r][13]]);
    SV_B2G(3, 4, 9, 14, m[SIG[r][14]], m[SIG[r][15]]);
  }
#undef SV_B2G
  SV_UNROLL for (int i = 0; i < 8; ++i) h[i] = sv_xor3_64(h[i], v[i], v[i + 8]);
}

// Verify-cache key: BLAKE2b-256 of pk(32) || sig(64) || msg(len), as 8 LE words.
// pk and sig are 4-byte aligned (16 in the engine's buffers); msg any alignment.
SV_COLD void sv_cache_key(uint32_t out[8], const uint32_t* pk, const uint32_t* sig, const uint8_t* msg,
                          uint32_t len) {
  uint64_t h[8] = {0x6a09e667f3bcc908ULL ^ 0x01010020ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  const uint64_t total = 96ull + len;
  const uint64_t nb = (total + 127) / 128;  // >= 1
  SV_NOUNROLL for (uint64_t b = 0; b < nb; ++b) {
    uint64_t m[16];
    SV_UNROLL for (int i = 0; i < 16; ++i) {
      uint32_t lo, hi;
      const uint64_t q = b * 128 + 8 * (uint64_t)i;  // byte position of the word
      if (b == 0 && i < 4) {
        lo = pk[2 * i]; hi = pk[2 * i + 1];
      } else if (b == 0 && i < 12) {
        lo = sig[2 * (i - 4)]; hi = sig[2 * (i - 4) + 1];
      } else {
        const int64_t o = (int64_t)(q - 96);
        lo = sv_ld32(msg + o, (int64_t)len - o);
        hi = sv_ld32(msg + o + 4, (int64_t)len - o - 4);
      }
      m[i] = sv_pack64(lo, hi);
    }
    const bool last = b + 1 == nb;
    blake2b_compress(h, m, last ? total : (b + 1) * 128, last);
  }
  SV_UNROLL for (int i = 0; i < 4; ++i) {
    out[2 * i] = (uint32_t)h[i];
    out[2 * i + 1] = (uint32_t)(h[i] >> 32);
  }
}

// ------------------------------------------------------------------ SHA-256
SV_CONST uint32_t SV_SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

SV_HD void sha256_compress(uint32_t st[8], uint32_t w[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  SV_NOUNROLL for (int pass = 0; pass < 4; ++pass) {
    SV_UNROLL for (int i = 0; i < 16; ++i) {
      if (pass > 0) {
        const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
        const uint32_t s0 = sv_xor3_32(sv_rotr32(w15, 7), sv_rotr32(w15, 18), w15 >> 3);
        const uint32_t s1 = sv_xor3_32(sv_rotr32(w2, 17), sv_rotr32(w2, 19), w2 >> 10);
        w[i] += s0 + w[(i + 9) & 15] + s1;
      }
      const uint32_t S1 = sv_xor3_32(sv_rotr32(e, 6), sv_rotr32(e, 11), sv_rotr32(e, 25));
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = h + S1 + ch + SV_SHA256_K[pass * 16 + i] + w[i];
      const uint32_t S0 = sv_xor3_32(sv_rotr32(a, 2), sv_rotr32(a, 13), sv_rotr32(a, 22));
      const uint32_t mj = sv_maj32(a, b, c);
      h = g; g = f; f = e; e = d + t1;
      d = c; c = b; b = a; a = t1 + S0 + mj;
    }
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// SHA-256 of data[0..len) as 8 big-endian words packed little-endian (i.e.
// out bytes == the digest bytes).
SV_COLD void sv_sha256(uint32_t out[8], const uint8_t* data, uint32_t len) {
  uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint64_t L = len;
  const uint64_t nb = (L + 9 + 63) / 64;
  SV_NOUNROLL for (uint64_t b = 0; b < nb; ++b) {
    uint32_t w[16];
    SV_UNROLL for (int i = 0; i < 16; ++i) {
      const uint64_t q = b * 64 + 4 * (uint64_t)i;
      uint32_t v = q < L ? sv_ld32(data + q, (int64_t)(L - q)) : 0u;
      if (L >= q && L < q + 4) v |= 0x80u << (8u * (uint32_t)(L - q));  // the padding bit
      v = sv_bswap32b(v);
      if (b + 1 == nb && i == 14) v = (uint32_t)(L >> 29);
      if (b + 1 == nb && i == 15) v = (uint32_t)(L << 3);
      w[i] = v;
    }
    sha256_compress(st, w);
  }
  SV_UNROLL for (int i = 0; i < 8; ++i) out[i] = sv_bswap32b(st[i]);
}
