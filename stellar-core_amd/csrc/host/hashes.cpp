// BLAKE2b-256 (RFC 7693) and SHA-256 (FIPS 180-4), written from the specs.
// Checked against Python hashlib in tests/test_host_mirror.py.
#include "hashes.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace stellar {
namespace hostcrypto {

namespace {

// RFC 7693 §2.6: IV = SHA-512 initial values
constexpr uint64_t kIV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                         0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                         0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
// RFC 7693 §2.7 message schedule SIGMA
constexpr uint8_t kSigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

inline uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

inline uint64_t load64le(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

}  // namespace

Blake2b256::Blake2b256() : t_{0, 0}, fill_(0) {
  for (int i = 0; i < 8; ++i) h_[i] = kIV[i];
  h_[0] ^= 0x01010000ULL ^ 32u;  // depth 1, fanout 1, no key, digest length 32
}

#if defined(__x86_64__)
// AVX2 form of the same compression (x86-64 hosts that have it; chosen at run
// time): the state as four rows of four 64-bit words, the four G functions of
// a column (then a diagonal) step in one vector each, the diagonal step by
// rotating rows 2-4 (RFC 7693 3.2's G on (v0,v4,v8,v12) .. (v3,v7,v11,v15),
// then (v0,v5,v10,v15) ..).  Rotations by 32 / 24 / 16 are byte shuffles, by
// 63 a shift and an add.
__attribute__((target("avx2"))) void blake2b_compress_avx2(uint64_t h[8], const uint8_t* block, uint64_t t0,
                                                           uint64_t t1, bool last) {
  uint64_t m[16];
  std::memcpy(m, block, sizeof m);
  const __m256i r16 = _mm256_setr_epi8(2, 3, 4, 5, 6, 7, 0, 1, 10, 11, 12, 13, 14, 15, 8, 9, 2, 3, 4, 5, 6, 7, 0, 1,
                                       10, 11, 12, 13, 14, 15, 8, 9);
  const __m256i r24 = _mm256_setr_epi8(3, 4, 5, 6, 7, 0, 1, 2, 11, 12, 13, 14, 15, 8, 9, 10, 3, 4, 5, 6, 7, 0, 1, 2,
                                       11, 12, 13, 14, 15, 8, 9, 10);
  __m256i a = _mm256_loadu_si256((const __m256i*)h);
  __m256i b = _mm256_loadu_si256((const __m256i*)(h + 4));
  __m256i c = _mm256_loadu_si256((const __m256i*)kIV);
  __m256i d = _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(kIV + 4)),
                               _mm256_setr_epi64x((long long)t0, (long long)t1, last ? -1LL : 0LL, 0LL));
  const __m256i a0 = a, b0 = b;
#define SV_B2_G(mx, my)                                                            \
  a = _mm256_add_epi64(_mm256_add_epi64(a, mx), b);                                \
  d = _mm256_shuffle_epi32(_mm256_xor_si256(d, a), _MM_SHUFFLE(2, 3, 0, 1));       \
  c = _mm256_add_epi64(c, d);                                                      \
  b = _mm256_shuffle_epi8(_mm256_xor_si256(b, c), r24);                            \
  a = _mm256_add_epi64(_mm256_add_epi64(a, my), b);                                \
  d = _mm256_shuffle_epi8(_mm256_xor_si256(d, a), r16);                            \
  c = _mm256_add_epi64(c, d);                                                      \
  b = _mm256_xor_si256(b, c);                                                      \
  b = _mm256_xor_si256(_mm256_srli_epi64(b, 63), _mm256_add_epi64(b, b));
#define SV_B2_M(r, i, j, k, l) \
  _mm256_setr_epi64x((long long)m[kSigma[r][i]], (long long)m[kSigma[r][j]], (long long)m[kSigma[r][k]], \
                     (long long)m[kSigma[r][l]])
// (rows a, c, d rotate, not b: see the AVX-512 form below)
#define SV_B2_ROUND(r)                                                                             \
  SV_B2_G(SV_B2_M(r, 0, 2, 4, 6), SV_B2_M(r, 1, 3, 5, 7))                                          \
  a = _mm256_permute4x64_epi64(a, _MM_SHUFFLE(2, 1, 0, 3));                                        \
  c = _mm256_permute4x64_epi64(c, _MM_SHUFFLE(0, 3, 2, 1));                                        \
  d = _mm256_permute4x64_epi64(d, _MM_SHUFFLE(1, 0, 3, 2));                                        \
  SV_B2_G(SV_B2_M(r, 14, 8, 10, 12), SV_B2_M(r, 15, 9, 11, 13))                                    \
  a = _mm256_permute4x64_epi64(a, _MM_SHUFFLE(0, 3, 2, 1));                                        \
  c = _mm256_permute4x64_epi64(c, _MM_SHUFFLE(2, 1, 0, 3));                                        \
  d = _mm256_permute4x64_epi64(d, _MM_SHUFFLE(1, 0, 3, 2));
  SV_B2_ROUND(0) SV_B2_ROUND(1) SV_B2_ROUND(2) SV_B2_ROUND(3) SV_B2_ROUND(4) SV_B2_ROUND(5)
  SV_B2_ROUND(6) SV_B2_ROUND(7) SV_B2_ROUND(8) SV_B2_ROUND(9) SV_B2_ROUND(10) SV_B2_ROUND(11)
#undef SV_B2_ROUND
#undef SV_B2_M
#undef SV_B2_G
  _mm256_storeu_si256((__m256i*)h, _mm256_xor_si256(a0, _mm256_xor_si256(a, c)));
  _mm256_storeu_si256((__m256i*)(h + 4), _mm256_xor_si256(b0, _mm256_xor_si256(b, d)));
}
const bool kHaveAvx2 = __builtin_cpu_supports("avx2");

// AVX-512VL form (chosen at run time where the host has it): the same four
// rows, every G's message vector ONE two-table permute (vpermt2q) of the 16
// message words held in two 512-bit registers instead of four scalar inserts,
// and the rotations single vprorq instructions.  (In both vector forms the
// message word is added to a before b: b is the end of the previous G's
// dependency chain, a + m is not.)
__attribute__((target("avx512f,avx512vl"))) void blake2b_compress_avx512(uint64_t h[8], const uint8_t* block,
                                                                         uint64_t t0, uint64_t t1, bool last) {
  const __m512i mlo = _mm512_loadu_si512((const void*)block);
  const __m512i mhi = _mm512_loadu_si512((const void*)(block + 64));
  __m256i a = _mm256_loadu_si256((const __m256i*)h);
  __m256i b = _mm256_loadu_si256((const __m256i*)(h + 4));
  __m256i c = _mm256_loadu_si256((const __m256i*)kIV);
  __m256i d = _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(kIV + 4)),
                               _mm256_setr_epi64x((long long)t0, (long long)t1, last ? -1LL : 0LL, 0LL));
  const __m256i a0 = a, b0 = b;
#define SV_B5_G(mx, my)                                 \
  a = _mm256_add_epi64(_mm256_add_epi64(a, mx), b);     \
  d = _mm256_ror_epi64(_mm256_xor_si256(d, a), 32);     \
  c = _mm256_add_epi64(c, d);                           \
  b = _mm256_ror_epi64(_mm256_xor_si256(b, c), 24);     \
  a = _mm256_add_epi64(_mm256_add_epi64(a, my), b);     \
  d = _mm256_ror_epi64(_mm256_xor_si256(d, a), 16);     \
  c = _mm256_add_epi64(c, d);                           \
  b = _mm256_ror_epi64(_mm256_xor_si256(b, c), 63);
#define SV_B5_M(r, i, j, k, l)                                                                                  \
  _mm512_castsi512_si256(_mm512_permutex2var_epi64(                                                           \
      mlo, _mm512_setr_epi64(kSigma[r][i], kSigma[r][j], kSigma[r][k], kSigma[r][l], 0, 0, 0, 0), mhi))
// The diagonal step rotates rows a, c and d, never b: b is the end of each
// G's dependency chain and the next G starts with a + b, so a permute of b
// (3 cycles) would sit on the critical path, while a, c and d were last
// written 8, 2 and 6 operations before the end of the G and their permutes
// overlap it.  Relative to a, the rows are then offset by (1, 2, 3) lanes, as
// the diagonals need; lane i runs diagonal G (i + 3) % 4, so its message
// words are sigma[8 + 2j], sigma[9 + 2j] with j = (i + 3) % 4.
#define SV_B5_ROUND(r)                                                        \
  SV_B5_G(SV_B5_M(r, 0, 2, 4, 6), SV_B5_M(r, 1, 3, 5, 7))                     \
  a = _mm256_permute4x64_epi64(a, _MM_SHUFFLE(2, 1, 0, 3));                   \
  c = _mm256_permute4x64_epi64(c, _MM_SHUFFLE(0, 3, 2, 1));                   \
  d = _mm256_permute4x64_epi64(d, _MM_SHUFFLE(1, 0, 3, 2));                   \
  SV_B5_G(SV_B5_M(r, 14, 8, 10, 12), SV_B5_M(r, 15, 9, 11, 13))               \
  a = _mm256_permute4x64_epi64(a, _MM_SHUFFLE(0, 3, 2, 1));                   \
  c = _mm256_permute4x64_epi64(c, _MM_SHUFFLE(2, 1, 0, 3));                   \
  d = _mm256_permute4x64_epi64(d, _MM_SHUFFLE(1, 0, 3, 2));
  SV_B5_ROUND(0) SV_B5_ROUND(1) SV_B5_ROUND(2) SV_B5_ROUND(3) SV_B5_ROUND(4) SV_B5_ROUND(5)
  SV_B5_ROUND(6) SV_B5_ROUND(7) SV_B5_ROUND(8) SV_B5_ROUND(9) SV_B5_ROUND(10) SV_B5_ROUND(11)
#undef SV_B5_ROUND
#undef SV_B5_M
#undef SV_B5_G
  _mm256_storeu_si256((__m256i*)h, _mm256_xor_si256(a0, _mm256_xor_si256(a, c)));
  _mm256_storeu_si256((__m256i*)(h + 4), _mm256_xor_si256(b0, _mm256_xor_si256(b, d)));
}
const bool kHaveAvx512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
                         getenv("SVH_NO_AVX512") == nullptr;
#endif

void Blake2b256::compress(const uint8_t* block, bool last) {
#if defined(__x86_64__)
  if (kHaveAvx512) {
    blake2b_compress_avx512(h_, block, t_[0], t_[1], last);
    return;
  }
  if (kHaveAvx2) {
    blake2b_compress_avx2(h_, block, t_[0], t_[1], last);
    return;
  }
#endif
  uint64_t m[16];
  std::memcpy(m, block, sizeof m);  // (little-endian host: the words as stored)
  uint64_t v0 = h_[0], v1 = h_[1], v2 = h_[2], v3 = h_[3], v4 = h_[4], v5 = h_[5], v6 = h_[6], v7 = h_[7];
  uint64_t v8 = kIV[0], v9 = kIV[1], v10 = kIV[2], v11 = kIV[3];
  uint64_t v12 = kIV[4] ^ t_[0], v13 = kIV[5] ^ t_[1], v14 = last ? ~kIV[6] : kIV[6], v15 = kIV[7];
  // every round and G spelled out with constant sigma indices, so the 16
  // state words stay in registers (a loop over kSigma kept them in memory:
  // ~14 cycles/byte; this form is ~3)
#define SV_G(a, b, c, d, x, y) \
  a = a + b + (x);             \
  d = rotr64(d ^ a, 32);       \
  c = c + d;                   \
  b = rotr64(b ^ c, 24);       \
  a = a + b + (y);             \
  d = rotr64(d ^ a, 16);       \
  c = c + d;                   \
  b = rotr64(b ^ c, 63);
#define SV_ROUND(r)                                                   \
  SV_G(v0, v4, v8, v12, m[kSigma[r][0]], m[kSigma[r][1]])             \
  SV_G(v1, v5, v9, v13, m[kSigma[r][2]], m[kSigma[r][3]])             \
  SV_G(v2, v6, v10, v14, m[kSigma[r][4]], m[kSigma[r][5]])            \
  SV_G(v3, v7, v11, v15, m[kSigma[r][6]], m[kSigma[r][7]])            \
  SV_G(v0, v5, v10, v15, m[kSigma[r][8]], m[kSigma[r][9]])            \
  SV_G(v1, v6, v11, v12, m[kSigma[r][10]], m[kSigma[r][11]])          \
  SV_G(v2, v7, v8, v13, m[kSigma[r][12]], m[kSigma[r][13]])           \
  SV_G(v3, v4, v9, v14, m[kSigma[r][14]], m[kSigma[r][15]])
  SV_ROUND(0) SV_ROUND(1) SV_ROUND(2) SV_ROUND(3) SV_ROUND(4) SV_ROUND(5)
  SV_ROUND(6) SV_ROUND(7) SV_ROUND(8) SV_ROUND(9) SV_ROUND(10) SV_ROUND(11)
#undef SV_ROUND
#undef SV_G
  h_[0] ^= v0 ^ v8;
  h_[1] ^= v1 ^ v9;
  h_[2] ^= v2 ^ v10;
  h_[3] ^= v3 ^ v11;
  h_[4] ^= v4 ^ v12;
  h_[5] ^= v5 ^ v13;
  h_[6] ^= v6 ^ v14;
  h_[7] ^= v7 ^ v15;
}

void Blake2b256::add(const uint8_t* p, size_t n) {
  // a block is compressed only once more input follows it (the last block is
  // compressed by finish() with the final flag); full blocks of the input are
  // compressed in place, only a partial block is copied into buf_
  if (n == 0) return;
  if (fill_ > 0) {
    const size_t take = std::min(128 - fill_, n);
    std::memcpy(buf_ + fill_, p, take);
    fill_ += take;
    p += take;
    n -= take;
    if (n == 0) return;
    bump(128);
    compress(buf_, false);
    fill_ = 0;
  }
  while (n > 128) {
    bump(128);
    compress(p, false);
    p += 128;
    n -= 128;
  }
  std::memcpy(buf_, p, n);
  fill_ = n;
}

Hash32 Blake2b256::finish() {
  bump(fill_);
  std::memset(buf_ + fill_, 0, 128 - fill_);
  compress(buf_, true);
  Hash32 out;
  std::memcpy(out.data(), h_, 32);  // (little-endian host: the state words as bytes)
  return out;
}

Hash32 blake2b256(const uint8_t* p, size_t n) {
  Blake2b256 b;
  b.add(p, n);
  return b.finish();
}

Hash32 sha256(const uint8_t* p, size_t n) {
  static const uint32_t K[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  const uint64_t bits = (uint64_t)n * 8;
  const size_t total = ((n + 9 + 63) / 64) * 64;
  uint8_t blk[64];
  for (size_t off = 0; off < total; off += 64) {
    for (int i = 0; i < 64; ++i) {
      const size_t k = off + i;
      uint8_t b;
      if (k < n) b = p[k];
      else if (k == n) b = 0x80;
      else if (k >= total - 8) b = (uint8_t)(bits >> (8 * (total - 1 - k)));
      else b = 0;
      blk[i] = b;
    }
    uint32_t w[64];
    for (int t = 0; t < 16; ++t)
      w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) | ((uint32_t)blk[4 * t + 2] << 8) |
             blk[4 * t + 3];
    for (int t = 16; t < 64; ++t) {
      const uint32_t s0 = rotr32(w[t - 15], 7) ^ rotr32(w[t - 15], 18) ^ (w[t - 15] >> 3);
      const uint32_t s1 = rotr32(w[t - 2], 17) ^ rotr32(w[t - 2], 19) ^ (w[t - 2] >> 10);
      w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = h[0], b2 = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int t = 0; t < 64; ++t) {
      const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = hh + S1 + ch + K[t] + w[t];
      const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
      const uint32_t mj = (a & b2) ^ (a & c) ^ (b2 & c);
      const uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b2; b2 = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b2; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  Hash32 out;
  for (int i = 0; i < 8; ++i)
    for (int k = 0; k < 4; ++k) out[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
  return out;
}

}  // namespace hostcrypto
}  // namespace stellar
