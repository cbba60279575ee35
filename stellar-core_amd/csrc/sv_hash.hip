// gfx950 batch hashing kernels: verify-cache keys
// BLAKE2b-256(pk || sig || msg) and SHA-256 of byte strings, one lane per item,
// grid-stride.  The per-lane algorithms are hash_dev.h; these kernels are
// memory- and latency-light companions of the verify kernel (~3-6k VALU per
// item against ~450k for a verification), launched on the same stream.
#include <hip/hip_runtime.h>

#include "hash_dev.h"

#define SV_HBLOCK 256

struct sv_hparams {
  const uint32_t* pk;       // n x 32 B (cache keys only; 4-byte aligned)
  const uint32_t* sig;      // n x 64 B (cache keys only)
  const uint8_t* msg;       // fixed: n x fixed_len ; var: bytes at off[i]
  const uint64_t* off;
  const uint32_t* len;
  uint32_t fixed_len;       // 0 = variable length
  uint64_t n;
  uint32_t* out;            // n x 8 words (32-byte digests)
};

__device__ __forceinline__ void sv_item_msg(const sv_hparams& p, uint64_t i, const uint8_t*& m, uint32_t& L) {
  if (p.fixed_len) {
    m = p.msg + i * (uint64_t)p.fixed_len;
    L = p.fixed_len;
  } else {
    m = p.msg + p.off[i];
    L = p.len[i];
  }
}

__global__ __launch_bounds__(SV_HBLOCK) void sv_cachekey_kernel(sv_hparams p) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t* m;
    uint32_t L;
    sv_item_msg(p, i, m, L);
    uint32_t k[8];
    sv_cache_key(k, p.pk + 8 * i, p.sig + 16 * i, m, L);
    SV_UNROLL for (int w = 0; w < 8; ++w) p.out[8 * i + w] = k[w];
  }
}

__global__ __launch_bounds__(SV_HBLOCK) void sv_sha256_kernel(sv_hparams p) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t* m;
    uint32_t L;
    sv_item_msg(p, i, m, L);
    uint32_t d[8];
    sv_sha256(d, m, L);
    SV_UNROLL for (int w = 0; w < 8; ++w) p.out[8 * i + w] = d[w];
  }
}

extern "C" {

// kind 0: cache keys (pk, sig, msg), kind 1: SHA-256 (msg only)
hipError_t sv_launch_hash(int kind, unsigned max_blocks, const void* pk, const void* sig, const void* msg,
                          const uint64_t* off, const uint32_t* len, uint32_t fixed_len, uint64_t n, void* out,
                          hipStream_t s) {
  sv_hparams p;
  p.pk = (const uint32_t*)pk;
  p.sig = (const uint32_t*)sig;
  p.msg = (const uint8_t*)msg;
  p.off = off;
  p.len = len;
  p.fixed_len = fixed_len;
  p.n = n;
  p.out = (uint32_t*)out;
  uint64_t need = (n + SV_HBLOCK - 1) / SV_HBLOCK;
  const unsigned grid = (unsigned)(need < max_blocks ? (need ? need : 1) : max_blocks);
  if (kind == 0) hipLaunchKernelGGL(sv_cachekey_kernel, dim3(grid), dim3(SV_HBLOCK), 0, s, p);
  else hipLaunchKernelGGL(sv_sha256_kernel, dim3(grid), dim3(SV_HBLOCK), 0, s, p);
  return hipGetLastError();
}

}  // extern "C"
