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

// Cache keys of a latency-lane batch, whose image the kernel reads in place
// from mapped host memory: there every dependent round trip costs ~2 us and
// the per-lane kernel above reads each message dword by dword at a stride of
// one message per lane (~64 lines per load instruction), which measured
// ~140 us for 1k SCP envelopes.  Here one wave stages the 16-byte-aligned
// windows of its 64 messages in LDS first -- item j's window by the whole
// wave, one 16-byte load per lane, so each load instruction is one contiguous
// run -- and pk / sig come as 16-byte loads; each lane then hashes its item
// from LDS (a message longer than the window is read from memory).
#define SV_KWIN 33  // quads per staged window: a 512-byte message at any alignment
__global__ __launch_bounds__(64) void sv_cachekey_lds_kernel(sv_hparams p) {
  __shared__ uint4 s_win[64][SV_KWIN];
  // (the latency lane's verify kernels run at priority 3: at the default
  // priority these waves would wait out the comb kernel on every shared SIMD)
  __builtin_amdgcn_s_setprio(3);
  const uint32_t lane = threadIdx.x;
  const uint64_t base = (uint64_t)blockIdx.x * 64;
  const uint64_t last = p.n - 1;
  const uint64_t i = base + lane;
  const uint64_t ii = i <= last ? i : last;
  // every lane fetches its item's message address first (one load each, in
  // parallel: the offsets live in the same mapped image, a round trip apiece),
  // then item j's window is loaded by the whole wave with j's address read
  // from lane j (v_readlane), by LDS-DMA (global_load_lds_dwordx4: no VGPR
  // round trip, so the 64 loads are in flight together and cost one wait)
  const uint8_t* m;
  uint32_t L;
  sv_item_msg(p, ii, m, L);
  const uint32_t lead = (uint32_t)((uintptr_t)m & 15u);
  const uint32_t nq = (lead + L + 15u) >> 4;
  const uint64_t wa = (uint64_t)(uintptr_t)(m - lead);
  const uint32_t wlo = (uint32_t)wa, whi = (uint32_t)(wa >> 32);
  // (pk and sig in flight with the windows)
  uint32_t pk[8], sig[16];
  {
    const uint4* a = (const uint4*)(p.pk + 8 * ii);
    const uint4* b = (const uint4*)(p.sig + 16 * ii);
    SV_UNROLL for (int q = 0; q < 2; ++q) {
      const uint4 v = a[q];
      pk[4 * q] = v.x; pk[4 * q + 1] = v.y; pk[4 * q + 2] = v.z; pk[4 * q + 3] = v.w;
    }
    SV_UNROLL for (int q = 0; q < 4; ++q) {
      const uint4 v = b[q];
      sig[4 * q] = v.x; sig[4 * q + 1] = v.y; sig[4 * q + 2] = v.z; sig[4 * q + 3] = v.w;
    }
  }
  SV_NOUNROLL for (uint32_t j = 0; j < 64; ++j) {
    const uint32_t nqj = (uint32_t)__builtin_amdgcn_readlane((int)nq, (int)j);
    const uint64_t aj = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)whi, (int)j) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)wlo, (int)j);
    if (nqj <= SV_KWIN && lane < nqj)
      __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)(aj + 16u * lane),
                                       (__attribute__((address_space(3))) void*)((char*)&s_win[j][0]), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the DMA'd windows are in LDS)
  const bool fits = nq <= SV_KWIN;
  uint32_t k[8];
  sv_cache_key(k, pk, sig, fits ? (const uint8_t*)&s_win[lane][0] + lead : m, L);
  if (i <= last) {
    uint4* o = (uint4*)(p.out + 8 * i);
    o[0] = uint4{k[0], k[1], k[2], k[3]};
    o[1] = uint4{k[4], k[5], k[6], k[7]};
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

// kind 0: cache keys (pk, sig, msg), kind 1: SHA-256 (msg only), kind 2: cache
// keys of an image in mapped host memory (windows staged in LDS; pk and sig
// 16-byte aligned, out 16-byte aligned)
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
  if (kind == 2) {
    if (n) hipLaunchKernelGGL(sv_cachekey_lds_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, p);
  } else if (kind == 0) {
    hipLaunchKernelGGL(sv_cachekey_kernel, dim3(grid), dim3(SV_HBLOCK), 0, s, p);
  } else {
    hipLaunchKernelGGL(sv_sha256_kernel, dim3(grid), dim3(SV_HBLOCK), 0, s, p);
  }
  return hipGetLastError();
}

}  // extern "C"
