// Shared qualifiers for the device arithmetic headers.
//
// The arithmetic headers are written once and compiled for gfx950 by hipcc.
// tests/native/ also compiles them for the host with g++ (SV_HOST_TEST) so the
// limb-bound reasoning can be fuzzed on CPU against Python big integers; that
// host build is test infrastructure only and is never linked into the product.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SV_HD __host__ __device__ __forceinline__
// SV_COLD marks the once-per-signature phases (exponentiation chains,
// decompression, mod-L reduction, Euclid, table build).  They are inlined
// like everything else: out of line, their array
// and struct arguments travel through scratch memory at every call (the prep
// kernel spent ~23 % of its wave time waiting on memory); inlined, the whole
// per-signature path stays in registers: -4.7 % end-to-end measured, with no
// measurable instruction-cache misses (SQC_ICACHE_MISSES / HITS < 0.03 %).
#define SV_COLD __host__ __device__ __forceinline__
#define SV_CONST __constant__
#else
#define SV_HD static inline
#define SV_COLD static
#define SV_CONST static const
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// Keeps the scheduler from interleaving independent field operations, which
// otherwise multiplies their live ranges and spills VGPRs.
#define SV_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define SV_FENCE() ((void)0)
#endif

#if defined(__HIPCC__) || defined(__clang__)
#define SV_UNROLL _Pragma("unroll")
#define SV_NOUNROLL _Pragma("unroll 1")
#else
// g++ (host builds: the CPU path sv_cpu.cpp, tests/native): full unrolling
// keeps the limb arrays in registers, as on the device
#define SV_UNROLL _Pragma("GCC unroll 64")
#define SV_NOUNROLL _Pragma("GCC unroll 1")
#endif

// 64-bit word from its 32-bit halves.  On the device as a bit cast of a
// two-dword vector: LLVM turns the usual (hi << 32) | lo into a disjoint add
// and then splits every 64-bit add of the result into a zero-extended
// v_lshl_add_u64 plus a v_add_u32 on the high half (and v_movs to build the
// zero-extended pairs): 55 -> 47 instructions per SHA-512 round with the
// message schedule, 32 -> 29 without.
SV_HD uint64_t sv_pack64(uint32_t lo, uint32_t hi) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u2_t __attribute__((ext_vector_type(2)));
  const u2_t v = {lo, hi};
  return __builtin_bit_cast(uint64_t, v);
#else
  return ((uint64_t)hi << 32) | lo;
#endif
}

// Three-input bit functions as gfx950's v_bitop3_b32 (any function of three
// inputs by its 8-entry truth table, one VALU op per 32-bit half): xor3 (0x96,
// the Sigma / sigma functions) and maj (0xE8).  LLVM emits two v_xor_b32 for
// a ^ b ^ c and canonicalises every C spelling of maj to and/or/xor; the
// truth tables of both are symmetric in the operands.
SV_HD uint64_t sv_xor3_64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x96);
  return sv_pack64(lo, hi);
#else
  return a ^ b ^ c;
#endif
}
SV_HD uint32_t sv_xor3_32(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}
SV_HD uint64_t sv_maj64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0xE8);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0xE8);
  return sv_pack64(lo, hi);
#else
  return (a & b) ^ (c & (a ^ b));
#endif
}
SV_HD uint32_t sv_maj32(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
#else
  return (a & b) ^ (c & (a ^ b));
#endif
}
