// VALU issue-rate microbenchmark for the non-multiply instructions of the
// GF(2^255-19) carry chain and point formulas on gfx950 (MI355X), plus
// v_mad_u64_u32 with distinct carry-out SGPR pairs per chain.
//
// Each lane runs 8 independent chains of one instruction (rate), or the
// field carry step (v_lshrrev_b64 -> v_lshl_add_u64 -> v_and_b32) as ONE
// dependent chain (latency) and as 8 interleaved chains (rate).
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o tools/ubench_valu
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define ITERS 16384
__device__ unsigned long long g_clk[2][4096];
#define STAMP0 unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#define STAMP1                                                                               \
  if (threadIdx.x == 0) {                                                                    \
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
    g_clk[0][blockIdx.x & 4095] = t1 - t0;                                                   \
    g_clk[1][blockIdx.x & 4095] = r1 - r0;                                                   \
  }
#define CHAIN8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

#define K64(NAME, ASM)                                                   \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                   \
    uint32_t a = threadIdx.x + seed;                                     \
    uint64_t acc[8];                                                     \
    for (int i = 0; i < 8; ++i) acc[i] = ((uint64_t)a << 20) + i;        \
    STAMP0 for (int it = 0; it < ITERS; ++it) {                          \
      CHAIN8(ASM)                                                        \
    }                                                                    \
    STAMP1 uint64_t s = 0;                                               \
    for (int i = 0; i < 8; ++i) s ^= acc[i];                             \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32)); \
  }
#define K32(NAME, ASM)                                                   \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                   \
    uint32_t a = threadIdx.x + seed, b = a * 7u + 3u;                    \
    uint32_t acc[8];                                                     \
    for (int i = 0; i < 8; ++i) acc[i] = a + i;                          \
    STAMP0 for (int it = 0; it < ITERS; ++it) {                          \
      CHAIN8(ASM)                                                        \
    }                                                                    \
    STAMP1 uint32_t s = 0;                                               \
    for (int i = 0; i < 8; ++i) s ^= acc[i] + b;                         \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                      \
  }

#define X_SHR64(i) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(acc[i]));
#define X_LSHLADD(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(acc[i]));
#define X_AND(i) asm volatile("v_and_b32 %0, 0x3ffffff, %0" : "+v"(acc[i]));
#define X_ADD32(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(b));
#define X_ALIGN(i) asm volatile("v_alignbit_b32 %0, %0, %1, 26" : "+v"(acc[i]) : "v"(b));
#define X_CND(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(acc[i]) : "v"(b));
#define X_SHL32(i) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(acc[i]));
// select with a lane mask held in an ordinary SGPR pair (the form the compiler
// emits for per-lane conditions computed once), and a DPP quad broadcast
#define X_CNDS(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(acc[i]) : "v"(b) : "s40", "s41");
#define X_DPP(i) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf" : "=v"(acc[i]) : "v"(acc[(i + 1) & 7]));
#define X_MUL19(i) asm volatile("v_mul_lo_u32 %0, %0, 19" : "+v"(acc[i]));
#define X_MAD_VCC(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(acc[i]) : "v"(a) : "vcc");

K64(k_shr64, X_SHR64)
K64(k_lshladd, X_LSHLADD)
K32(k_and, X_AND)
K32(k_add32, X_ADD32)
K32(k_align, X_ALIGN)
K32(k_cnd, X_CND)
K32(k_shl32, X_SHL32)
K32(k_cnds, X_CNDS)
K32(k_dpp, X_DPP)
K32(k_mul19, X_MUL19)
K64(k_mad_vcc, X_MAD_VCC)

// 8 chains, each writing its own SGPR pair s[10i..10i+1] (s[00:01] ... s[70:71])
__global__ void k_mad_spair(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint64_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = ((uint64_t)a << 20) + i;
  STAMP0 for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_mad_u64_u32 %0, s[20:21], %1, %1, %0" : "+v"(acc[0]) : "v"(a) : "s20", "s21");
    asm volatile("v_mad_u64_u32 %0, s[22:23], %1, %1, %0" : "+v"(acc[1]) : "v"(a) : "s22", "s23");
    asm volatile("v_mad_u64_u32 %0, s[24:25], %1, %1, %0" : "+v"(acc[2]) : "v"(a) : "s24", "s25");
    asm volatile("v_mad_u64_u32 %0, s[26:27], %1, %1, %0" : "+v"(acc[3]) : "v"(a) : "s26", "s27");
    asm volatile("v_mad_u64_u32 %0, s[28:29], %1, %1, %0" : "+v"(acc[4]) : "v"(a) : "s28", "s29");
    asm volatile("v_mad_u64_u32 %0, s[30:31], %1, %1, %0" : "+v"(acc[5]) : "v"(a) : "s30", "s31");
    asm volatile("v_mad_u64_u32 %0, s[32:33], %1, %1, %0" : "+v"(acc[6]) : "v"(a) : "s32", "s33");
    asm volatile("v_mad_u64_u32 %0, s[34:35], %1, %1, %0" : "+v"(acc[7]) : "v"(a) : "s34", "s35");
  }
  STAMP1 uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}

// one carry step c = h >> 26; h' += c; h &= mask  (3 instructions), 8 chains
#define CARRY_STEP(A, T)                                                        \
  {                                                                             \
    asm volatile("v_lshrrev_b64 %1, 26, %0\n v_lshl_add_u64 %0, %0, 0, %1"    \
                 : "+v"(A), "=&v"(T));                                          \
    uint32_t lo_ = (uint32_t)(A);                                               \
    asm volatile("v_and_b32 %0, 0x3ffffff, %0" : "+v"(lo_));                    \
    A = ((A) & 0xffffffff00000000ull) | lo_;                                    \
  }
#define X_CARRY(i) CARRY_STEP(acc[i], tmp[i])
__global__ void k_carry8(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint64_t acc[8], tmp[8];
  for (int i = 0; i < 8; ++i) acc[i] = ((uint64_t)a << 20) + i;
  STAMP0 for (int it = 0; it < ITERS; ++it) {
    CHAIN8(X_CARRY)
  }
  STAMP1 uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}
// the same step as ONE dependent chain (8 steps per iteration, each on the previous)
__global__ void k_carry1(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint64_t acc[8], tmp[8];
  for (int i = 0; i < 8; ++i) acc[i] = ((uint64_t)a << 20) + i;
  STAMP0 for (int it = 0; it < ITERS; ++it) {
#define X_DEP(i) CARRY_STEP(acc[0], tmp[i])
    CHAIN8(X_DEP)
#undef X_DEP
  }
  STAMP1 uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i] ^ tmp[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}
// dependent mad chain (one accumulator)
__global__ void k_mad_dep(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint64_t acc = a;
  STAMP0 for (int it = 0; it < ITERS; ++it) {
#define X_D(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(acc) : "v"(a) : "vcc");
    CHAIN8(X_D)
#undef X_D
  }
  STAMP1 out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(acc ^ (acc >> 32));
}

typedef void (*kfn)(uint32_t*, uint32_t);
static double g_ghz = 2.4;
static double run(kfn k, uint32_t* d, int blocks, int threads, int insts_per_chain_step) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  static unsigned long long h[2][4096];
  hipMemcpyFromSymbol(h, HIP_SYMBOL(g_clk), sizeof(h));
  int nb = blocks < 4096 ? blocks : 4096;
  double sc = 0, sr = 0;
  for (int i = 0; i < nb; ++i) {
    sc += h[0][i];
    sr += h[1][i];
  }
  g_ghz = (sc / sr) * 0.1;
  const double wave_insts = (double)ITERS * 8.0 * insts_per_chain_step;
  // cycles the SIMD spends per wave-instruction = wave lifetime / (insts of all waves on the SIMD)
  const double waves_per_simd = (double)blocks * threads / 64 / (4.0 * 256);
  const double simd_cyc_per_inst = (sc / nb) / (wave_insts * waves_per_simd);
  printf(" clock %.3f GHz  SIMD cycles per wave-instruction %.2f", g_ghz, simd_cyc_per_inst);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return simd_cyc_per_inst;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("device %s CUs=%d\n", p.gcnArchName, cus);
  const int threads = 256;
  uint32_t* d;
  hipMalloc(&d, sizeof(uint32_t) * cus * 8 * threads);
  struct {
    const char* name;
    kfn k;
    int insts;
  } ks[] = {{"v_lshrrev_b64", k_shr64, 1},     {"v_lshl_add_u64", k_lshladd, 1},
            {"v_and_b32", k_and, 1},           {"v_add_u32", k_add32, 1},
            {"v_alignbit_b32", k_align, 1},    {"v_cndmask_b32", k_cnd, 1},
            {"v_lshlrev_b32", k_shl32, 1},     {"v_mad_u64_u32 (vcc)", k_mad_vcc, 1},
            {"v_cndmask_b32_e64 (sgpr mask)", k_cnds, 1}, {"v_mov_b32_dpp quad_perm", k_dpp, 1},
            {"v_mul_lo_u32 x19", k_mul19, 1},
            {"v_mad_u64_u32 (8 sgpr pairs)", k_mad_spair, 1},
            {"carry step x8 chains", k_carry8, 3}, {"carry step 1 chain", k_carry1, 3},
            {"v_mad_u64_u32 1 dep chain", k_mad_dep, 1}};
  for (int occ : {1, 2}) {
    printf("== %d waves/SIMD ==\n", occ);
    for (auto& k : ks) {
      printf("%-30s", k.name);
      run(k.k, d, cus * occ, threads, k.insts);
      printf("\n");
    }
  }
  hipFree(d);
  return 0;
}
