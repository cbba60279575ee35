// Integer / FP64 multiply throughput microbenchmark for gfx950 (MI355X).
//
// Measures the per-chip issue rate of the instructions a GF(2^255-19) field
// multiply can be built from, so the roofline peak used in bench.py is a
// measured number and not an assumption. Each lane runs 8 independent
// dependency chains of one instruction kind; the grid fills every SIMD.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_imul.hip -o tools/ubench_imul
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 32768
__device__ unsigned long long g_clk[2][4096];
#define STAMP0 unsigned long long t0=__builtin_amdgcn_s_memtime(), r0=__builtin_amdgcn_s_memrealtime();
#define STAMP1 if(threadIdx.x==0){unsigned long long t1=__builtin_amdgcn_s_memtime(), r1=__builtin_amdgcn_s_memrealtime(); g_clk[0][blockIdx.x&4095]=t1-t0; g_clk[1][blockIdx.x&4095]=r1-r0;}

#define CHAIN8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

__global__ void k_mad_u64_u32(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed, b = a * 3u + 1u;
  uint64_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  STAMP0
  for (int it = 0; it < ITERS; ++it) {
#define X(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "vcc");
    CHAIN8(X)
#undef X
  }
  STAMP1
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}

__global__ void k_mul_lo_u32(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  STAMP0
  for (int it = 0; it < ITERS; ++it) {
#define X(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
    CHAIN8(X)
#undef X
  }
  STAMP1
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_hi_u32(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  STAMP0
  for (int it = 0; it < ITERS; ++it) {
#define X(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
    CHAIN8(X)
#undef X
  }
  STAMP1
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad_u32_u24(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  STAMP0
  for (int it = 0; it < ITERS; ++it) {
#define X(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(acc[i]) : "v"(a));
    CHAIN8(X)
#undef X
  }
  STAMP1
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_hi_u32_u24(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  STAMP0
  for (int it = 0; it < ITERS; ++it) {
#define X(i) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
    CHAIN8(X)
#undef X
  }
  STAMP1
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add_co_u32(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  STAMP0
  for (int it = 0; it < ITERS; ++it) {
#define X(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(acc[i]) : "v"(a) : "vcc");
    CHAIN8(X)
#undef X
  }
  STAMP1
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addc_co_u32(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  STAMP0
  for (int it = 0; it < ITERS; ++it) {
#define X(i) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[i]) : "v"(a) : "vcc");
    CHAIN8(X)
#undef X
  }
  STAMP1
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma_f64(uint32_t* out, uint32_t seed) {
  double a = 1.0 + 1e-9 * (threadIdx.x + seed);
  double acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  STAMP0
  for (int it = 0; it < ITERS; ++it) {
#define X(i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(acc[i]) : "v"(a));
    CHAIN8(X)
#undef X
  }
  STAMP1
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)__double2loint(s);
}

__global__ void k_fma_f32(uint32_t* out, uint32_t seed) {
  float a = 1.0f + 1e-6f * (threadIdx.x + seed);
  float acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  STAMP0
  for (int it = 0; it < ITERS; ++it) {
#define X(i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(acc[i]) : "v"(a));
    CHAIN8(X)
#undef X
  }
  STAMP1
  float s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(s);
}

typedef void (*kfn)(uint32_t*, uint32_t);
static double g_last_ghz = 2.4;

static double run(kfn k, uint32_t* d, int blocks, int threads) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u);  // warm
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  double ops = 5.0 * blocks * threads * (double)ITERS * 8.0;
  static unsigned long long h[2][4096];
  hipMemcpyFromSymbol(h, HIP_SYMBOL(g_clk), sizeof(h));
  int nb = blocks < 4096 ? blocks : 4096;
  double sc = 0, sr = 0;
  for (int i = 0; i < nb; ++i) { sc += h[0][i]; sr += h[1][i]; }
  double ghz = (sc / sr) * 0.1;  // memrealtime ticks at 100 MHz
  double cyc_per_inst = (sc / nb) / (ITERS * 8.0);
  printf("   in-kernel clock %.3f GHz, wave-cycles per instruction %.2f (waves/SIMD=%d) ",
         ghz, cyc_per_inst, blocks * threads / 64 / (4 * 256));
  g_last_ghz = ghz;
  return ops / (ms * 1e-3);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  int cus = p.multiProcessorCount;
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, cus, p.clockRate);
  int threads = 256;
  int blocks = cus * 8;  // 8 waves/SIMD
  uint32_t* d;
  hipMalloc(&d, sizeof(uint32_t) * blocks * threads);
  struct { const char* name; kfn k; } ks[] = {
      {"v_mad_u64_u32", k_mad_u64_u32}, {"v_mul_lo_u32", k_mul_lo_u32},
      {"v_mul_hi_u32", k_mul_hi_u32},   {"v_mad_u32_u24", k_mad_u32_u24},
      {"v_mul_hi_u32_u24", k_mul_hi_u32_u24}, {"v_add_co_u32", k_add_co_u32},
      {"v_addc_co_u32", k_addc_co_u32}, {"v_fma_f64", k_fma_f64},
      {"v_fma_f32", k_fma_f32}};
  for (int occ : {1, 2, 4, 8}) {
    int nblk = cus * occ;
    printf("== %d waves/SIMD ==\n", occ);
    for (auto& k : ks) {
      printf("%-18s", k.name);
      double r = run(k.k, d, nblk, threads);
      printf(" %.3e lane-ops/s = %.1f lane-ops/clk/CU at measured clock\n", r, r / (cus * g_last_ghz * 1e9));
    }
  }
  hipFree(d);
  return 0;
}
