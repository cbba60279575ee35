#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
// where does global_load_lds_dwordx4 with an immediate offset write in LDS?
__global__ __launch_bounds__(64) void k(const uint32_t* src, uint32_t* out) {
  __shared__ uint32_t lds[64 * 4 * 12];
  for (int i = threadIdx.x; i < 64 * 4 * 12; i += 64) lds[i] = 0xdeadbeef;
  __syncthreads();
  const uint32_t lane = threadIdx.x;
  const uint32_t* base = src + lane * 40;  // lane's 160-B entry
#define G(q) __builtin_amdgcn_global_load_lds((const void*)base, (__attribute__((address_space(3))) void*)(lds + q * 256), 16, q * 16, 0);
  G(0) G(1) G(2) G(3) G(4) G(5) G(6) G(7) G(8) G(9)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 4 * 12; i += 64) out[i] = lds[i];
}
int main() {
  uint32_t h[64 * 40];
  for (int i = 0; i < 64 * 40; ++i) h[i] = i;
  uint32_t *dsrc, *dout;
  hipMalloc(&dsrc, sizeof h);
  hipMalloc(&dout, 64 * 4 * 12 * 4);
  hipMemcpy(dsrc, h, sizeof h, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dsrc, dout);
  static uint32_t o[64 * 4 * 12];
  hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
  // H1: quad q of lane L at dword (q*64 + L)*4 holds src[L*40 + q*4 .. +3]
  int h1 = 0, h2 = 0;
  for (int q = 0; q < 10; ++q)
    for (int L = 0; L < 64; ++L)
      for (int d = 0; d < 4; ++d) {
        if (o[(q * 64 + L) * 4 + d] == (uint32_t)(L * 40 + q * 4 + d)) ++h1;
        const int a2 = (q * 64 + L) * 4 + q * 4 + d;
        if (a2 < 64 * 4 * 12 && o[a2] == (uint32_t)(L * 40 + q * 4 + d)) ++h2;
      }
  printf("H1 (offset on global only) matches %d / 2560; H2 (offset on both) %d / 2560\n", h1, h2);
  printf("o[0..7] = %x %x %x %x %x %x %x %x\n", o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]);
  printf("o[256..263] = %x %x %x %x %x %x %x %x\n", o[256], o[257], o[258], o[259], o[260], o[261], o[262], o[263]);
  return 0;
}
