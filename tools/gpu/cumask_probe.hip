// CU-reservation probe (developer tool, not part of the product): can a
// short high-priority kernel start while a long kernel holds the GPU?
//
// A "bulk" kernel whose workgroups each take a whole CU's LDS (one per CU)
// spins for ~30 ms on every CU it may use; a "latency" kernel of 16
// workgroups needing 64 KiB LDS each is launched on a high-priority stream a
// few ms later and its host round trip is timed.  Variants: the bulk stream
// with a full CU mask, and with the top R mask bits cleared (CUs reserved for
// the latency stream).
//
//   hipcc --offload-arch=gfx950 -O2 tools/gpu/cumask_probe.hip -o tools/gpu/cumask_probe.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

using Clk = std::chrono::steady_clock;
static double us(Clk::time_point a, Clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

// s_memrealtime runs at 100 MHz
__device__ __forceinline__ uint64_t rt() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(256) void bulk_kernel(uint32_t* out, uint64_t ticks) {
  extern __shared__ uint32_t lds[];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint64_t t0 = rt();
  uint32_t acc = lds[(threadIdx.x + 1) & 255];
  while (rt() - t0 < ticks) acc = acc * 1664525u + 1013904223u;
  if (acc == 0x12345678u) out[blockIdx.x] = acc;  // (keeps the loop)
}

__global__ __launch_bounds__(256) void lat_kernel(uint32_t* out, uint32_t tag) {
  extern __shared__ uint32_t lds[];
  lds[threadIdx.x] = tag + threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[64 + blockIdx.x] = lds[255];
}

int main(int argc, char** argv) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  size_t lds_max = 0;
  {
    int v = 0;
    CK(hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 0));
    lds_max = (size_t)v;
  }
  printf("CUs %d, LDS per CU %zu\n", cus, lds_max);
  CK(hipFuncSetAttribute((const void*)bulk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
  CK(hipFuncSetAttribute((const void*)lat_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t hs, extra[4];
  CK(hipStreamCreateWithPriority(&hs, hipStreamNonBlocking, greatest));
  for (auto& s : extra) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));  // (engine-like stream count)
  uint32_t* d;
  CK(hipMalloc((void**)&d, 4096));
  const uint64_t ticks = 3000000;  // 30 ms
  const int reserves[] = {0, 8, 16, 32, 64};
  for (int R : reserves) {
    hipStream_t bs;
    std::vector<uint32_t> mask((cus + 31) / 32, 0);
    for (int c = 0; c < cus - R; ++c) mask[c / 32] |= 1u << (c % 32);
    if (R == 0) CK(hipStreamCreateWithFlags(&bs, hipStreamNonBlocking));
    else CK(hipExtStreamCreateWithCUMask(&bs, (uint32_t)mask.size(), mask.data()));
    std::vector<double> lat, bulk;
    for (int it = 0; it < 6; ++it) {
      auto b0 = Clk::now();
      hipLaunchKernelGGL(bulk_kernel, dim3(2 * cus), dim3(256), lds_max, bs, d, ticks);
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
      auto t0 = Clk::now();
      hipLaunchKernelGGL(lat_kernel, dim3(16), dim3(256), 65536, hs, d, (uint32_t)it);
      CK(hipStreamSynchronize(hs));
      auto t1 = Clk::now();
      CK(hipStreamSynchronize(bs));
      auto b1 = Clk::now();
      if (it) {
        lat.push_back(us(t0, t1));
        bulk.push_back(us(b0, b1));
      }
    }
    std::sort(lat.begin(), lat.end());
    std::sort(bulk.begin(), bulk.end());
    printf("reserve %2d CUs: latency kernel round trip median %.1f us (max %.1f), bulk call %.1f ms\n", R,
           lat[lat.size() / 2], lat.back(), bulk[bulk.size() / 2] / 1e3);
    CK(hipStreamDestroy(bs));
  }
  return 0;
}
