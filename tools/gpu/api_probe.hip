// HIP runtime round-trip probe (developer tool, not part of the product):
// what a latency-lane batch pays in API and queue overhead on this box,
// independent of the verify kernels.  Every variant moves a 370 KB input
// image (a 1000-signature SCP batch) and returns 1000 verdict bytes around a
// trivial kernel; times are host wall clock, median of 200 runs.
//
//   hipcc --offload-arch=gfx950 -O2 tools/gpu/api_probe.hip -o /tmp/api_probe && /tmp/api_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
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

constexpr size_t kIn = 370 * 1024, kN = 1000;

// one thread per verdict: reads 370 B of "its" input, writes one byte
__global__ void touch_kernel(const uint8_t* in, uint8_t* out, uint32_t n, uint32_t tag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t acc = tag;
  const uint4* p = (const uint4*)(in + (size_t)i * 368);
  for (int k = 0; k < 23; ++k) acc += p[k].x ^ p[k].w;
  out[i] = (uint8_t)(acc | 1);
}
// the same, then the last workgroup to finish writes the completion flag
__global__ void touch_flag_kernel(const uint8_t* in, uint8_t* out, uint32_t n, uint32_t tag, uint32_t* count,
                                  volatile uint32_t* flag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    uint32_t acc = tag;
    const uint4* p = (const uint4*)(in + (size_t)i * 368);
    for (int k = 0; k < 23; ++k) acc += p[k].x ^ p[k].w;
    out[i] = (uint8_t)(acc | 1);
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t done = atomicAdd(count, 1u) + 1;
    if (done == gridDim.x) {
      *count = 0;
      __threadfence_system();
      *flag = tag;
    }
  }
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t hs, ns;
  CK(hipStreamCreateWithPriority(&hs, hipStreamNonBlocking, greatest));
  CK(hipStreamCreateWithFlags(&ns, hipStreamNonBlocking));
  uint8_t *h_in, *h_out, *d_in, *d_out, *m_out;
  uint32_t *d_cnt, *m_flag;
  CK(hipHostMalloc((void**)&h_in, kIn, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&h_out, 4096, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&m_out, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&m_flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipMalloc((void**)&d_in, kIn));
  CK(hipMalloc((void**)&d_out, 4096));
  CK(hipMalloc((void**)&d_cnt, 64));
  CK(hipMemset(d_cnt, 0, 64));
  memset(h_in, 7, kIn);
  *m_flag = 0;
  uint8_t* m_out_d;
  uint32_t* m_flag_d;
  CK(hipHostGetDevicePointer((void**)&m_out_d, m_out, 0));
  CK(hipHostGetDevicePointer((void**)&m_flag_d, m_flag, 0));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const dim3 grid((kN + 63) / 64), blk(64);
  const int R = 200;

  for (int si = 0; si < 2; ++si) {
    hipStream_t s = si ? ns : hs;
    const char* sn = si ? "normal" : "high-prio";
    std::vector<double> a, b, c, d, e, f, g, call_h2d, call_k, call_d2h;
    for (int r = 0; r < R + 10; ++r) {
      // A: empty-ish kernel + stream sync
      auto t0 = Clk::now();
      hipLaunchKernelGGL(touch_kernel, grid, blk, 0, s, d_in, d_out, (uint32_t)kN, (uint32_t)r);
      CK(hipStreamSynchronize(s));
      auto t1 = Clk::now();
      // B: H2D + sync
      CK(hipMemcpyAsync(d_in, h_in, kIn, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      auto t2 = Clk::now();
      // C: the lane's shape: H2D, kernel, D2H, event record, event sync
      auto c0 = Clk::now();
      CK(hipMemcpyAsync(d_in, h_in, kIn, hipMemcpyHostToDevice, s));
      auto c1 = Clk::now();
      hipLaunchKernelGGL(touch_kernel, grid, blk, 0, s, d_in, d_out, (uint32_t)kN, (uint32_t)r);
      auto c2 = Clk::now();
      CK(hipMemcpyAsync(h_out, d_out, kN, hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(ev, s));
      auto c3 = Clk::now();
      CK(hipEventSynchronize(ev));
      auto t3 = Clk::now();
      // D: H2D, kernel writes verdicts + flag into mapped host memory, host spins
      const uint32_t tag = 0x1000 + r;
      auto t4 = Clk::now();
      CK(hipMemcpyAsync(d_in, h_in, kIn, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(touch_flag_kernel, grid, blk, 0, s, d_in, m_out_d, (uint32_t)kN, tag, d_cnt, m_flag_d);
      while (__atomic_load_n(m_flag, __ATOMIC_ACQUIRE) != tag) {
      }
      auto t5 = Clk::now();
      CK(hipStreamSynchronize(s));
      // E: zero-copy input too: kernel reads the pinned image directly
      const uint32_t tag2 = 0x100000 + r;
      auto t6 = Clk::now();
      hipLaunchKernelGGL(touch_flag_kernel, grid, blk, 0, s, h_in, m_out_d, (uint32_t)kN, tag2, d_cnt, m_flag_d);
      while (__atomic_load_n(m_flag, __ATOMIC_ACQUIRE) != tag2) {
      }
      auto t7 = Clk::now();
      CK(hipStreamSynchronize(s));
      // F: H2D + kernel + D2H + hipStreamSynchronize (no event)
      auto t8 = Clk::now();
      CK(hipMemcpyAsync(d_in, h_in, kIn, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(touch_kernel, grid, blk, 0, s, d_in, d_out, (uint32_t)kN, (uint32_t)r);
      CK(hipMemcpyAsync(h_out, d_out, kN, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      auto t9 = Clk::now();
      // G: H2D + kernel + D2H, spin on hipEventQuery
      auto ta = Clk::now();
      CK(hipMemcpyAsync(d_in, h_in, kIn, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(touch_kernel, grid, blk, 0, s, d_in, d_out, (uint32_t)kN, (uint32_t)r);
      CK(hipMemcpyAsync(h_out, d_out, kN, hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(ev, s));
      while (hipEventQuery(ev) == hipErrorNotReady) {
      }
      auto tb = Clk::now();
      if (r < 10) continue;
      a.push_back(us(t0, t1));
      b.push_back(us(t1, t2));
      c.push_back(us(c0, t3));
      call_h2d.push_back(us(c0, c1));
      call_k.push_back(us(c1, c2));
      call_d2h.push_back(us(c2, c3));
      d.push_back(us(t4, t5));
      e.push_back(us(t6, t7));
      f.push_back(us(t8, t9));
      g.push_back(us(ta, tb));
    }
    printf("[%s] kernel+streamsync %.1f | H2D370K+sync %.1f | lane shape (H2D,k,D2H,evsync) %.1f "
           "[calls: h2d %.1f launch %.1f d2h+rec %.1f] | H2D,k->mapped+spin %.1f | zero-copy in+out spin %.1f | "
           "H2D,k,D2H,streamsync %.1f | H2D,k,D2H,eventquery-spin %.1f us\n",
           sn, median(a), median(b), median(c), median(call_h2d), median(call_k), median(call_d2h), median(d),
           median(e), median(f), median(g));
  }
  // verdict sanity
  for (size_t i = 0; i < kN; ++i)
    if (!(m_out[i] & 1)) {
      printf("bad mapped verdict %zu\n", i);
      return 1;
    }
  return 0;
}
