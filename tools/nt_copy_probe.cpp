#include <emmintrin.h>
#include <immintrin.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <thread>
#include <vector>
static void stream_copy(void* d, const void* s, size_t n) {
  char* dst = (char*)d; const char* src = (const char*)s;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    __m128i a = _mm_loadu_si128((const __m128i*)(src + i));
    __m128i b = _mm_loadu_si128((const __m128i*)(src + i + 16));
    __m128i c = _mm_loadu_si128((const __m128i*)(src + i + 32));
    __m128i e = _mm_loadu_si128((const __m128i*)(src + i + 48));
    _mm_stream_si128((__m128i*)(dst + i), a);
    _mm_stream_si128((__m128i*)(dst + i + 16), b);
    _mm_stream_si128((__m128i*)(dst + i + 32), c);
    _mm_stream_si128((__m128i*)(dst + i + 48), e);
  }
  if (i < n) memcpy(dst + i, src + i, n - i);
  _mm_sfence();
}
int main(int argc, char** argv) {
  int T = atoi(argv[1]); size_t N = (size_t)1 << 27;  // 128 MB
  char* src = (char*)aligned_alloc(4096, N); char* dst = (char*)aligned_alloc(4096, N);
  memset(src, 1, N); memset(dst, 2, N);
  for (int mode = 0; mode < 2; ++mode) {
    double best = 1e9;
    for (int r = 0; r < 5; ++r) {
      auto t0 = std::chrono::steady_clock::now();
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t) th.emplace_back([&, t] {
        size_t part = 1 << 18;
        for (size_t o = (size_t)t * part; o < N; o += (size_t)T * part)
          mode ? stream_copy(dst + o, src + o, part) : (void)memcpy(dst + o, src + o, part);
      });
      for (auto& x : th) x.join();
      best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    printf("T=%d %s %.1f GB/s\n", T, mode ? "stream" : "memcpy", N / best / 1e9);
  }
}
