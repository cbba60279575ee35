// Developer tool: host BLAKE2b-256 of a 352-byte verify
// cache key input (pk || sig || 256-byte message, the reference's
// benchmarkOpsPerSecond shape) -- the mirror's hostcrypto::blake2b256 against
// libsodium's crypto_generichash (dlopen), ns per key, and equality.
//   g++ -O2 -std=c++17 -Istellar-core_amd/csrc/host tools/b2bench.cpp \
//       stellar-core_amd/csrc/host/hashes.cpp -ldl -o tools/b2bench
#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "hashes.h"
using namespace stellar::hostcrypto;
typedef int (*gh_t)(unsigned char*, size_t, const unsigned char*, unsigned long long, const unsigned char*, size_t);
int main(int argc, char** argv) {
  const char* lib = argc > 1 ? argv[1] : "/opt/conda/lib/libsodium.so.23";
  void* h = dlopen(lib, RTLD_NOW);
  if (!h) {
    printf("no libsodium at %s\n", lib);
    return 1;
  }
  ((int (*)())dlsym(h, "sodium_init"))();
  gh_t gh = (gh_t)dlsym(h, "crypto_generichash");
  const size_t N = 10000, L = 352;
  std::vector<uint8_t> buf(N * L);
  for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(i * 2654435761u >> 13);
  uint8_t out[32];
  double best_a = 1e9, best_b = 1e9;
  uint64_t acc = 0;
  for (int rep = 0; rep < 5; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    for (int p = 0; p < 10; ++p)
      for (size_t i = 0; i < N; ++i) {
        Hash32 x = blake2b256(&buf[i * L], L);
        acc += x[0];
      }
    auto t1 = std::chrono::steady_clock::now();
    for (int p = 0; p < 10; ++p)
      for (size_t i = 0; i < N; ++i) {
        gh(out, 32, &buf[i * L], L, nullptr, 0);
        acc += out[0];
      }
    auto t2 = std::chrono::steady_clock::now();
    best_a = std::min(best_a, std::chrono::duration<double, std::nano>(t1 - t0).count() / (10 * N));
    best_b = std::min(best_b, std::chrono::duration<double, std::nano>(t2 - t1).count() / (10 * N));
  }
  for (size_t i = 0; i < 1000; ++i) {
    for (size_t len : {(size_t)0, (size_t)1, (size_t)127, (size_t)128, (size_t)129, (size_t)255, (size_t)256, L}) {
      Hash32 x = blake2b256(&buf[i * L], std::min(len, L));
      gh(out, 32, &buf[i * L], std::min(len, L), nullptr, 0);
      if (memcmp(x.data(), out, 32)) {
        printf("MISMATCH at len %zu\n", len);
        return 1;
      }
    }
  }
  printf("{\"bytes\": %zu, \"mirror_ns\": %.1f, \"libsodium_ns\": %.1f, \"equal\": true, \"acc\": %llu}\n", L, best_a,
         best_b, (unsigned long long)(acc & 1));
  return 0;
}
