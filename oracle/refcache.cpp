// REFERENCE-SHAPE COMPARATOR -- test/bench infrastructure only (bench.py
// config1.hit_path).  Never part of the product path.
//
// Times the verify-cache HIT path the way the reference runs it, beside the
// mirror's (svh_bench_verify_hits), in the shape of the reference's
// "verify-hit benchmarking" (CryptoTests.cpp:308-316 ->
// SecretKey::benchmarkOpsPerSecond(.., 10000, 10), SecretKey.cpp:214-241):
//   PubKeyUtils::verifySig, SecretKey.cpp:435-468: the cache key is libsodium
//     BLAKE2b-256 of pk || sig || msg (verifySigCacheKey, SecretKey.cpp:50-61,
//     crypto/BLAKE2.cpp: crypto_generichash_init / update / final), then under
//     gVerifySigCacheMutex `exists(key)` followed by `get(key)`;
//   RandomEvictionCache.h: a std::unordered_map<uint256, {lastAccess, value}>
//     (plus a vector of entry pointers for the random eviction), every get
//     bumping the generation counter;
//   std::hash<uint256> (util/HashOfHash.cpp): libsodium crypto_shorthash
//     (SipHash-2-4) of the key's first 8 bytes under shortHash's gKeyMutex
//     (crypto/ShortHash.cpp computeHash) -- once per map lookup.
// A miss verifies with crypto_sign_verify_detached and puts the verdict.
// libsodium is dlopen'd (the reference links it); the verdict of every timed
// call must be true.
#include <dlfcn.h>

#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

struct Sodium {
  int (*verify)(const unsigned char*, const unsigned char*, unsigned long long, const unsigned char*) = nullptr;
  int (*gh_init)(void*, const unsigned char*, size_t, size_t) = nullptr;
  int (*gh_update)(void*, const unsigned char*, unsigned long long) = nullptr;
  int (*gh_final)(void*, unsigned char*, size_t) = nullptr;
  size_t (*gh_statebytes)(void) = nullptr;
  int (*shorthash)(unsigned char*, const unsigned char*, unsigned long long, const unsigned char*) = nullptr;
  void (*shorthash_keygen)(unsigned char*) = nullptr;
};
Sodium S;

using Key = std::array<uint8_t, 32>;
unsigned char gShortKey[16];
std::mutex gKeyMutex;  // shortHash's (ShortHash.cpp)

struct KeyHash {
  size_t operator()(Key const& k) const noexcept {
    std::lock_guard<std::mutex> g(gKeyMutex);
    uint64_t res;
    S.shorthash(reinterpret_cast<unsigned char*>(&res), k.data(), 8, gShortKey);
    return (size_t)res;
  }
};

struct Cache {
  struct Val {
    uint64_t lastAccess;
    bool value;
  };
  std::unordered_map<Key, Val, KeyHash> map;
  std::vector<std::pair<const Key, Val>*> ptrs;
  uint64_t gen = 0;
  uint64_t hits = 0, misses = 0;
  Cache() {
    map.reserve(0xffff + 1);
    ptrs.reserve(0xffff + 1);
  }
  bool exists(Key const& k) {
    const bool e = map.find(k) != map.end();
    if (!e) ++misses;
    return e;
  }
  bool get(Key const& k) {
    auto it = map.find(k);
    ++hits;
    it->second.lastAccess = ++gen;
    return it->second.value;
  }
  void put(Key const& k, bool v) {
    ++gen;
    auto it = map.find(k);
    if (it != map.end()) {
      it->second = Val{gen, v};
      return;
    }
    auto r = map.emplace(k, Val{gen, v});
    ptrs.push_back(&*r.first);
  }
};
Cache gCache;
std::mutex gCacheMutex;  // gVerifySigCacheMutex

Key cacheKey(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, size_t len) {
  alignas(64) unsigned char st[512];
  Key out;
  S.gh_init(st, nullptr, 0, 32);
  S.gh_update(st, pk, 32);
  S.gh_update(st, sig, 64);
  S.gh_update(st, msg, len);
  S.gh_final(st, out.data(), 32);
  return out;
}

bool verifySig(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, size_t len) {
  const Key k = cacheKey(pk, sig, msg, len);
  {
    std::lock_guard<std::mutex> g(gCacheMutex);
    if (gCache.exists(k)) return gCache.get(k);
  }
  const bool ok = S.verify(sig, msg, len, pk) == 0;
  std::lock_guard<std::mutex> g(gCacheMutex);
  gCache.put(k, ok);
  return ok;
}

}  // namespace

extern "C" int refcache_bench_hits(const char* sodium_path, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                                   size_t msg_len, size_t n, int passes, int threads, double* hits_per_s,
                                   double* fill_s) {
  void* h = dlopen(sodium_path, RTLD_NOW | RTLD_LOCAL);
  if (!h || passes < 2 || threads < 1) return -1;
  int (*init)(void) = (int (*)(void))dlsym(h, "sodium_init");
  S.verify = (decltype(S.verify))dlsym(h, "crypto_sign_verify_detached");
  S.gh_init = (decltype(S.gh_init))dlsym(h, "crypto_generichash_init");
  S.gh_update = (decltype(S.gh_update))dlsym(h, "crypto_generichash_update");
  S.gh_final = (decltype(S.gh_final))dlsym(h, "crypto_generichash_final");
  S.gh_statebytes = (decltype(S.gh_statebytes))dlsym(h, "crypto_generichash_statebytes");
  S.shorthash = (decltype(S.shorthash))dlsym(h, "crypto_shorthash");
  S.shorthash_keygen = (decltype(S.shorthash_keygen))dlsym(h, "crypto_shorthash_keygen");
  if (!init || init() < 0 || !S.verify || !S.gh_init || !S.gh_update || !S.gh_final || !S.shorthash ||
      !S.shorthash_keygen || !S.gh_statebytes || S.gh_statebytes() > 512)
    return -2;
  S.shorthash_keygen(gShortKey);
  {
    std::lock_guard<std::mutex> g(gCacheMutex);
    gCache.map.clear();
    gCache.ptrs.clear();
  }
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  bool ok = true;
  for (size_t i = 0; i < n; ++i) ok = verifySig(pk + 32 * i, sig + 64 * i, msg + i * msg_len, msg_len) && ok;
  const auto t1 = clk::now();
  if (fill_s) *fill_s = std::chrono::duration<double>(t1 - t0).count();
  std::atomic<bool> all{ok};
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      bool good = true;
      const size_t start = n * (size_t)t / (size_t)threads;
      for (int pass = 1; pass < passes; ++pass)
        for (size_t k = 0; k < n; ++k) {
          const size_t i = (start + k) % n;
          good = verifySig(pk + 32 * i, sig + 64 * i, msg + i * msg_len, msg_len) && good;
        }
      if (!good) all.store(false);
    });
  for (auto& x : th) x.join();
  const double dt = std::chrono::duration<double>(clk::now() - t1).count();
  *hits_per_s = (double)n * (double)(passes - 1) * (double)threads / dt;
  return all.load() ? 0 : -3;
}
