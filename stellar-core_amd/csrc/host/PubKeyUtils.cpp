// See PubKeyUtils.h.  Reference: /root/reference/src/crypto/SecretKey.cpp:37-61
// (cache + key), :317-339 (cache control), :435-468 (verifySig);
// /root/reference/src/util/RandomEvictionCache.h:20-245 (the cache).
#include "PubKeyUtils.h"

#include <atomic>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <unordered_map>

#include "../../../include/stellar_sigverify.h"
#include "hashes.h"

namespace stellar {
namespace {

struct HashOfHash {
  size_t operator()(Hash const& h) const {
    uint64_t v;
    std::memcpy(&v, h.data(), 8);  // keys are BLAKE2b outputs: uniformly distributed
    return (size_t)v;
  }
};

// Restatement of RandomEvictionCache<Hash, bool>(maxSize, separatePRNG=true):
// hash map plus a vector of stable entry pointers; when over capacity, pick
// two entries uniformly at random and evict the less recently accessed one.
class RandomEvictionCache {
 public:
  explicit RandomEvictionCache(size_t maxSize) : maxSize_(maxSize) {
    map_.reserve(maxSize + 1);
    ptrs_.reserve(maxSize + 1);
  }
  void maybeSeed(unsigned seed) { rng_.seed(seed); }
  bool exists(Hash const& k) const { return map_.find(k) != map_.end(); }
  bool get(Hash const& k) {
    auto& cv = map_.at(k);
    cv.lastAccess = ++generation_;
    return cv.value;
  }
  void put(Hash const& k, bool v) {
    ++generation_;
    auto pr = map_.insert({k, Value{generation_, v}});
    if (pr.second) {
      ptrs_.push_back(&*pr.first);
      if (ptrs_.size() > maxSize_) evictOne();
    } else {
      pr.first->second = Value{generation_, v};
    }
  }
  void clear() {
    ptrs_.clear();
    map_.clear();
  }
  size_t size() const { return map_.size(); }

 private:
  struct Value {
    uint64_t lastAccess;
    bool value;
  };
  using Map = std::unordered_map<Hash, Value, HashOfHash>;
  void evictOne() {
    const size_t sz = ptrs_.size();
    if (sz == 0) return;
    std::uniform_int_distribution<size_t> dist(0, sz - 1);
    Map::value_type*& a = ptrs_.at(dist(rng_));
    Map::value_type*& b = ptrs_.at(dist(rng_));
    Map::value_type*& victim = a->second.lastAccess < b->second.lastAccess ? a : b;
    map_.erase(victim->first);
    std::swap(victim, ptrs_.back());
    ptrs_.pop_back();
  }
  size_t maxSize_;
  uint64_t generation_ = 0;
  Map map_;
  std::vector<Map::value_type*> ptrs_;
  std::minstd_rand rng_;  // stellar_default_random_engine, src/util/Math.h:26
};

std::mutex gVerifySigCacheMutex;
RandomEvictionCache gVerifySigCache(0xffff);
uint64_t gVerifyCacheHit = 0;
uint64_t gVerifyCacheMiss = 0;
uint64_t gEngineSigs = 0;
uint64_t gEngineBatches = 0;
std::atomic<PubKeyUtils::BatchVerifyFn> gTestVerifier{nullptr};

Hash verifySigCacheKey(PublicKey const& key, Signature const& signature, ByteSlice const& bin) {
  hostcrypto::Blake2b256 h;
  h.add(key.ed25519().data(), 32);
  h.add(signature.data(), signature.size());
  h.add(bin.data(), bin.size());
  return h.finish();
}

// Sends the misses to the engine (GPU) in one batch.
void dispatch(std::vector<PubKeyUtils::VerifyItem const*> const& items, std::vector<uint8_t>& verdict) {
  const size_t n = items.size();
  verdict.assign(n, 0);
  if (n == 0) return;
  std::vector<uint8_t> pk(32 * n), sig(64 * n);
  std::vector<uint64_t> off(n);
  std::vector<uint32_t> len(n);
  size_t total = 0;
  bool all32 = true;
  for (size_t i = 0; i < n; ++i) {
    total += items[i]->msg.size();
    all32 = all32 && items[i]->msg.size() == 32;
  }
  std::vector<uint8_t> msg(total ? total : 1);
  size_t pos = 0;
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&pk[32 * i], items[i]->key->ed25519().data(), 32);
    std::memcpy(&sig[64 * i], items[i]->signature->data(), 64);
    off[i] = pos;
    len[i] = (uint32_t)items[i]->msg.size();
    if (len[i]) std::memcpy(&msg[pos], items[i]->msg.data(), len[i]);
    pos += len[i];
  }
  int rc;
  PubKeyUtils::BatchVerifyFn tv = gTestVerifier.load();
  if (tv) {
    rc = tv(pk.data(), sig.data(), msg.data(), off.data(), len.data(), n, verdict.data());
  } else if (all32) {
    rc = sv_ed25519_verify_batch_fixed(pk.data(), sig.data(), msg.data(), 32, n, verdict.data(), nullptr);
  } else {
    rc = sv_ed25519_verify_batch(pk.data(), sig.data(), msg.data(), off.data(), len.data(), n, verdict.data(),
                                 nullptr);
  }
  if (rc != SV_OK) {
    throw VerifyEngineError(std::string("ed25519 batch verification failed (") + std::to_string(rc) +
                            "): " + (tv ? "test verifier" : sv_last_error_string()));
  }
}

}  // namespace

namespace PubKeyUtils {

std::vector<bool> verifySigBatch(std::vector<VerifyItem> const& items) {
  const size_t n = items.size();
  std::vector<bool> out(n, false);
  std::vector<Hash> keys(n);
  std::vector<int64_t> missSlot(n, -1);  // index into `misses` for rows resolved by the engine
  std::vector<VerifyItem const*> misses;
  std::unordered_map<Hash, size_t, HashOfHash> batchFirst;  // duplicates inside this batch
  {
    std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
    for (size_t i = 0; i < n; ++i) {
      if (items[i].key->type() != PUBLIC_KEY_TYPE_ED25519)
        throw std::invalid_argument("verifySigBatch: non-ed25519 key");  // releaseAssert, SecretKey.cpp:440
      if (items[i].signature->size() != 64) continue;                   // SecretKey.cpp:441-444
      keys[i] = verifySigCacheKey(*items[i].key, *items[i].signature, items[i].msg);
      if (gVerifySigCache.exists(keys[i])) {
        ++gVerifyCacheHit;
        out[i] = gVerifySigCache.get(keys[i]);
        continue;
      }
      auto it = batchFirst.find(keys[i]);
      if (it != batchFirst.end()) {
        // a sequential caller would hit the entry its first occurrence stored
        ++gVerifyCacheHit;
        missSlot[i] = (int64_t)it->second;
        continue;
      }
      batchFirst.emplace(keys[i], misses.size());
      missSlot[i] = (int64_t)misses.size();
      misses.push_back(&items[i]);
    }
  }
  std::vector<uint8_t> verdict;
  dispatch(misses, verdict);  // outside the lock: the engine call is long
  std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
  if (!misses.empty()) {
    gEngineSigs += misses.size();
    gEngineBatches += 1;
  }
  for (size_t m = 0; m < misses.size(); ++m) {
    const size_t i = (size_t)(misses[m] - items.data());
    ++gVerifyCacheMiss;
    gVerifySigCache.put(keys[i], verdict[m] != 0);
  }
  for (size_t i = 0; i < n; ++i)
    if (missSlot[i] >= 0) out[i] = verdict[(size_t)missSlot[i]] != 0;
  return out;
}

bool verifySig(PublicKey const& key, Signature const& signature, ByteSlice const& bin) {
  std::vector<VerifyItem> one{VerifyItem{&key, &signature, bin}};
  return verifySigBatch(one)[0];
}

void clearVerifySigCache() {
  std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
  gVerifySigCache.clear();
}

void maybeSeedVerifySigCache(unsigned int seed) {
  std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
  gVerifySigCache.maybeSeed(seed);
}

void flushVerifySigCacheCounts(uint64_t& hits, uint64_t& misses) {
  std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
  hits = gVerifyCacheHit;
  misses = gVerifyCacheMiss;
  gVerifyCacheHit = 0;
  gVerifyCacheMiss = 0;
}

void setBatchVerifierForTesting(BatchVerifyFn fn) { gTestVerifier.store(fn); }

void flushEngineCounts(uint64_t& signatures, uint64_t& batches) {
  std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
  signatures = gEngineSigs;
  batches = gEngineBatches;
  gEngineSigs = 0;
  gEngineBatches = 0;
}

}  // namespace PubKeyUtils
}  // namespace stellar
