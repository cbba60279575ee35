// See PubKeyUtils.h.  Reference: /root/reference/src/crypto/SecretKey.cpp:37-61
// (cache + key), :317-339 (cache control), :435-468 (verifySig);
// /root/reference/src/util/RandomEvictionCache.h:20-245 (the cache).
#include "PubKeyUtils.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <random>
#include <string>

#include "../../../include/stellar_sigverify.h"
#include "hashes.h"

namespace stellar {
namespace {


inline uint64_t keyBits(Hash const& h) {
  uint64_t v;
  std::memcpy(&v, h.data(), 8);  // keys are BLAKE2b outputs: uniformly distributed
  return v;
}

// Restatement of RandomEvictionCache<Hash, bool>(maxSize, separatePRNG=true):
// entries plus a vector of entry references in insertion order (the
// reference's mValuePtrs); when over capacity, pick two positions of that
// vector uniformly at random, evict the less recently accessed entry and
// swap-remove its position -- the same draws and the same victims as the
// reference.  The key -> entry index is a flat linear-probing table
// (backward-shift deletion) instead of a node-based map: no allocation per
// insert/evict, which keeps large verifySigBatch calls from being bound by
// the allocator.
class RandomEvictionCache {
 public:
  explicit RandomEvictionCache(size_t maxSize) : maxSize_(maxSize) {
    size_t cap = 16;
    while (cap < 2 * (maxSize + 1)) cap <<= 1;
    table_.assign(cap, 0u);
    mask_ = cap - 1;
    entries_.reserve(maxSize + 1);
    order_.reserve(maxSize + 1);
  }
  void maybeSeed(unsigned seed) { rng_.seed(seed); }
  // Hint for a lookup a few items ahead (memory-level parallelism).
  void prefetch(Hash const& k) const { __builtin_prefetch(&table_[keyBits(k) & mask_]); }
  bool exists(Hash const& k) const { return find(k) != kNone; }
  bool get(Hash const& k) {
    Entry& e = entries_[find(k)];
    e.lastAccess = ++generation_;
    return e.value;
  }
  void put(Hash const& k, bool v) {
    ++generation_;
    const uint32_t id = find(k);
    if (id != kNone) {
      entries_[id].lastAccess = generation_;
      entries_[id].value = v;
      return;
    }
    uint32_t nid;
    if (!freeIds_.empty()) {
      nid = freeIds_.back();
      freeIds_.pop_back();
      entries_[nid] = Entry{k, generation_, v};
    } else {
      nid = (uint32_t)entries_.size();
      entries_.push_back(Entry{k, generation_, v});
    }
    insertSlot(k, nid);
    order_.push_back(nid);
    if (order_.size() > maxSize_) evictOne();
  }
  void clear() {
    std::fill(table_.begin(), table_.end(), 0u);
    entries_.clear();
    freeIds_.clear();
    order_.clear();
  }
  size_t size() const { return order_.size(); }

 private:
  static constexpr uint32_t kNone = 0xffffffffu;
  struct Entry {
    Hash key;
    uint64_t lastAccess;
    bool value;
  };
  // slot = (tag << 32) | (entry id + 1), 0 = empty; the tag (key bits 32..63)
  // settles almost every mismatch without touching the entry slab
  static uint64_t tagOf(Hash const& k) { return keyBits(k) >> 32; }
  uint32_t find(Hash const& k) const {
    const uint64_t tag = tagOf(k);
    for (size_t s = keyBits(k) & mask_;; s = (s + 1) & mask_) {
      const uint64_t t = table_[s];
      if (t == 0) return kNone;
      if ((t >> 32) == tag && entries_[(uint32_t)t - 1].key == k) return (uint32_t)t - 1;
    }
  }
  void insertSlot(Hash const& k, uint32_t id) {
    size_t s = keyBits(k) & mask_;
    while (table_[s] != 0) s = (s + 1) & mask_;
    table_[s] = (tagOf(k) << 32) | (uint64_t)(id + 1);
  }
  void eraseSlot(Hash const& k, uint32_t id) {
    size_t s = keyBits(k) & mask_;
    while ((uint32_t)table_[s] != id + 1) s = (s + 1) & mask_;
    // backward-shift deletion keeps every probe chain intact
    size_t hole = s;
    for (size_t j = (hole + 1) & mask_; table_[j] != 0; j = (j + 1) & mask_) {
      const size_t home = keyBits(entries_[(uint32_t)table_[j] - 1].key) & mask_;
      if (((j - home) & mask_) >= ((j - hole) & mask_)) {
        table_[hole] = table_[j];
        hole = j;
      }
    }
    table_[hole] = 0;
  }
  void evictOne() {
    const size_t sz = order_.size();
    if (sz == 0) return;
    std::uniform_int_distribution<size_t> dist(0, sz - 1);
    const size_t ia = dist(rng_);
    const size_t ib = dist(rng_);
    const size_t iv = entries_[order_[ia]].lastAccess < entries_[order_[ib]].lastAccess ? ia : ib;
    const uint32_t victim = order_[iv];
    eraseSlot(entries_[victim].key, victim);
    freeIds_.push_back(victim);
    std::swap(order_[iv], order_.back());
    order_.pop_back();
  }
  size_t maxSize_;
  size_t mask_;
  uint64_t generation_ = 0;
  std::vector<uint64_t> table_;
  std::vector<Entry> entries_;
  std::vector<uint32_t> freeIds_;
  std::vector<uint32_t> order_;
  std::minstd_rand rng_;  // stellar_default_random_engine, src/util/Math.h:26
};

// First occurrence of each key inside one batch (flat linear probing).
class BatchFirstIndex {
 public:
  static constexpr uint32_t kNone = 0xffffffffu;
  explicit BatchFirstIndex(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 2) cap <<= 1;
    slot_.assign(cap, 0u);
    mask_ = cap - 1;
  }
  // Position in `firstRows` of the first row whose key equals keys[row]; if
  // there is none, appends `row` to firstRows and returns kNone.
  uint32_t findOrAdd(std::vector<Hash> const& keys, size_t row, std::vector<size_t>& firstRows) {
    Hash const& k = keys[row];
    for (size_t s = keyBits(k) & mask_;; s = (s + 1) & mask_) {
      if (slot_[s] == 0) {
        slot_[s] = (uint32_t)firstRows.size() + 1;
        firstRows.push_back(row);
        return kNone;
      }
      if (keys[firstRows[slot_[s] - 1]] == k) return slot_[s] - 1;
    }
  }

 private:
  size_t mask_;
  std::vector<uint32_t> slot_;  // position in firstRows + 1; 0 = empty
};

std::mutex gVerifySigCacheMutex;
RandomEvictionCache gVerifySigCache(0xffff);
uint64_t gVerifyCacheHit = 0;
uint64_t gVerifyCacheMiss = 0;
uint64_t gEngineSigs = 0;
uint64_t gEngineBatches = 0;
std::atomic<PubKeyUtils::BatchVerifyFn> gTestVerifier{nullptr};
std::atomic<PubKeyUtils::KeyedBatchVerifyFn> gTestKeyedVerifier{nullptr};
std::atomic<size_t> gKeyedThreshold{4096};

Hash verifySigCacheKey(PublicKey const& key, Signature const& signature, ByteSlice const& bin) {
  hostcrypto::Blake2b256 h;
  h.add(key.ed25519().data(), 32);
  h.add(signature.data(), signature.size());
  h.add(bin.data(), bin.size());
  return h.finish();
}

// Per-thread staging for engine calls: reused across calls so a large batch
// does not pay fresh page faults for ~200 B/signature of packing buffers.
struct Staging {
  std::vector<uint8_t> pk, sig, msg;
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
};
Staging& staging() {
  static thread_local Staging st;
  return st;
}

// Sends `items` to the engine (GPU) in one batch.  With `keys` non-null the
// engine also returns each item's BLAKE2b cache key (keyed pass, f4), written
// to keys[0..n) (Hash is 32 contiguous bytes).
void dispatch(std::vector<PubKeyUtils::VerifyItem const*> const& items, std::vector<uint8_t>& verdict,
              Hash* keys = nullptr) {
  const size_t n = items.size();
  verdict.assign(n, 0);
  if (n == 0) return;
  Staging& st = staging();
  st.pk.resize(32 * n);
  st.sig.resize(64 * n);
  st.off.resize(n);
  st.len.resize(n);
  size_t total = 0;
  bool all32 = true;
  for (size_t i = 0; i < n; ++i) {
    total += items[i]->msg.size();
    all32 = all32 && items[i]->msg.size() == 32;
  }
  st.msg.resize(total ? total : 1);
  size_t pos = 0;
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&st.pk[32 * i], items[i]->key->ed25519().data(), 32);
    std::memcpy(&st.sig[64 * i], items[i]->signature->data(), 64);
    st.off[i] = pos;
    st.len[i] = (uint32_t)items[i]->msg.size();
    if (st.len[i]) std::memcpy(&st.msg[pos], items[i]->msg.data(), st.len[i]);
    pos += st.len[i];
  }
  int rc;
  bool testing = false;
  static_assert(sizeof(Hash) == 32, "Hash must be 32 contiguous bytes");
  if (keys) {
    uint8_t* kb = reinterpret_cast<uint8_t*>(keys);
    PubKeyUtils::KeyedBatchVerifyFn tk = gTestKeyedVerifier.load();
    testing = tk != nullptr;
    rc = tk ? tk(st.pk.data(), st.sig.data(), st.msg.data(), st.off.data(), st.len.data(), n, verdict.data(), kb)
            : sv_ed25519_verify_batch_keyed(st.pk.data(), st.sig.data(), st.msg.data(), st.off.data(),
                                            st.len.data(), n, verdict.data(), kb, nullptr);
  } else {
    PubKeyUtils::BatchVerifyFn tv = gTestVerifier.load();
    testing = tv != nullptr;
    if (tv) {
      rc = tv(st.pk.data(), st.sig.data(), st.msg.data(), st.off.data(), st.len.data(), n, verdict.data());
    } else if (all32) {
      rc = sv_ed25519_verify_batch_fixed(st.pk.data(), st.sig.data(), st.msg.data(), 32, n, verdict.data(),
                                         nullptr);
    } else {
      rc = sv_ed25519_verify_batch(st.pk.data(), st.sig.data(), st.msg.data(), st.off.data(), st.len.data(), n,
                                   verdict.data(), nullptr);
    }
  }
  if (rc != SV_OK) {
    throw VerifyEngineError(std::string("ed25519 batch verification failed (") + std::to_string(rc) +
                            "): " + (testing ? "test verifier" : sv_last_error_string()));
  }
}

}  // namespace

namespace PubKeyUtils {

std::vector<bool> verifySigBatch(std::vector<VerifyItem> const& items) {
  const size_t n = items.size();
  std::vector<bool> out(n, false);
  std::vector<Hash> keys(n);
  std::vector<VerifyItem const*> eligible;
  std::vector<size_t> eligibleRow;
  for (size_t i = 0; i < n; ++i) {
    if (items[i].key->type() != PUBLIC_KEY_TYPE_ED25519)
      throw std::invalid_argument("verifySigBatch: non-ed25519 key");  // releaseAssert, SecretKey.cpp:440
    if (items[i].signature->size() != 64) continue;                   // SecretKey.cpp:441-444
    eligible.push_back(&items[i]);
    eligibleRow.push_back(i);
  }
  const size_t thr = gKeyedThreshold.load();
  const bool keyed = thr != 0 && eligible.size() >= thr && gTestVerifier.load() == nullptr;
  std::vector<uint8_t> keyedVerdict;
  if (keyed) {
    // one engine pass over every eligible row: verdicts + cache keys (f4)
    if (eligible.size() == n) {
      dispatch(eligible, keyedVerdict, keys.data());
    } else {
      std::vector<Hash> ek(eligible.size());
      dispatch(eligible, keyedVerdict, ek.data());
      for (size_t e = 0; e < eligible.size(); ++e) keys[eligibleRow[e]] = ek[e];
    }
  } else {
    // hashed outside the cache lock
    for (size_t r : eligibleRow) keys[r] = verifySigCacheKey(*items[r].key, *items[r].signature, items[r].msg);
  }
  std::vector<int64_t> missSlot(n, -1);  // index into `misses` for rows resolved by the engine
  std::vector<size_t> misses;            // row of each distinct miss
  {
    BatchFirstIndex batchFirst(eligibleRow.size());  // duplicates inside this batch
    std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
    for (size_t e = 0; e < eligibleRow.size(); ++e) {
      const size_t i = eligibleRow[e];
      if (e + 8 < eligibleRow.size()) gVerifySigCache.prefetch(keys[eligibleRow[e + 8]]);
      if (gVerifySigCache.exists(keys[i])) {
        ++gVerifyCacheHit;
        out[i] = gVerifySigCache.get(keys[i]);
        continue;
      }
      const uint32_t first = batchFirst.findOrAdd(keys, i, misses);
      if (first != BatchFirstIndex::kNone) {
        // a sequential caller would hit the entry its first occurrence stored
        ++gVerifyCacheHit;
        missSlot[i] = (int64_t)first;
        continue;
      }
      missSlot[i] = (int64_t)(misses.size() - 1);
    }
    if (keyed) {
      // verdicts are already here: finish under the same lock
      std::vector<uint8_t> rowVerdict(n, 0);
      for (size_t e = 0; e < eligible.size(); ++e) rowVerdict[eligibleRow[e]] = keyedVerdict[e];
      gEngineSigs += eligible.size();
      gEngineBatches += 1;
      for (size_t m : misses) {
        ++gVerifyCacheMiss;
        gVerifySigCache.put(keys[m], rowVerdict[m] != 0);
      }
      for (size_t i = 0; i < n; ++i)
        if (missSlot[i] >= 0) out[i] = rowVerdict[misses[(size_t)missSlot[i]]] != 0;
      return out;
    }
  }
  std::vector<VerifyItem const*> missItems;
  missItems.reserve(misses.size());
  for (size_t m : misses) missItems.push_back(&items[m]);
  std::vector<uint8_t> verdict;
  dispatch(missItems, verdict);  // outside the lock: the engine call is long
  std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
  if (!misses.empty()) {
    gEngineSigs += misses.size();
    gEngineBatches += 1;
  }
  for (size_t m = 0; m < misses.size(); ++m) {
    ++gVerifyCacheMiss;
    gVerifySigCache.put(keys[misses[m]], verdict[m] != 0);
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
void setKeyedBatchVerifierForTesting(KeyedBatchVerifyFn fn) { gTestKeyedVerifier.store(fn); }
void setKeyedBatchThreshold(size_t minItems) { gKeyedThreshold.store(minItems); }

void flushEngineCounts(uint64_t& signatures, uint64_t& batches) {
  std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
  signatures = gEngineSigs;
  batches = gEngineBatches;
  gEngineSigs = 0;
  gEngineBatches = 0;
}

}  // namespace PubKeyUtils
}  // namespace stellar
