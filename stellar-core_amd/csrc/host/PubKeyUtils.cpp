// See PubKeyUtils.h.  Reference: /root/reference/src/crypto/SecretKey.cpp:37-61
// (cache + key), :317-339 (cache control), :435-468 (verifySig);
// /root/reference/src/util/RandomEvictionCache.h:20-245 (the cache);
// /root/reference/lib/util/stdrandom.h (the pinned uniform_int_distribution).
#include "PubKeyUtils.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <functional>
#include <limits>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <random>
#include <string>
#include <thread>

#include "../../../include/stellar_sigverify.h"
#include "../pool.h"
#include "HostPool.h"
#include "KeyMemo.h"
#include "hashes.h"

namespace stellar {
namespace {

sv::Pool& hostPool() {
  static sv::Pool p(std::min(8u, std::max(2u, std::thread::hardware_concurrency())));
  return p;
}

// Runs fn(i) for i in [0, n) over up to `maxParts` pool tasks (serially for
// small n).
template <class F>
void parallelFor(size_t n, size_t grain, F fn) {
  const size_t parts = std::max<size_t>(1, std::min<size_t>(hostPool().size() + 1, n / std::max<size_t>(1, grain)));
  if (parts == 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  hostPool().run(parts, [&](size_t t) {
    const size_t a = n * t / parts, b = n * (t + 1) / parts;
    for (size_t i = a; i < b; ++i) fn(i);
  });
}

// uniform_int_distribution<size_t>(lo, hi)(g) exactly as libc++ computes it
// (the algorithm stellar-core pins in lib/util/stdrandom.h so results do not
// vary between standard libraries), for std::minstd_rand -- the reference's
// stellar_default_random_engine (src/util/Math.h:26), whose result_type is a
// 64-bit unsigned long on this ABI.  The draw builds a w-bit number (w =
// bits of the range) from engine outputs: n outputs of w0 bits (n0 of them)
// or w0 + 1 bits, each rejection-sampled below the largest multiple of 2^w0
// (2^(w0+1)) within the engine range, and the whole is rejected while >= the
// range.
// The draw's parameters depend only on (lo, hi), so they are computed once
// (a cache draws over the same range for every eviction: the divisions below
// were most of an eviction's cost).
struct UniformDraw {
  using U = uint64_t;
  static constexpr size_t Dt = 64;
  size_t lo = 0, n = 0, n0 = 0, w0 = 0;
  U r = 1, y0 = 0, y1 = 0, mask0 = 0, mask1 = 0;
  UniformDraw() = default;
  UniformDraw(size_t lo_, size_t hi) : lo(lo_) {
    r = (U)hi - (U)lo + 1;
    if (r == 1) return;
    size_t w;
    if (r == 0) {
      w = Dt;
    } else {
      w = Dt - (size_t)__builtin_clzll(r) - 1;
      if ((r & (std::numeric_limits<U>::max() >> (Dt - w))) != 0) ++w;
    }
    const U R = (U)std::minstd_rand::max() - (U)std::minstd_rand::min() + 1;  // 2^31 - 2
    const size_t m = 63 - (size_t)__builtin_clzll(R);                        // floor(log2 R) = 30
    n = w / m + (w % m != 0);
    w0 = w / n;
    y0 = w0 < Dt ? (R >> w0) << w0 : 0;
    if (R - y0 > y0 / n) {
      ++n;
      w0 = w / n;
      y0 = w0 < Dt ? (R >> w0) << w0 : 0;
    }
    n0 = n - w % n;
    y1 = w0 < Dt - 1 ? (R >> (w0 + 1)) << (w0 + 1) : 0;
    mask0 = w0 > 0 ? ~U(0) >> (Dt - w0) : U(0);
    mask1 = w0 < Dt - 1 ? ~U(0) >> (Dt - (w0 + 1)) : ~U(0);
  }
  U bits(std::minstd_rand& g) const {
    U s = 0;
    for (size_t k = 0; k < n0; ++k) {
      U u;
      do {
        u = (U)g() - (U)std::minstd_rand::min();
      } while (u >= y0);
      s = w0 < Dt ? (s << w0) : 0;
      s += u & mask0;
    }
    for (size_t k = n0; k < n; ++k) {
      U u;
      do {
        u = (U)g() - (U)std::minstd_rand::min();
      } while (u >= y1);
      s = w0 < Dt - 1 ? (s << (w0 + 1)) : 0;
      s += u & mask1;
    }
    return s;
  }
  size_t operator()(std::minstd_rand& g) const {
    if (r == 1) return lo;
    if (r == 0) return (size_t)bits(g);
    U u;
    do {
      u = bits(g);
    } while (u >= r);
    return (size_t)(u + lo);
  }
};
inline uint64_t keyBits(Hash const& h) {
  uint64_t v;
  std::memcpy(&v, h.data(), 8);  // keys are BLAKE2b outputs: uniformly distributed
  return v;
}

// Restatement of RandomEvictionCache<Hash, bool>(maxSize, separatePRNG=true):
// entries plus a vector of entry references in insertion order (the
// reference's mValuePtrs); when over capacity, draw two positions of that
// vector (UniformDraw above, the reference's rand_uniform), evict the less
// recently accessed entry and swap-remove its position.  get() and put() bump
// a generation counter exactly as maybeGet()/put() do.
//
// Layout (the batch walk is a long serial chain of these operations, so it is
// built to miss in cache as rarely as possible):
//   table_   key -> entry id, flat linear probing with backward-shift deletion,
//            at load <= 1/8 (4 MB for the 0xffff cache: against load 1/2 the
//            batch walk's probe runs and shifts are short enough to cut its
//            time by ~35 %, profiles/r03/walk_pieces/);
//            a slot holds the key's low 32 bits (home position + tag that
//            settles almost every mismatch) and the entry id + 1;
//   per insertion-order position: the entry id, its key's low 32 bits and its
//            last-access generation -- so an eviction (two draws, compare,
//            unlink) reads only these 1 MB of arrays and the table, never the
//            32-byte keys;
//   entries_ key, value, pending owner, back-pointer to the position.
//
// Pending entries: a non-keyed verifySigBatch inserts its misses in item
// order BEFORE verifying them (the value is filled in afterwards), so the
// draws, generations and victims are those of sequential verifySig calls.  A
// pending entry of another batch reads as a miss (that caller verifies and
// puts it itself, as concurrent verifySig calls would).
class RandomEvictionCache {
 public:
  static constexpr uint32_t kNone = 0xffffffffu;
  struct Entry {
    Hash key;
    uint64_t owner;  // != 0: pending, value not known yet (batch id)
    uint32_t pendIdx;
    uint32_t pos;    // index in the insertion-order arrays
    bool value;
  };

  explicit RandomEvictionCache(size_t maxSize) : maxSize_(maxSize), draw_(0, maxSize) {
    size_t cap = 16;
    while (cap < 8 * (maxSize + 1)) cap <<= 1;
    table_.assign(cap, 0u);
    mask_ = cap - 1;
    entries_.reserve(maxSize + 1);
    ordId_.reserve(maxSize + 1);
    ordTag_.reserve(maxSize + 1);
    ordGen_.reserve(maxSize + 1);
  }
  void maybeSeed(unsigned seed) {
    rng_.seed(seed);
    fcount_ = 0;  // the queued draws came from the old seed
  }
  // Queues the draws of up to `evictions` future evictions (at most as many
  // as `items` inserts could cause); returns how many are queued.
  size_t preDraw(size_t evictions) {
    drawAhead(std::min(evictions, fcount_ + 4096));
    return fcount_;
  }
  size_t queuedDraws() const { return fcount_; }
  void prefetch(Hash const& k) const { __builtin_prefetch(&table_[keyBits(k) & mask_]); }
  // second stage of the walk's prefetch (the slot of k was prefetched a few
  // items earlier): the entry of the first slot whose tag matches k
  void prefetchFound(Hash const& k) const {
    const uint64_t tag = keyBits(k) & 0xffffffffu;
    for (size_t s = tag & mask_;; s = (s + 1) & mask_) {
      const uint64_t t = table_[s];
      if (t == 0) return;
      if ((t >> 32) == tag) {
        __builtin_prefetch(&entries_[(uint32_t)t - 1], 1);
        return;
      }
    }
  }
  uint32_t find(Hash const& k) const {
    const uint64_t tag = keyBits(k) & 0xffffffffu;
    for (size_t s = tag & mask_;; s = (s + 1) & mask_) {
      const uint64_t t = table_[s];
      if (t == 0) return kNone;
      if ((t >> 32) == tag && entries_[(uint32_t)t - 1].key == k) return (uint32_t)t - 1;
    }
  }
  Entry& at(uint32_t id) { return entries_[id]; }
  // maybeGet() on a found entry
  Entry& touch(uint32_t id) {
    Entry& e = entries_[id];
    ordGen_[e.pos] = ++generation_;
    return e;
  }
  // put(); owner != 0 inserts a pending value.  Returns the entry id.
  uint32_t put(Hash const& k, bool v, uint64_t owner = 0, uint32_t pendIdx = 0) {
    const uint32_t id = find(k);
    if (id != kNone) {
      update(id, v, owner, pendIdx);
      return id;
    }
    return insertNew(k, v, owner, pendIdx);
  }
  // put() of a key find() just reported present (id) ...
  void update(uint32_t id, bool v, uint64_t owner, uint32_t pendIdx) {
    Entry& e = entries_[id];
    ordGen_[e.pos] = ++generation_;
    e.value = v;
    e.owner = owner;
    e.pendIdx = pendIdx;
  }
  // ... or absent (the caller's find() returned kNone)
  uint32_t insertNew(Hash const& k, bool v, uint64_t owner, uint32_t pendIdx) {
    ++generation_;
    const uint32_t pos = (uint32_t)ordId_.size();
    uint32_t nid;
    if (!freeIds_.empty()) {
      nid = freeIds_.back();
      freeIds_.pop_back();
      entries_[nid] = Entry{k, owner, pendIdx, pos, v};
    } else {
      nid = (uint32_t)entries_.size();
      entries_.push_back(Entry{k, owner, pendIdx, pos, v});
    }
    const uint32_t tag = (uint32_t)keyBits(k);
    insertSlot(tag, nid);
    ordId_.push_back(nid);
    ordTag_.push_back(tag);
    ordGen_.push_back(generation_);
    if (ordId_.size() > maxSize_) evictOne();
    if (!freeIds_.empty()) __builtin_prefetch(&entries_[freeIds_.back()], 1);  // the next insert's slot
    return nid;
  }
  // fills in a pending value if entry `id` still holds this batch's item (it
  // may have been evicted and its id reused since)
  // (clearVerifySigCache between a batch's walk and its resolve leaves ids
  // past the cleared table: nothing to fill in then)
  void resolve(uint32_t id, uint64_t owner, uint32_t pendIdx, bool v) {
    if (id >= entries_.size()) return;
    Entry& e = entries_[id];
    if (e.owner == owner && e.pendIdx == pendIdx) {
      e.value = v;
      e.owner = 0;
    }
  }
  void prefetchEntry(uint32_t id) const {
    if (id < entries_.size()) __builtin_prefetch(&entries_[id], 1);
  }
  void clear() {
    std::fill(table_.begin(), table_.end(), 0u);
    entries_.clear();
    freeIds_.clear();
    ordId_.clear();
    ordTag_.clear();
    ordGen_.clear();
  }
  size_t size() const { return ordId_.size(); }
  std::vector<Hash> keysInOrder() const {
    std::vector<Hash> out;
    out.reserve(ordId_.size());
    for (uint32_t id : ordId_) out.push_back(entries_[id].key);
    return out;
  }

 private:
  void insertSlot(uint32_t tag, uint32_t id) {
    size_t s = tag & mask_;
    while (table_[s] != 0) s = (s + 1) & mask_;
    table_[s] = ((uint64_t)tag << 32) | (uint64_t)(id + 1);
  }
  void eraseSlot(uint32_t tag, uint32_t id) {
    size_t s = tag & mask_;
    while ((uint32_t)table_[s] != id + 1) s = (s + 1) & mask_;
    // backward-shift deletion keeps every probe chain intact (an occupant's
    // home slot is its tag & mask)
    size_t hole = s;
    for (size_t j = (hole + 1) & mask_; table_[j] != 0; j = (j + 1) & mask_) {
      const size_t home = (size_t)(table_[j] >> 32) & mask_;
      if (((j - home) & mask_) >= ((j - hole) & mask_)) {
        table_[hole] = table_[j];
        hole = j;
      }
    }
    table_[hole] = 0;
  }
  // Eviction draws are made ahead of time.  Every eviction happens at size
  // maxSize + 1, so its two draws are UniformDraw(0, maxSize) -- the same
  // sequence sequential code would draw, just computed early: at least kAhead
  // evictions ahead (so the victims' order-array entries and, half-way,
  // their table slots can be prefetched), or many more when a large batch
  // pre-draws while it waits for its keys (preDraw).  Queued draws belong to
  // the future whatever happens in between (the sequence never depends on
  // the cache's contents); maybeSeed drops them.
  static constexpr size_t kAhead = 16;
  void drawAhead(size_t want) {
    while (fcount_ < want) {
      const uint32_t a = (uint32_t)draw_(rng_);
      const uint32_t b = (uint32_t)draw_(rng_);
      if (fcount_ == future_.size()) {  // grow the ring (unwrapping it; sizes are powers of two)
        std::vector<std::pair<uint32_t, uint32_t>> g(std::max<size_t>(64, 2 * future_.size()));
        for (size_t k = 0; k < fcount_; ++k) g[k] = futureAt(k);
        future_.swap(g);
        fhead_ = 0;
      }
      future_[(fhead_ + fcount_) & (future_.size() - 1)] = {a, b};
      ++fcount_;
    }
  }
  std::pair<uint32_t, uint32_t> const& futureAt(size_t k) const {
    return future_[(fhead_ + k) & (future_.size() - 1)];
  }
  void evictOne() {
    const size_t sz = ordId_.size();
    if (sz == 0) return;
    drawAhead(kAhead + 1);
    const size_t ia = futureAt(0).first, ib = futureAt(0).second;
    fhead_ = (fhead_ + 1) & (future_.size() - 1);
    --fcount_;
    {  // kAhead ahead: the candidates' order-array entries
      auto const& f = futureAt(kAhead - 1);
      if (f.first < ordGen_.capacity() && f.second < ordGen_.capacity()) {
        __builtin_prefetch(ordGen_.data() + f.first);
        __builtin_prefetch(ordGen_.data() + f.second);
        __builtin_prefetch(ordTag_.data() + f.first);
        __builtin_prefetch(ordTag_.data() + f.second);
        __builtin_prefetch(ordId_.data() + f.first);
        __builtin_prefetch(ordId_.data() + f.second);
      }
    }
    {  // half-way ahead: the candidate victims' table slots and entries (the
       // victim's entry is rewritten by the next insert)
      auto const& f = futureAt(kAhead / 2);
      __builtin_prefetch(&table_[ordTag_[f.first] & mask_]);
      __builtin_prefetch(&table_[ordTag_[f.second] & mask_]);
      if (f.first < ordId_.size() && f.second < ordId_.size()) {
        __builtin_prefetch(&entries_[ordId_[f.first]], 1);
        __builtin_prefetch(&entries_[ordId_[f.second]], 1);
      }
    }
    const size_t iv = ordGen_[ia] < ordGen_[ib] ? ia : ib;
    const uint32_t victim = ordId_[iv];
    eraseSlot(ordTag_[iv], victim);
    freeIds_.push_back(victim);
    // swap-remove position iv (the reference's swap with mValuePtrs.back())
    const size_t last = sz - 1;
    if (iv != last) {
      ordId_[iv] = ordId_[last];
      ordTag_[iv] = ordTag_[last];
      ordGen_[iv] = ordGen_[last];
      entries_[ordId_[iv]].pos = (uint32_t)iv;
    }
    ordId_.pop_back();
    ordTag_.pop_back();
    ordGen_.pop_back();
  }
  size_t maxSize_;
  UniformDraw draw_;  // uniform_int_distribution(0, maxSize_)
  size_t mask_;
  uint64_t generation_ = 0;
  std::vector<uint64_t> table_;
  std::vector<Entry> entries_;
  std::vector<uint32_t> freeIds_;
  std::vector<uint32_t> ordId_, ordTag_;
  std::vector<uint64_t> ordGen_;
  std::minstd_rand rng_;  // stellar_default_random_engine, src/util/Math.h:26
  std::vector<std::pair<uint32_t, uint32_t>> future_;  // ring of queued draws
  size_t fhead_ = 0, fcount_ = 0;
};

std::mutex gVerifySigCacheMutex;
RandomEvictionCache gVerifySigCache(0xffff);
uint64_t gVerifyCacheHit = 0;
uint64_t gVerifyCacheMiss = 0;
uint64_t gBatchId = 0;  // owner ids of pending entries (under the mutex)
thread_local uint64_t tVerifySigHits = 0, tVerifySigMisses = 0;  // flushThreadVerifySigCounts
std::atomic<uint64_t> gGpuSigs{0}, gGpuBatches{0}, gCpuSigs{0}, gFallbacks{0};
// batch-size and latency histograms (log2 buckets), per path
std::atomic<uint64_t> gHist[4][PubKeyUtils::EngineHistograms::kBuckets];

int log2Bucket(uint64_t v) {
  int b = 0;
  while (v > 1 && b + 1 < PubKeyUtils::EngineHistograms::kBuckets) {
    v >>= 1;
    ++b;
  }
  return b;
}
void recordBatch(bool gpu, size_t n, std::chrono::steady_clock::time_point t0) {
  const auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
  gHist[gpu ? 0 : 2][log2Bucket(n)].fetch_add(1, std::memory_order_relaxed);
  gHist[gpu ? 1 : 3][log2Bucket((uint64_t)(us < 0 ? 0 : us))].fetch_add(1, std::memory_order_relaxed);
}
// runs f() (an engine or CPU-path verification of n items) and records it
template <class F>
auto timedBatch(bool gpu, size_t n, F&& f) -> decltype(f()) {
  const auto t0 = std::chrono::steady_clock::now();
  auto r = f();
  recordBatch(gpu, n, t0);
  return r;
}
std::atomic<PubKeyUtils::BatchVerifyFn> gTestVerifier{nullptr};
std::atomic<PubKeyUtils::KeyedBatchVerifyFn> gTestKeyedVerifier{nullptr};
std::atomic<size_t> gKeyedThreshold{256};
std::atomic<size_t> gCpuThreshold{1};
const bool gTrace = getenv("SV_HOST_TRACE") != nullptr;  // stage timings of keyed batches to stderr
std::chrono::steady_clock::time_point gTraceMarshal;   // (SV_HOST_TRACE: engine inputs marshalled)

using Item = PubKeyUtils::VerifyItem;
// keyed batches at least this large walk the cache on the calling thread while
// the engine call runs on a helper (verifySigBatch)
constexpr size_t kThreadedWalkMin = 16384;
// eviction draws queued ahead by a waiting walk at most (8 MB of pairs)
constexpr size_t kPreDrawMax = size_t(1) << 20;
// Keyed batches below kThreadedWalkMin with SV_HOST_KEYS=1: the cache keys
// are hashed on the host pool while this thread waits on the engine's
// verdicts-only call, and the helper that hashes the last slice walks the
// cache, instead of the engine's hash kernel sharing the GPU with the verify
// kernel (the default).
bool hostKeysBeside() {
  static const bool b = [] {
    const char* e = getenv("SV_HOST_KEYS");
    return e != nullptr && std::atoi(e) != 0;
  }();
  return b;
}

// Per-thread scratch reused across calls: a large batch does not pay fresh
// page faults for its index, key and pointer arrays every time.
struct Scratch {
  std::vector<size_t> rows, missRows, missItems;
  std::vector<Hash> keys;
  std::vector<uint8_t> verdict, mv;
  std::vector<uint32_t> ref, ids;
  std::vector<const uint8_t*> pk, sig, msg;
  std::vector<uint32_t> len;
  // pk / sig / msg / len already hold the engine inputs of `rows` (filled by
  // verifySigBatch's pooled row pass; gpuVerify then skips its own)
  bool rowsMarshalled = false;
  // SoA copy for the test hooks (the engine itself gathers)
  std::vector<uint8_t> ppk, psig, pmsg;
  std::vector<uint64_t> poff;
  std::vector<uint32_t> plen;
};
Scratch& scratch() {
  static thread_local Scratch s;
  return s;
}

// Fills in this batch's pending values: item k's entry is ids[k] (kNone: no
// pending insert), under the cache mutex.  (Split over 4 helper threads by
// entry id it measured slower than this prefetching loop: 0.40 vs 0.29 ms per
// 100k on MI355X hosts.)
void resolvePending(const uint32_t* ids, const uint8_t* v, size_t n, uint64_t owner) {
  constexpr uint32_t kNone = RandomEvictionCache::kNone;
  std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
  for (size_t k = 0; k < n; ++k) {
    if (k + 8 < n && ids[k + 8] != kNone) gVerifySigCache.prefetchEntry(ids[k + 8]);
    if (ids[k] != kNone) gVerifySigCache.resolve(ids[k], owner, (uint32_t)k, v[k] != 0);
  }
}

void packForTestHook(std::vector<Item> const& items, std::vector<size_t> const& rows, Scratch& st) {
  const size_t n = rows.size();
  st.ppk.resize(32 * n);
  st.psig.resize(64 * n);
  st.poff.resize(n);
  st.plen.resize(n);
  size_t total = 0;
  for (size_t r : rows) total += items[r].msg.size();
  st.pmsg.resize(std::max<size_t>(1, total));
  size_t pos = 0;
  for (size_t i = 0; i < n; ++i) {
    Item const& it = items[rows[i]];
    std::memcpy(&st.ppk[32 * i], it.key->ed25519().data(), 32);
    std::memcpy(&st.psig[64 * i], it.signature.data(), 64);
    st.poff[i] = pos;
    st.plen[i] = (uint32_t)it.msg.size();
    if (st.plen[i]) std::memcpy(&st.pmsg[pos], it.msg.data(), st.plen[i]);
    pos += st.plen[i];
  }
}

// CPU path over items[rows] (the engine's own algorithm, host build).
void cpuVerify(std::vector<Item> const& items, std::vector<size_t> const& rows, uint8_t* verdict) {
  parallelFor(rows.size(), 4, [&](size_t i) {
    Item const& it = items[rows[i]];
    verdict[i] = sv_ed25519_verify_cpu(it.key->ed25519().data(), it.signature.data(), it.msg.data(),
                                       it.msg.size()) == 1
                     ? 1
                     : 0;
  });
  gCpuSigs += rows.size();
}

// The memo of derived cache keys (KeyMemo.h; SV_KEY_MEMO=0 turns it off).
bool memoOn() {
  static const bool b = [] {
    const char* e = getenv("SV_KEY_MEMO");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return b;
}
KeyMemo& keyMemo() {
  static KeyMemo m;
  return m;
}
// verifySigCacheKey through the memo (64-byte signatures only: a shorter one
// never reaches the cache, SecretKey.cpp:441-444).  store: a key derived here
// enters the memo (the miss path, where a verification follows anyway; the
// hit path only reads it: a store there would cost every first-time hit)
Hash memoKey(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg, bool store) {
  Hash k;
  if (memoOn() && sig.size() == 64) {
    if (keyMemo().find(key.ed25519().data(), sig.data(), msg.data(), msg.size(), k.data())) return k;
    k = PubKeyUtils::verifySigCacheKey(key, sig, msg);
    if (store) keyMemo().put(key.ed25519().data(), sig.data(), msg.data(), msg.size(), k.data());
    return k;
  }
  return PubKeyUtils::verifySigCacheKey(key, sig, msg);
}

// Keys derived for at most this many items at once enter the memo: single
// verifySig misses (a tx's signatures checked on receipt, then again at
// nomination and apply) -- not a micro-batch's hundreds.  Stores of a
// micro-batch's keys measured later verdicts for config 4's paced SCP bursts
// on the flush worker (~0.07 ms) and still ~0.1 ms when made on the host pool
// right after the walk, while the GPU verifies; the main thread's verifySig
// ceiling rose from ~1.0-1.5M/s to 2.4-3.5M/s, but its p50 did not improve
// (profiles/r06/config4/c4_memo_*.jsonl).
constexpr size_t kMemoStoreMax = 16;

void hostKeys(std::vector<Item> const& items, std::vector<size_t> const& rows, Hash* keys) {
  const bool store = rows.size() <= kMemoStoreMax;
  parallelFor(rows.size(), 256, [&](size_t i) {
    Item const& it = items[rows[i]];
    keys[i] = memoKey(*it.key, it.signature, it.msg, store);
  });
}

// GPU engine over items[rows] (gather: the engine packs straight from the
// items); keys != nullptr also returns the cache keys.  Returns the engine's
// status; the caller falls back to the CPU path on any error.
void runProgress(void* ctx, size_t ready) { (*static_cast<std::function<void(size_t)>*>(ctx))(ready); }

// keysReady (keyed passes): keysReady(k) runs once keys [0, k) are in `keys`,
// for increasing k up to n; the engine calls it while the GPU still verifies
// (one-chunk batches, the keys in pieces), else it runs once here.
int gpuVerify(std::vector<Item> const& items, std::vector<size_t> const& rows, uint8_t* verdict, Hash* keys,
              std::function<void(size_t)>* keysReady = nullptr, Scratch* scr = nullptr) {
  const size_t n = rows.size();
  static_assert(sizeof(Hash) == 32, "Hash must be 32 contiguous bytes");
  uint8_t* kb = reinterpret_cast<uint8_t*>(keys);
  Scratch& st = scr ? *scr : scratch();  // (the caller's: this may run on a helper thread)
  if (keys) {
    if (PubKeyUtils::KeyedBatchVerifyFn tk = gTestKeyedVerifier.load()) {
      packForTestHook(items, rows, st);
      const int rc = tk(st.ppk.data(), st.psig.data(), st.pmsg.data(), st.poff.data(), st.plen.data(), n, verdict, kb);
      if (rc == SV_OK && keysReady) (*keysReady)(n);
      return rc;
    }
  } else if (PubKeyUtils::BatchVerifyFn tv = gTestVerifier.load()) {
    packForTestHook(items, rows, st);
    return tv(st.ppk.data(), st.psig.data(), st.pmsg.data(), st.poff.data(), st.plen.data(), n, verdict);
  }
  if (!(st.rowsMarshalled && &rows == &st.rows && st.pk.size() == n)) {
    st.pk.resize(n);
    st.sig.resize(n);
    st.msg.resize(n);
    st.len.resize(n);
    // (each item's key is a pointer to chase: on the pool for large batches,
    // this is in front of the first piece of keys)
    parallelFor(n, 16384, [&](size_t i) {
      Item const& it = items[rows[i]];
      st.pk[i] = it.key->ed25519().data();
      st.sig[i] = it.signature.data();
      st.msg[i] = it.msg.data();
      st.len[i] = (uint32_t)it.msg.size();
    });
  }
  st.rowsMarshalled = false;
  if (gTrace) gTraceMarshal = std::chrono::steady_clock::now();
  if (keysReady)
    return sv_ed25519_verify_batch_gather_progress(st.pk.data(), st.sig.data(), st.msg.data(), st.len.data(), n,
                                                   verdict, kb, runProgress, keysReady, nullptr);
  return sv_ed25519_verify_batch_gather(st.pk.data(), st.sig.data(), st.msg.data(), st.len.data(), n, verdict, kb,
                                        nullptr);
}

}  // namespace

size_t hostPoolThreads() { return hostPool().size() + 1; }

void hostParallelFor(size_t n, size_t grain, std::function<void(size_t, size_t)> const& range) {
  const size_t parts = std::max<size_t>(1, std::min<size_t>(hostPool().size() + 1, n / std::max<size_t>(1, grain)));
  if (parts == 1) {
    range(0, n);
    return;
  }
  hostPool().run(parts, [&](size_t t) { range(n * t / parts, n * (t + 1) / parts); });
}

namespace PubKeyUtils {

Hash verifySigCacheKey(PublicKey const& key, Signature const& signature, ByteSlice const& bin) {
  return verifySigCacheKey(key, ByteSlice(signature), bin);
}

Hash verifySigCacheKey(PublicKey const& key, ByteSlice const& signature, ByteSlice const& bin) {
  hostcrypto::Blake2b256 h;
  h.add(key.ed25519().data(), 32);
  h.add(signature.data(), signature.size());
  h.add(bin.data(), bin.size());
  return h.finish();
}

std::vector<bool> verifySigBatch(std::vector<VerifyItem> const& items, std::vector<Hash>* keysOut) {
  const auto tEnter = gTrace ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
  const size_t n = items.size();
  std::vector<bool> out(n, false);
  Scratch& sc = scratch();
  std::vector<size_t>& rows = sc.rows;  // eligible items
  rows.clear();
  sc.rowsMarshalled = false;
  const size_t parts = std::min<size_t>(hostPool().size() + 1, n / 16384);
  if (parts <= 1) {
    for (size_t i = 0; i < n; ++i) {
      if (items[i].key->type() != PUBLIC_KEY_TYPE_ED25519)
        throw std::invalid_argument("verifySigBatch: non-ed25519 key");  // releaseAssert, SecretKey.cpp:440
      if (items[i].signature.size() != 64) continue;                   // SecretKey.cpp:441-444
      rows.push_back(i);
    }
  } else {
    // the same checks and the same rows, on the pool: count per part, then
    // fill each part's rows at its offset
    std::vector<size_t> cnt(parts + 1, 0);
    std::atomic<bool> bad{false};
    hostPool().run(parts, [&](size_t t) {
      size_t c = 0;
      for (size_t i = n * t / parts, b = n * (t + 1) / parts; i < b; ++i) {
        if (items[i].key->type() != PUBLIC_KEY_TYPE_ED25519) bad.store(true, std::memory_order_relaxed);
        c += items[i].signature.size() == 64;
      }
      cnt[t + 1] = c;
    });
    if (bad.load()) throw std::invalid_argument("verifySigBatch: non-ed25519 key");  // releaseAssert, SecretKey.cpp:440
    for (size_t t = 0; t < parts; ++t) cnt[t + 1] += cnt[t];
    const size_t E = cnt[parts];
    rows.resize(E);
    // (the engine's input pointers in the same pass: gpuVerify of these rows
    // need not walk the items again)
    sc.pk.resize(E);
    sc.sig.resize(E);
    sc.msg.resize(E);
    sc.len.resize(E);
    hostPool().run(parts, [&](size_t t) {
      size_t o = cnt[t];
      for (size_t i = n * t / parts, b = n * (t + 1) / parts; i < b; ++i) {
        Item const& it = items[i];
        if (it.signature.size() != 64) continue;  // SecretKey.cpp:441-444
        rows[o] = i;
        sc.pk[o] = it.key->ed25519().data();
        sc.sig[o] = it.signature.data();
        sc.msg[o] = it.msg.data();
        sc.len[o] = (uint32_t)it.msg.size();
        ++o;
      }
    });
    sc.rowsMarshalled = true;
  }
  if (keysOut) keysOut->assign(n, Hash{});
  const size_t E = rows.size();
  if (E == 0) return out;
  std::vector<Hash>& keys = sc.keys;
  keys.resize(E);
  std::vector<uint8_t>& verdict = sc.verdict;
  verdict.assign(E, 0);

  const size_t thr = gKeyedThreshold.load();
  if (thr != 0 && E >= thr && gTestVerifier.load() == nullptr) {
    // keyed: every eligible item verified and hashed in one engine pass.  The
    // cache walk (phase 1: hits, misses inserted pending in item order) runs
    // as soon as the keys are back, overlapping the GPU's verification; the
    // pending values are filled in once the verdicts arrive (phase 3).
    constexpr uint32_t kNone = RandomEvictionCache::kNone;
    std::vector<uint8_t>& hit = sc.mv;
    hit.assign(E, 0);
    std::vector<uint32_t>& pid = sc.ref;  // entry id of each pending insert
    pid.assign(E, kNone);
    uint64_t owner = 0;
    bool walked = false;
    size_t done = 0;  // items walked so far (the keys arrive in pieces)
    // verdictsIn: the engine call has returned, so a miss can be inserted
    // with its verdict (no pending state, nothing left for resolvePending)
    bool verdictsIn = false;
    size_t pendEnd = E;  // items [0, pendEnd) may hold pending inserts
    std::function<void(size_t)> phase1 = [&](size_t ready) {
      // (locked per piece: other callers' verifySig calls may fall between
      // two pieces, as they may between two calls of a sequential loop)
      std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
      if (done == 0) owner = ++gBatchId;
      if (verdictsIn) {
        pendEnd = std::min(pendEnd, done);
        for (size_t e = done; e < ready; ++e) {
          if (e + 8 < ready) gVerifySigCache.prefetch(keys[e + 8]);
          if (e + 4 < ready) gVerifySigCache.prefetchFound(keys[e + 4]);
          const uint32_t id = gVerifySigCache.find(keys[e]);
          if (id != kNone) {
            auto const& ent = gVerifySigCache.at(id);
            if (ent.owner == 0 || ent.owner == owner) {
              ++gVerifyCacheHit;
              auto& t = gVerifySigCache.touch(id);
              if (t.owner == 0) {
                hit[e] = 1;
                out[rows[e]] = t.value;
              }
              continue;
            }
            ++gVerifyCacheMiss;
            gVerifySigCache.update(id, verdict[e] != 0, 0, 0);
            continue;
          }
          ++gVerifyCacheMiss;
          gVerifySigCache.insertNew(keys[e], verdict[e] != 0, 0, 0);
        }
        done = ready;
        if (done == E) walked = true;
        return;
      }
      for (size_t e = done; e < ready; ++e) {
        if (e + 8 < ready) gVerifySigCache.prefetch(keys[e + 8]);
        if (e + 4 < ready) gVerifySigCache.prefetchFound(keys[e + 4]);
        const uint32_t id = gVerifySigCache.find(keys[e]);
        if (id != kNone) {
          auto const& ent = gVerifySigCache.at(id);
          if (ent.owner == 0 || ent.owner == owner) {  // cached, or an earlier item of this batch
            ++gVerifyCacheHit;
            auto& t = gVerifySigCache.touch(id);
            if (t.owner == 0) {
              hit[e] = 1;
              out[rows[e]] = t.value;
            }
            continue;
          }
          ++gVerifyCacheMiss;  // another batch's pending entry: put() over it
          gVerifySigCache.update(id, false, owner, (uint32_t)e);
          pid[e] = id;
          continue;
        }
        ++gVerifyCacheMiss;
        pid[e] = gVerifySigCache.insertNew(keys[e], false, owner, (uint32_t)e);
      }
      done = ready;
      if (done == E) walked = true;
    };
    const bool trace = gTrace;
    const auto tA = std::chrono::steady_clock::now();
    std::chrono::steady_clock::time_point tB{}, tC{};
    std::function<void(size_t)> walk = phase1;
    if (trace)
      phase1 = [&](size_t ready) {
        if (done == 0) tB = std::chrono::steady_clock::now();
        walk(ready);
        tC = std::chrono::steady_clock::now();
      };
    int erc;
    if (E < kThreadedWalkMin && hostKeysBeside() && gTestKeyedVerifier.load() == nullptr) {
      // this thread runs the engine call (task 0 of the pool run); the
      // helpers hash slices of the keys, and the one that finishes the last
      // slice walks the cache (phase 1: misses inserted pending) while the
      // GPU still verifies
      const size_t H = std::max<size_t>(1, std::min<size_t>(hostPool().size(), E / 64));
      std::atomic<size_t> left{H};
      std::exception_ptr walkExc, engExc;
      hostPool().run(H + 1, [&](size_t t) {
        if (t == 0) {  // (nothing may leave a task: run() returns only after every task)
          try {
            erc = timedBatch(true, E, [&] { return gpuVerify(items, rows, verdict.data(), nullptr, nullptr, &sc); });
          } catch (...) {
            engExc = std::current_exception();
            erc = SV_ERR_INVALID_ARG;
          }
          return;
        }
        const size_t a = E * (t - 1) / H, b = E * t / H;
        for (size_t e = a; e < b; ++e) {
          Item const& it = items[rows[e]];
          keys[e] = memoKey(*it.key, it.signature, it.msg, false);
        }
        if (left.fetch_sub(1, std::memory_order_acq_rel) == 1) {
          try {
            phase1(E);
          } catch (...) {
            walkExc = std::current_exception();
          }
        }
      });
      if (engExc) std::rethrow_exception(engExc);
      if (walkExc) std::rethrow_exception(walkExc);
    } else if (E >= kThreadedWalkMin) {
      // Large batches: the engine call runs on a helper thread and publishes
      // how many keys are in (the engine delivers them in pieces); this thread
      // walks the cache as they land -- the thread whose caches hold the
      // verify cache from earlier calls.
      // Once there is nothing to walk or pre-draw, this thread sleeps on `cv`
      // (after a short spin: a piece of keys is usually close) instead of
      // holding a core for the whole engine call.  An exception on the engine
      // thread is carried over and rethrown here after the join; the join
      // also runs when this thread's walk throws (EngJoin).
      std::atomic<size_t> ready{0};
      std::atomic<bool> fin{false};
      std::mutex wm;
      std::condition_variable cv;
      std::exception_ptr engExc;
      std::function<void(size_t)> publish = [&](size_t r) {
        {
          std::lock_guard<std::mutex> lk(wm);
          ready.store(r, std::memory_order_release);
        }
        cv.notify_one();
      };
      std::thread eng([&] {
        try {
          erc = timedBatch(true, E, [&] { return gpuVerify(items, rows, verdict.data(), keys.data(), &publish, &sc); });
        } catch (...) {
          engExc = std::current_exception();
          erc = SV_ERR_INVALID_ARG;
        }
        {
          std::lock_guard<std::mutex> lk(wm);
          fin.store(true, std::memory_order_release);
        }
        cv.notify_one();
      });
      struct EngJoin {
        std::thread& t;
        ~EngJoin() {
          if (t.joinable()) t.join();
        }
      } engJoin{eng};
      size_t drawn = 0;
      for (;;) {
        const bool f = fin.load(std::memory_order_acquire);
        const size_t r = ready.load(std::memory_order_acquire);
        if (r > done) {
          // (once the engine has returned, every verdict is in `verdict`;
          // walked in slices so the switch happens as soon as it has)
          if (f && erc == SV_OK) verdictsIn = true;
          phase1(std::min(r, done + 8192));
          continue;
        }
        if (f || done == E) break;
        if (drawn < std::min<size_t>(E - done, kPreDrawMax)) {
          // waiting for keys: queue the eviction draws the walk may need
          // (at most one per remaining item, at most kPreDrawMax queued), a
          // slice per lock hold
          std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
          const size_t before = gVerifySigCache.queuedDraws();
          drawn = gVerifySigCache.preDraw(std::min<size_t>(E - done, kPreDrawMax));
          if (drawn == before) drawn = E;  // (nothing more to queue)
          continue;
        }
        // nothing to do until the next piece or the end of the engine call
        const auto spinEnd = std::chrono::steady_clock::now() + std::chrono::microseconds(20);
        while (ready.load(std::memory_order_acquire) <= done && !fin.load(std::memory_order_acquire) &&
               std::chrono::steady_clock::now() < spinEnd)
          std::this_thread::yield();
        std::unique_lock<std::mutex> lk(wm);
        cv.wait(lk, [&] { return ready.load(std::memory_order_acquire) > done || fin.load(std::memory_order_acquire); });
      }
      eng.join();
      if (engExc) std::rethrow_exception(engExc);
    } else {
      erc = timedBatch(true, E, [&] { return gpuVerify(items, rows, verdict.data(), keys.data(), &phase1, &sc); });
    }
    if (erc == SV_OK) {
      gGpuSigs += E;
      gGpuBatches += 1;
      if (trace) {
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        const auto tD = std::chrono::steady_clock::now();
        fprintf(stderr,
                "[verifySigBatch keyed n=%zu] rows %.3f ms, then: inputs marshalled %.3f ms, keys ready %.3f ms, walk "
                "%.3f ms, verdicts %.3f ms after walk\n",
                E, ms(tEnter, tA), gTraceMarshal > tA ? ms(tA, gTraceMarshal) : 0.0, ms(tA, tB), ms(tB, tC), ms(tC, tD));
      }
    } else {
      ++gFallbacks;
      if (!walked) {
        hostKeys(items, rows, keys.data());
        phase1(E);  // (continues a walk the engine's pieces had started)
      }
      timedBatch(false, E, [&] { cpuVerify(items, rows, verdict.data()); return 0; });
    }
    if (!walked) phase1(E);  // (not reached: the engine ran it on success)
    const auto tE = std::chrono::steady_clock::now();
    resolvePending(pid.data(), verdict.data(), pendEnd, owner);
    if (trace)
      fprintf(stderr, "[verifySigBatch keyed n=%zu] resolve %.3f ms\n", E,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tE).count());
    for (size_t e = 0; e < E; ++e)
      if (!hit[e]) out[rows[e]] = verdict[e] != 0;
  } else {
    hostKeys(items, rows, keys.data());
    // phase 1: walk the cache in item order; misses are inserted pending
    std::vector<size_t>& missRows = sc.missRows;  // eligible index of each distinct miss
    missRows.clear();
    std::vector<uint32_t>& ref = sc.ref;
    ref.assign(E, RandomEvictionCache::kNone);
    std::vector<uint32_t>& missIds = sc.ids;  // entry id of each pending insert
    missIds.clear();
    uint64_t owner;
    {
      std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
      owner = ++gBatchId;
      for (size_t e = 0; e < E; ++e) {
        if (e + 8 < E) gVerifySigCache.prefetch(keys[e + 8]);
        if (e + 4 < E) gVerifySigCache.prefetchFound(keys[e + 4]);
        const uint32_t id = gVerifySigCache.find(keys[e]);
        if (id != RandomEvictionCache::kNone) {
          auto const& ent = gVerifySigCache.at(id);
          if (ent.owner == 0) {
            ++gVerifyCacheHit;
            out[rows[e]] = gVerifySigCache.touch(id).value;
            continue;
          }
          if (ent.owner == owner) {  // an earlier item of this batch
            ++gVerifyCacheHit;
            ref[e] = gVerifySigCache.touch(id).pendIdx;
            continue;
          }
        }
        ++gVerifyCacheMiss;
        ref[e] = (uint32_t)missRows.size();
        missIds.push_back(id != RandomEvictionCache::kNone ? (gVerifySigCache.update(id, false, owner, ref[e]), id)
                                                           : gVerifySigCache.insertNew(keys[e], false, owner, ref[e]));
        missRows.push_back(e);
      }
    }
    // phase 2: verify the misses (outside the lock: the engine call is long)
    const size_t M = missRows.size();
    std::vector<size_t>& missItems = sc.missItems;
    missItems.resize(M);
    for (size_t m = 0; m < M; ++m) missItems[m] = rows[missRows[m]];
    std::vector<uint8_t>& mv = sc.mv;
    mv.assign(M, 0);
    if (M > 0) {
      if (M <= gCpuThreshold.load() && gTestVerifier.load() == nullptr) {
        timedBatch(false, M, [&] { cpuVerify(items, missItems, mv.data()); return 0; });
      } else if (timedBatch(true, M, [&] { return gpuVerify(items, missItems, mv.data(), nullptr); }) == SV_OK) {
        gGpuSigs += M;
        gGpuBatches += 1;
      } else {
        ++gFallbacks;
        timedBatch(false, M, [&] { cpuVerify(items, missItems, mv.data()); return 0; });
      }
    }
    // phase 3: fill in the pending values
    resolvePending(missIds.data(), mv.data(), M, owner);
    for (size_t e = 0; e < E; ++e)
      if (ref[e] != RandomEvictionCache::kNone) out[rows[e]] = mv[ref[e]] != 0;
  }
  if (keysOut)
    for (size_t e = 0; e < E; ++e) (*keysOut)[rows[e]] = keys[e];
  return out;
}

std::vector<bool> verifySigBatch(std::vector<VerifyItem> const& items) { return verifySigBatch(items, nullptr); }

void verifyBatchUncached(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                         const uint32_t* len, size_t n, uint8_t* verdict) {
  if (n == 0) return;
  BatchVerifyFn tv = gTestVerifier.load();
  if (!tv && n <= gCpuThreshold.load()) {
    timedBatch(false, n, [&] { return sv_ed25519_verify_batch_cpu(pk, sig, msg, off, len, n, verdict, 0); });
    gCpuSigs += n;
    return;
  }
  const int rc = timedBatch(true, n, [&] {
    return tv ? tv(pk, sig, msg, off, len, n, verdict)
              : sv_ed25519_verify_batch(pk, sig, msg, off, len, n, verdict, nullptr);
  });
  if (rc == SV_OK) {
    gGpuSigs += n;
    gGpuBatches += 1;
    return;
  }
  ++gFallbacks;
  timedBatch(false, n, [&] { return sv_ed25519_verify_batch_cpu(pk, sig, msg, off, len, n, verdict, 0); });
  gCpuSigs += n;
}

bool verifySig(PublicKey const& key, Signature const& signature, ByteSlice const& bin) {
  // the hit path as the reference runs it (SecretKey.cpp:446-456): key, one
  // lock, lookup, touch -- no batch bookkeeping; anything else (a miss, or an
  // entry another batch has pending) takes the batch path, which re-derives
  // the key and decides exactly as for a one-item batch
  if (key.type() == PUBLIC_KEY_TYPE_ED25519 && signature.size() == 64) {
    const Hash k = memoKey(key, ByteSlice(signature), bin, false);
    std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
    const uint32_t id = gVerifySigCache.find(k);
    if (id != RandomEvictionCache::kNone && gVerifySigCache.at(id).owner == 0) {
      ++gVerifyCacheHit;
      ++tVerifySigHits;
      return gVerifySigCache.touch(id).value;
    }
  }
  ++tVerifySigMisses;
  std::vector<VerifyItem> one{VerifyItem{&key, ByteSlice(signature), bin}};
  return verifySigBatch(one, nullptr)[0];
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

void flushThreadVerifySigCounts(uint64_t& hits, uint64_t& misses) {
  hits = tVerifySigHits;
  misses = tVerifySigMisses;
  tVerifySigHits = tVerifySigMisses = 0;
}

void setBatchVerifierForTesting(BatchVerifyFn fn) { gTestVerifier.store(fn); }
void setKeyedBatchVerifierForTesting(KeyedBatchVerifyFn fn) { gTestKeyedVerifier.store(fn); }
void setKeyedBatchThreshold(size_t minItems) { gKeyedThreshold.store(minItems); }
void setCpuBatchThreshold(size_t maxMisses) { gCpuThreshold.store(maxMisses); }

EngineCounts flushEngineCounts() {
  EngineCounts c;
  c.gpuSignatures = gGpuSigs.exchange(0);
  c.gpuBatches = gGpuBatches.exchange(0);
  c.cpuSignatures = gCpuSigs.exchange(0);
  c.fallbacks = gFallbacks.exchange(0);
  return c;
}

EngineHistograms flushEngineHistograms() {
  EngineHistograms h;
  for (int b = 0; b < EngineHistograms::kBuckets; ++b) {
    h.gpuBatchSize[b] = gHist[0][b].exchange(0);
    h.gpuLatencyUs[b] = gHist[1][b].exchange(0);
    h.cpuBatchSize[b] = gHist[2][b].exchange(0);
    h.cpuLatencyUs[b] = gHist[3][b].exchange(0);
  }
  return h;
}

void flushEngineCounts(uint64_t& signatures, uint64_t& batches) {
  signatures = gGpuSigs.exchange(0);
  batches = gGpuBatches.exchange(0);
}

std::vector<Hash> cacheKeysForTesting() {
  std::lock_guard<std::mutex> guard(gVerifySigCacheMutex);
  return gVerifySigCache.keysInOrder();
}

}  // namespace PubKeyUtils
}  // namespace stellar
