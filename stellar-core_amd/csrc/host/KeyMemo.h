// Memo of verify-cache keys by their exact input bytes.
//
// Every PubKeyUtils::verifySig call derives the cache key BLAKE2b-256(pk ||
// sig || msg) before it can look the verdict up
// (/root/reference/src/crypto/SecretKey.cpp:446-457, verifySigCacheKey
// :50-61): ~0.5 us for an SCP envelope, most of a cache hit.  stellar-core
// verifies the same (pk, sig, msg) twice on purpose -- the overlay's
// pre-verify fills the cache (Peer.cpp:963-970, here a micro-batch whose keys
// the GPU hashed) and the main thread's HerderImpl::verifyEnvelope then hits
// it (HerderImpl.cpp:2414-2432) -- so the second derivation repeats work done
// moments before.  The memo keeps the last derivation per slot, with the bytes
// it was derived from; a lookup returns the key only when pk, sig and msg are
// byte-for-byte those bytes, so it returns exactly what verifySigCacheKey
// would.  The cache itself (lookup by key, touch, hit / miss counts,
// eviction) is unchanged: the memo only skips a pure function's recomputation.
//
// Direct-mapped, kSlots slots indexed by a salted hash of the signature (an
// adversary choosing signatures can only make slots overwrite each other,
// i.e. fall back to hashing); a dense array of per-slot tags (32 bits of the
// same hash) turns away most misses before the slot is read.  Messages longer
// than kMsgMax are not memoized.  Keys enter the memo where they are derived
// on the host for a single verification or a handful (PubKeyUtils.cpp
// kMemoStoreMax), not from micro-batches: measured on config 4, storing ~400
// slots per micro-batch on the flush worker delayed every verdict by more
// than the main thread's hits saved (profiles/r06/config4/c4_memo_ab*.jsonl).
// Each slot is a seqlock: a writer takes it by moving its sequence to odd
// (a busy slot is skipped: the memo may always decline), a reader copies and
// compares the bytes and accepts them only if the sequence was even and
// unchanged around the copy.  The bytes are read and written as relaxed
// 64-bit atomics, so concurrent access is defined behaviour.
#pragma once

#include <array>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <memory>
#include <random>

namespace stellar {

class KeyMemo {
 public:
  static constexpr size_t kSlotsLog2 = 15;
  static constexpr size_t kSlots = size_t(1) << kSlotsLog2;
  static constexpr size_t kMsgMax = 384;  // SCP statements are 128-384 bytes (BASELINE config 4)

  KeyMemo() : slots_(new Slot[kSlots]), tags_(new std::atomic<uint32_t>[kSlots]) {
    for (size_t i = 0; i < kSlots; ++i) tags_[i].store(0, std::memory_order_relaxed);
    std::random_device rd;
    salt_ = ((uint64_t)rd() << 32) ^ rd() ^ 0x9E3779B97F4A7C15ull;
  }

  // true (and key set) iff the slot for sig holds a key derived from exactly
  // (pk, sig, msg)
  bool find(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t msgLen, uint8_t key[32]) const {
    if (msgLen > kMsgMax) return false;
    uint32_t tag;
    const size_t i = index(sig, &tag);
    // (the dense tag array answers most misses from cache, without touching
    // the slot's ~0.5 KB)
    if (tags_[i].load(std::memory_order_relaxed) != tag) return false;
    Slot const& s = slots_[i];
    const uint32_t s1 = s.seq.load(std::memory_order_acquire);
    if ((s1 & 1u) != 0 || s1 == 0) return false;
    if (s.msgLen.load(std::memory_order_relaxed) != msgLen) return false;
    if (!same(s.sig, sig, 64) || !same(s.pk, pk, 32) || !same(s.msg, msg, msgLen)) return false;
    uint64_t k[4];
    for (int w = 0; w < 4; ++w) k[w] = s.key[w].load(std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_acquire);
    if (s.seq.load(std::memory_order_relaxed) != s1) return false;
    std::memcpy(key, k, 32);
    return true;
  }

  void put(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t msgLen, const uint8_t key[32]) {
    if (msgLen > kMsgMax) return;
    uint32_t tag;
    const size_t i = index(sig, &tag);
    Slot& s = slots_[i];
    uint32_t e = s.seq.load(std::memory_order_relaxed);
    if ((e & 1u) != 0 || !s.seq.compare_exchange_strong(e, e + 1, std::memory_order_acquire)) return;
    std::atomic_thread_fence(std::memory_order_release);  // (the odd sequence before the bytes)
    store(s.sig, sig, 64);
    store(s.pk, pk, 32);
    store(s.msg, msg, msgLen);
    uint64_t k[4];
    std::memcpy(k, key, 32);
    for (int w = 0; w < 4; ++w) s.key[w].store(k[w], std::memory_order_relaxed);
    s.msgLen.store((uint32_t)msgLen, std::memory_order_relaxed);
    tags_[i].store(tag, std::memory_order_relaxed);
    s.seq.store(e + 2, std::memory_order_release);
  }

  void clear() {
    for (size_t i = 0; i < kSlots; ++i) {
      uint32_t e = slots_[i].seq.load(std::memory_order_relaxed);
      if ((e & 1u) == 0 && slots_[i].seq.compare_exchange_strong(e, 0, std::memory_order_acq_rel))
        tags_[i].store(0, std::memory_order_relaxed);
    }
  }

 private:
  using Word = std::atomic<uint64_t>;
  struct Slot {
    std::atomic<uint32_t> seq{0};  // even: stable (0: empty), odd: being written
    std::atomic<uint32_t> msgLen{0};
    Word pk[4], sig[8], key[4];
    Word msg[kMsgMax / 8];
  };
  static_assert(kMsgMax % 8 == 0, "message words");

  size_t index(const uint8_t sig[64], uint32_t* tag) const {
    uint64_t a, b;
    std::memcpy(&a, sig, 8);
    std::memcpy(&b, sig + 32, 8);
    uint64_t h = (a ^ salt_) * 0x9E3779B97F4A7C15ull;
    h ^= (b + salt_) * 0xC2B2AE3D27D4EB4Full;
    *tag = (uint32_t)h | 1u;  // (never 0: an empty slot's tag)
    return (size_t)(h >> (64 - kSlotsLog2));
  }
  // n bytes of p as 8-byte words, the last one zero-padded
  static uint64_t word(const uint8_t* p, size_t n, size_t i) {
    uint64_t w = 0;
    const size_t o = 8 * i;
    std::memcpy(&w, p + o, n - o >= 8 ? 8 : n - o);
    return w;
  }
  static bool same(Word const* w, const uint8_t* p, size_t n) {
    for (size_t i = 0; 8 * i < n; ++i)
      if (w[i].load(std::memory_order_relaxed) != word(p, n, i)) return false;
    return true;
  }
  static void store(Word* w, const uint8_t* p, size_t n) {
    for (size_t i = 0; 8 * i < n; ++i) w[i].store(word(p, n, i), std::memory_order_relaxed);
  }

  std::unique_ptr<Slot[]> slots_;
  std::unique_ptr<std::atomic<uint32_t>[]> tags_;  // per slot: a tag of its signature (0: empty)
  uint64_t salt_;
};

}  // namespace stellar
