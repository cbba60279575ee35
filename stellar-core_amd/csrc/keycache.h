// Host index of a device slot's key-table cache (warm-key latency path,
// comb.h / sv_comb.hip).  Maps a 32-byte ed25519 public key to a cache slot
// whose device tables ({0..8} * 16^j * (-A)) the comb kernel reads.
//
// The cache holds derived public data only: a slot's tables are a pure
// function of the key bytes, so a hit never changes a verdict, only which
// kernel computes it.  Keys are compared in full (the hash only picks the
// probe start).
//
// Policy:
//   * admission: a missing key is built on its first sighting while the cache
//     has a free slot; once it is full, only on its second sighting (a small
//     set-associative filter of fingerprints), so one-off transaction keys and
//     junk never evict the validator keys that reappear in every SCP batch;
//   * eviction by CLOCK (second chance) over READY slots; a slot touched by
//     the batch being planned is never evicted;
//   * a slot is BUILDING from the moment its build is queued until the build's
//     event completes (promoted by the caller via set_ready()).
#pragma once

#include <cstdint>
#include <cstring>
#include <vector>

namespace sv {

class KeyIndex {
 public:
  enum : uint8_t { FREE = 0, BUILDING = 1, READY = 2 };

  void reset(size_t cap) {
    cap_ = cap;
    size_t t = 1;
    while (t < 2 * cap + 2) t <<= 1;
    mask_ = t - 1;
    idx_.assign(cap ? t : 0, -1);
    keys_.assign(32 * cap, 0);
    state_.assign(cap, FREE);
    gen_.assign(cap, 0);
    used_.assign(cap, 0);
    ref_.assign(cap, 0);
    seen_.assign(cap ? 4 * kSeenSets : 0, 0);
    free_.clear();
    for (size_t c = cap; c > 0; --c) free_.push_back((int32_t)(c - 1));
    live_ = 0;
    hand_ = 0;
  }
  size_t capacity() const { return cap_; }
  size_t size() const { return live_; }

  int32_t find(const uint8_t* pk) const {
    if (!cap_) return -1;
    for (size_t i = hash(pk) & mask_;; i = (i + 1) & mask_) {
      const int32_t s = idx_[i];
      if (s < 0) return -1;
      if (std::memcmp(&keys_[32 * (size_t)s], pk, 32) == 0) return s;
    }
  }
  uint8_t state(int32_t s) const { return state_[s]; }
  uint64_t gen(int32_t s) const { return gen_[s]; }
  void touch(int32_t s, uint64_t now) {
    used_[s] = now;
    ref_[s] = 1;
  }
  void set_ready(int32_t s, uint64_t gen) {
    if (state_[s] == BUILDING && gen_[s] == gen) state_[s] = READY;
  }
  const uint8_t* key(int32_t s) const { return &keys_[32 * (size_t)s]; }

  // Admission of a key that missed: always while a slot is free; once the
  // cache is full, only on its second sighting (4-way set-associative filter
  // of fingerprints), so one-off keys never evict warm ones.
  bool admit(const uint8_t* pk) {
    if (!cap_) return false;
    if (live_ < cap_) return true;
    const uint64_t fp = hash(pk) | 1u;
    uint64_t* set = &seen_[4 * ((fp >> 20) & (kSeenSets - 1))];
    for (int w = 0; w < 4; ++w)
      if (set[w] == fp) {
        set[w] = 0;
        return true;
      }
    set[seen_rr_++ & 3] = fp;
    return false;
  }

  // A slot for pk (state BUILDING, generation gen), evicting if full; -1 when
  // every slot is BUILDING or used by the batch being planned (`now`).
  int32_t insert(const uint8_t* pk, uint64_t gen, uint64_t now, bool* evicted) {
    *evicted = false;
    if (!cap_) return -1;
    int32_t s = -1;
    if (!free_.empty()) {
      s = free_.back();
      free_.pop_back();
    } else {
      // CLOCK over READY slots not touched by this batch
      for (size_t k = 0; k < 2 * cap_ && s < 0; ++k) {
        const size_t c = hand_;
        hand_ = (hand_ + 1) % cap_;
        if (state_[c] != READY || used_[c] == now) continue;
        if (ref_[c]) {
          ref_[c] = 0;
          continue;
        }
        s = (int32_t)c;
      }
      if (s < 0) return -1;
      erase(s);
      free_.pop_back();  // (erase listed it as free: it is reused right here)
      *evicted = true;
    }
    std::memcpy(&keys_[32 * (size_t)s], pk, 32);
    state_[s] = BUILDING;
    gen_[s] = gen;
    used_[s] = now;
    ref_[s] = 1;
    ++live_;
    for (size_t i = hash(pk) & mask_;; i = (i + 1) & mask_)
      if (idx_[i] < 0) {
        idx_[i] = s;
        break;
      }
    return s;
  }

  // Drops a slot whose build (generation gen) failed: back to FREE.
  void drop(int32_t s, uint64_t gen) {
    if (state_[s] == BUILDING && gen_[s] == gen) erase(s);
  }

 private:
  static constexpr size_t kSeenSets = 4096;
  size_t cap_ = 0, mask_ = 0, live_ = 0, hand_ = 0, seen_rr_ = 0;
  std::vector<int32_t> idx_, free_;
  std::vector<uint8_t> keys_, state_, ref_;
  std::vector<uint64_t> gen_, used_, seen_;

  static uint64_t load64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
  }
  size_t hash(const uint8_t* pk) const {
    // keys are adversary-chosen: mix 16 bytes (a collision only costs probes)
    const uint64_t x = load64(pk) * 0x9e3779b97f4a7c15ull ^ load64(pk + 8) * 0xc2b2ae3d27d4eb4full;
    return (size_t)(x ^ (x >> 29));
  }
  // removes slot s from the probe table (backward-shift deletion keeps every
  // remaining key reachable from its hash position)
  void erase(int32_t s) {
    size_t i = hash(&keys_[32 * (size_t)s]) & mask_;
    while (idx_[i] != s) i = (i + 1) & mask_;
    size_t j = i;
    for (;;) {
      j = (j + 1) & mask_;
      if (idx_[j] < 0) break;
      const size_t home = hash(&keys_[32 * (size_t)idx_[j]]) & mask_;
      // move idx_[j] into the hole at i if its home is not in (i, j]
      const bool in_range = i <= j ? (home > i && home <= j) : (home > i || home <= j);
      if (!in_range) {
        idx_[i] = idx_[j];
        i = j;
      }
    }
    idx_[i] = -1;
    state_[s] = FREE;
    ref_[s] = 0;
    free_.push_back(s);
    --live_;
  }
};

}  // namespace sv
