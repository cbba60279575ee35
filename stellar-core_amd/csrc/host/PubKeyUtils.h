// C++ host mirror of stellar-core's verification boundary, re-targeted at the
// MI355X engine (include/stellar_sigverify.h).
//
// Reference interface (same names, argument meaning and error behaviour):
//   bool PubKeyUtils::verifySig(PublicKey const&, Signature const&, ByteSlice const&)
//       /root/reference/src/crypto/SecretKey.h:139-140, SecretKey.cpp:435-468
//   void clearVerifySigCache(); void maybeSeedVerifySigCache(unsigned);
//   void flushVerifySigCacheCounts(uint64_t& hits, uint64_t& misses)
//       SecretKey.h:142-144, SecretKey.cpp:317-339
// New:
//   std::vector<bool> verifySigBatch(std::vector<VerifyItem> const&)
//
// Semantics kept from SecretKey.cpp:435-468: a signature whose size != 64 is
// rejected before any cache interaction; the cache key is BLAKE2b-256(pk ||
// sig || msg); the process-global 0xffff-entry random-eviction cache
// (RandomEvictionCache.h, two draws of the libc++ uniform_int_distribution
// stellar-core pins in lib/util/stdrandom.h) is consulted before dispatch and
// BOTH verdicts are stored; hit/miss counters.  verifySigBatch(items) leaves
// the cache, its counters and the verdicts exactly as the same items passed
// one by one to verifySig would (tests/test_host_mirror.py replays it against
// a sequential restatement of the reference cache).
//
// Like the reference, nothing here throws on a verification problem:
// misses go to the GPU engine in one batch; a single miss (or any batch of at
// most cpuBatchThreshold misses) runs on the engine's CPU path
// (sv_ed25519_verify_batch_cpu: the same algorithm compiled for the host,
// cheaper than a GPU round trip); if the GPU engine returns an error the batch
// is re-run on the CPU path -- an engine error is never a reject and never an
// exception.  engineFallbacks counts those re-runs.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace stellar {

using uint256 = std::array<uint8_t, 32>;
using Hash = std::array<uint8_t, 32>;

enum PublicKeyType : int32_t { PUBLIC_KEY_TYPE_ED25519 = 0 };

// XDR union PublicKey restated for its only arm (ed25519 uint256).
struct PublicKey {
  PublicKeyType type_ = PUBLIC_KEY_TYPE_ED25519;
  uint256 key_{};
  PublicKeyType type() const { return type_; }
  uint256& ed25519() { return key_; }
  uint256 const& ed25519() const { return key_; }
};

// XDR Signature = opaque<64>, held inline: at most 64 bytes, so a tx set's
// ~30k decorated signatures cost no heap allocation each (xdrpp's
// opaque_vec<64> is a std::vector).  The vector operations the mirror uses.
class Signature {
 public:
  static constexpr size_t kMax = 64;
  Signature() = default;
  explicit Signature(size_t n) { resize(n); }
  template <class It>
  Signature(It first, It last) {
    assign(first, last);
  }
  template <class It>
  void assign(It first, It last) {
    size_t n = 0;
    for (It it = first; it != last; ++it) {
      if (n == kMax) throw std::length_error("Signature: more than 64 bytes (XDR opaque<64>)");
      buf_[n++] = (uint8_t)*it;
    }
    n_ = (uint8_t)n;
  }
  // (bytes: one copy instead of the iterator loop)
  void assign(const uint8_t* first, const uint8_t* last) {
    const size_t n = (size_t)(last - first);
    if (n > kMax) throw std::length_error("Signature: more than 64 bytes (XDR opaque<64>)");
    if (n) std::memcpy(buf_, first, n);
    n_ = (uint8_t)n;
  }
  void resize(size_t n) {
    if (n > kMax) throw std::length_error("Signature: more than 64 bytes (XDR opaque<64>)");
    for (size_t k = n_; k < n; ++k) buf_[k] = 0;
    n_ = (uint8_t)n;
  }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  uint8_t* data() { return buf_; }
  const uint8_t* data() const { return buf_; }
  uint8_t* begin() { return buf_; }
  uint8_t* end() { return buf_ + n_; }
  const uint8_t* begin() const { return buf_; }
  const uint8_t* end() const { return buf_ + n_; }
  uint8_t& operator[](size_t i) { return buf_[i]; }
  uint8_t operator[](size_t i) const { return buf_[i]; }
  bool operator==(Signature const& o) const {
    if (n_ != o.n_) return false;
    for (size_t k = 0; k < n_; ++k)
      if (buf_[k] != o.buf_[k]) return false;
    return true;
  }
  bool operator!=(Signature const& o) const { return !(*this == o); }

 private:
  uint8_t buf_[kMax] = {};
  uint8_t n_ = 0;
};

// Non-owning (pointer, size), src/crypto/ByteSlice.h:19-80
struct ByteSlice {
  const uint8_t* p = nullptr;
  size_t n = 0;
  ByteSlice() = default;
  ByteSlice(const uint8_t* d, size_t s) : p(d), n(s) {}
  template <class C>
  ByteSlice(C const& c) : p(reinterpret_cast<const uint8_t*>(c.data())), n(c.size()) {}
  const uint8_t* data() const { return p; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const uint8_t* begin() const { return p; }
  const uint8_t* end() const { return p + n; }
};

namespace PubKeyUtils {

// One verification: borrowed key, signature bytes (size != 64 is rejected
// before any cache interaction, as in verifySig) and message.
struct VerifyItem {
  PublicKey const* key;
  ByteSlice signature;
  ByteSlice msg;
};

bool verifySig(PublicKey const& key, Signature const& signature, ByteSlice const& bin);
std::vector<bool> verifySigBatch(std::vector<VerifyItem> const& items);
// Same, also returning every item's verify-cache key (keysOut[i]; items whose
// signature size != 64 get an all-zero key) -- for callers that index their
// own side tables by it without hashing again.
std::vector<bool> verifySigBatch(std::vector<VerifyItem> const& items, std::vector<Hash>* keysOut);

// Engine-only batch over contiguous SoA buffers (message i = msg[off[i] ..
// off[i] + len[i])), no cache interaction: the GPU engine (or the test
// verifier), the CPU path for at most cpuBatchThreshold items or on an engine
// error.  Callers that keep their own verdict tables (SignatureBatchPrefetch,
// catchup replay) use this.
void verifyBatchUncached(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                         const uint32_t* len, size_t n, uint8_t* verdict);

void clearVerifySigCache();
void maybeSeedVerifySigCache(unsigned int seed);
void flushVerifySigCacheCounts(uint64_t& hits, uint64_t& misses);
// Hits / misses of the calling thread's own verifySig calls since its last
// call of this function (flushes them).  Diagnostic: a caller that follows an
// earlier pre-verify (HerderImpl::verifyEnvelope after Peer.cpp's) learns
// whether its calls were served from the cache, which the process-wide
// counters above cannot tell while other threads verify.
void flushThreadVerifySigCounts(uint64_t& hits, uint64_t& misses);

// BLAKE2b-256(pk || sig || msg), SecretKey.cpp:50-61
Hash verifySigCacheKey(PublicKey const& key, Signature const& signature, ByteSlice const& bin);
Hash verifySigCacheKey(PublicKey const& key, ByteSlice const& signature, ByteSlice const& bin);

// Engine override for tests (cf. the reference's BUILD_TESTS hooks such as
// AlwaysValidSignatureChecker, SignatureChecker.h:41-63): when set, GPU-bound
// misses are sent to `fn` instead of the GPU.  A non-zero return is treated
// like an engine error (CPU fallback).  Pass nullptr to restore.
using BatchVerifyFn = int (*)(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                              const uint32_t* len, size_t n, uint8_t* verdict);
void setBatchVerifierForTesting(BatchVerifyFn fn);

// Keyed batches: a verifySigBatch call with at least
// `minItems` eligible signatures sends ALL of them to the engine in one pass
// that returns verdicts AND the BLAKE2b cache keys (sv_ed25519_verify_batch_gather
// with keys), so the host never hashes; the cache is then walked once in item
// order, exactly as sequential verifySig calls would.  0 disables.  Default 256.
void setKeyedBatchThreshold(size_t minItems);
using KeyedBatchVerifyFn = int (*)(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                                   const uint32_t* len, size_t n, uint8_t* verdict, uint8_t* keys);
void setKeyedBatchVerifierForTesting(KeyedBatchVerifyFn fn);

// Batches with at most this many cache misses run on the CPU path instead of
// the GPU (default 1: a single verifySig never pays a GPU round trip).
void setCpuBatchThreshold(size_t maxMisses);

// Observability: signatures sent to the GPU engine, engine calls (batches),
// signatures verified on the CPU path, and engine errors that were re-run on
// the CPU path, since the last flush.
struct EngineCounts {
  uint64_t gpuSignatures = 0, gpuBatches = 0, cpuSignatures = 0, fallbacks = 0;
};
EngineCounts flushEngineCounts();
void flushEngineCounts(uint64_t& signatures, uint64_t& batches);

// Histograms beside the crypto.verify.{hit,miss,total} meters
// (/root/reference/docs/metrics.md:48-50): every verification call that
// reaches the engine (gpu*) or the CPU path (cpu*) is counted by its batch
// size and its wall latency in microseconds, in bucket b = floor(log2(v))
// (b = 0 also holds v = 0; the last bucket holds everything above).  Bounded
// (fixed buckets), lock-free; flushing reads and zeroes them.
struct EngineHistograms {
  static constexpr int kBuckets = 32;
  uint64_t gpuBatchSize[kBuckets], gpuLatencyUs[kBuckets], cpuBatchSize[kBuckets], cpuLatencyUs[kBuckets];
};
EngineHistograms flushEngineHistograms();

// Test hook: cache keys currently held, in the cache's insertion-order vector
// (the reference's mValuePtrs), for replay tests of the eviction policy.
std::vector<Hash> cacheKeysForTesting();

}  // namespace PubKeyUtils
}  // namespace stellar
