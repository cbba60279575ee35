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
// sig || msg); the process-global 0xffff-entry random-eviction cache is
// consulted before dispatch; BOTH verdicts are stored; hit/miss counters.
// Difference: misses go to the GPU engine in one batch, and a device error is
// thrown as VerifyEngineError (never turned into a reject).
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
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

// XDR Signature = opaque<64>
using Signature = std::vector<uint8_t>;

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

class VerifyEngineError : public std::runtime_error {
 public:
  explicit VerifyEngineError(std::string const& m) : std::runtime_error(m) {}
};

namespace PubKeyUtils {

struct VerifyItem {
  PublicKey const* key;
  Signature const* signature;
  ByteSlice msg;
};

bool verifySig(PublicKey const& key, Signature const& signature, ByteSlice const& bin);
std::vector<bool> verifySigBatch(std::vector<VerifyItem> const& items);

void clearVerifySigCache();
void maybeSeedVerifySigCache(unsigned int seed);
void flushVerifySigCacheCounts(uint64_t& hits, uint64_t& misses);

// Engine override for tests (cf. the reference's BUILD_TESTS hooks such as
// AlwaysValidSignatureChecker, SignatureChecker.h:41-63): when set, cache
// misses are sent to `fn` instead of the GPU.  Pass nullptr to restore.
using BatchVerifyFn = int (*)(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                              const uint32_t* len, size_t n, uint8_t* verdict);
void setBatchVerifierForTesting(BatchVerifyFn fn);

// Keyed batches: a verifySigBatch call with at least
// `minItems` eligible signatures sends ALL of them to the engine in one pass
// that returns verdicts AND the BLAKE2b cache keys (sv_ed25519_verify_batch_keyed),
// so the host never hashes; cache bookkeeping (hits, in-batch duplicates,
// misses, insertions, counters) is then identical to the hashed path.
// 0 disables.  Default 4096.
void setKeyedBatchThreshold(size_t minItems);
using KeyedBatchVerifyFn = int (*)(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                                   const uint32_t* len, size_t n, uint8_t* verdict, uint8_t* keys);
void setKeyedBatchVerifierForTesting(KeyedBatchVerifyFn fn);

// Number of signatures sent to the engine and number of engine calls
// (batches) since the last flush -- observability for batch sizes.
void flushEngineCounts(uint64_t& signatures, uint64_t& batches);

}  // namespace PubKeyUtils
}  // namespace stellar
