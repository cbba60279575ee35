// Host-side hashes used around the verification boundary.
//   BLAKE2b-256: the verify-cache key, stellar-core src/crypto/SecretKey.cpp:50-61
//                (BLAKE2 wrapper src/crypto/BLAKE2.cpp:31-75, libsodium
//                crypto_generichash with a 32-byte output) -- RFC 7693.
//   SHA-256:     HASH_X signers, src/transactions/SignatureUtils.cpp:86-93 -- FIPS 180-4.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>

namespace stellar {
namespace hostcrypto {

using Hash32 = std::array<uint8_t, 32>;

// Incremental BLAKE2b with a 32-byte digest and no key.
class Blake2b256 {
 public:
  Blake2b256();
  void add(const uint8_t* p, size_t n);
  Hash32 finish();

 private:
  void compress(const uint8_t* block, bool last);
  void bump(size_t bytes) {  // the 128-bit byte counter
    t_[0] += bytes;
    if (t_[0] < bytes) ++t_[1];
  }
  uint64_t h_[8];
  uint64_t t_[2];
  uint8_t buf_[128];
  size_t fill_;
};

Hash32 blake2b256(const uint8_t* p, size_t n);
Hash32 sha256(const uint8_t* p, size_t n);

}  // namespace hostcrypto
}  // namespace stellar
