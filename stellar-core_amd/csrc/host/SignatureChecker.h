// Restatement of stellar-core's multisig signature checker with a GPU batch
// pre-pass.
//
// Reference:
//   SignatureChecker      /root/reference/src/transactions/SignatureChecker.h:18-39,
//                         SignatureChecker.cpp:20-158
//   SignatureUtils        /root/reference/src/transactions/SignatureUtils.cpp:30-61 (verify,
//                         verifyEd25519SignedPayload), :86-93 (verifyHashX),
//                         :95-136 (getSignedPayloadHint, getHint, doesHintMatch)
//
// The checker's decision logic is unchanged (greedy weight accumulation in
// the order PRE_AUTH_TX, HASH_X, ED25519, ED25519_SIGNED_PAYLOAD; a matching
// signer is erased; weight clamped to 255 from protocol 10; protocol 7 always
// passes).  What is new is SignatureBatchPrefetch: it enumerates every
// hint-matching (signature, signer) pair of MANY transactions (a tx set,
// TxSetFrame.cpp:427-457, or a ledger being applied, LedgerManagerImpl.cpp:
// 1582-1648), verifies them in one GPU batch, and hands the verdicts to the
// checkers as a side table -- so the per-tx checkers never wait on the GPU
// one signature at a time, and the 0xffff-entry global cache cannot evict a
// verdict before it is used.
#pragma once

#include <array>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "PubKeyUtils.h"

namespace stellar {

enum SignerKeyType : int32_t {
  SIGNER_KEY_TYPE_ED25519 = 0,
  SIGNER_KEY_TYPE_PRE_AUTH_TX = 1,
  SIGNER_KEY_TYPE_HASH_X = 2,
  SIGNER_KEY_TYPE_ED25519_SIGNED_PAYLOAD = 3,
};

struct SignerKey {
  SignerKeyType type = SIGNER_KEY_TYPE_ED25519;
  uint256 key{};                 // ed25519 / preAuthTx / hashX / signedPayload.ed25519
  std::vector<uint8_t> payload;  // signedPayload.payload (<= 64 bytes)
};

struct Signer {
  SignerKey key;
  uint32_t weight = 0;
};

using SignatureHint = std::array<uint8_t, 4>;

struct DecoratedSignature {
  SignatureHint hint{};
  Signature signature;
};

namespace SignatureUtils {
SignatureHint getHint(ByteSlice const& bs);
bool doesHintMatch(ByteSlice const& bs, SignatureHint const& hint);
SignatureHint getSignedPayloadHint(SignerKey const& signedPayloadSigner);
}  // namespace SignatureUtils

// Verdicts computed ahead of the checkers, keyed by the verify-cache key
// BLAKE2b-256(pk || sig || msg).
class SignatureBatchPrefetch {
 public:
  // Enumerate the hint-matching ed25519 / signed-payload pairs of one tx.
  void add(Hash const& contentsHash, std::vector<DecoratedSignature> const& signatures,
           std::vector<Signer> const& signers);
  // One GPU batch over everything added (through PubKeyUtils::verifySigBatch,
  // so the global cache is filled too).
  void run();
  // verdict for (pk, sig, msg) if prefetched
  bool lookup(uint256 const& pk, Signature const& sig, ByteSlice const& msg, bool& verdict) const;
  size_t pairs() const { return items_.size(); }

 private:
  struct Pending {
    PublicKey pk;
    Signature sig;
    std::vector<uint8_t> msg;
  };
  std::vector<Pending> items_;
  std::unordered_map<std::string, bool> verdicts_;
};

class SignatureChecker {
 public:
  SignatureChecker(uint32_t protocolVersion, Hash const& contentsHash,
                   std::vector<DecoratedSignature> const& signatures,
                   SignatureBatchPrefetch const* prefetched = nullptr);
  bool checkSignature(std::vector<Signer> const& signersV, int32_t neededWeight);
  bool checkAllSignaturesUsed() const;

 private:
  bool verifyEd25519(DecoratedSignature const& sig, uint256 const& key, ByteSlice const& msg) const;

  uint32_t mProtocolVersion;
  Hash const& mContentsHash;
  std::vector<DecoratedSignature> const& mSignatures;
  std::vector<bool> mUsedSignatures;
  SignatureBatchPrefetch const* mPrefetched;
};

}  // namespace stellar
