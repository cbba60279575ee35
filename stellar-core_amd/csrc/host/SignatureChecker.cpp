// See SignatureChecker.h.  Logic restated from
// /root/reference/src/transactions/SignatureChecker.cpp:30-158 and
// /root/reference/src/transactions/SignatureUtils.cpp:30-136.
#include "SignatureChecker.h"

#include <cstring>
#include <functional>
#include <string>

#include "hashes.h"

namespace stellar {

namespace SignatureUtils {

// last 4 bytes (or the whole slice, zero-padded, if shorter); SignatureUtils.cpp:112-127
SignatureHint getHint(ByteSlice const& bs) {
  SignatureHint res{};
  if (bs.empty()) return res;
  if (res.size() > bs.size()) std::memcpy(res.data(), bs.begin(), bs.size());
  else std::memcpy(res.data(), bs.end() - res.size(), res.size());
  return res;
}

// SignatureUtils.cpp:129-136
bool doesHintMatch(ByteSlice const& bs, SignatureHint const& hint) {
  if (bs.size() < hint.size()) return false;
  return std::memcmp(bs.end() - hint.size(), hint.data(), hint.size()) == 0;
}

// key hint XOR payload hint; SignatureUtils.cpp:95-109
SignatureHint getSignedPayloadHint(SignerKey const& s) {
  SignatureHint a = getHint(ByteSlice(s.key.data(), 32));
  SignatureHint b = getHint(ByteSlice(s.payload.data(), s.payload.size()));
  SignatureHint h;
  for (int i = 0; i < 4; ++i) h[i] = a[i] ^ b[i];
  return h;
}

}  // namespace SignatureUtils

namespace {

std::string cacheKeyString(uint256 const& pk, Signature const& sig, ByteSlice const& msg) {
  hostcrypto::Blake2b256 h;
  h.add(pk.data(), 32);
  h.add(sig.data(), sig.size());
  h.add(msg.data(), msg.size());
  auto d = h.finish();
  return std::string(reinterpret_cast<const char*>(d.data()), d.size());
}

uint32_t clampWeight(uint32_t protocol, uint32_t w) { return (protocol >= 10 && w > 255) ? 255 : w; }

}  // namespace

// ---------------------------------------------------------------- prefetch
void SignatureBatchPrefetch::add(Hash const& contentsHash, std::vector<DecoratedSignature> const& signatures,
                                 std::vector<Signer> const& signers) {
  for (auto const& sig : signatures) {
    if (sig.signature.size() != 64) continue;  // verifySig rejects before verifying
    for (auto const& s : signers) {
      if (s.key.type == SIGNER_KEY_TYPE_ED25519) {
        if (!SignatureUtils::doesHintMatch(ByteSlice(s.key.key.data(), 32), sig.hint)) continue;
        Pending p;
        p.pk.ed25519() = s.key.key;
        p.sig = sig.signature;
        p.msg.assign(contentsHash.begin(), contentsHash.end());
        items_.push_back(std::move(p));
      } else if (s.key.type == SIGNER_KEY_TYPE_ED25519_SIGNED_PAYLOAD) {
        SignatureHint h = SignatureUtils::getSignedPayloadHint(s.key);
        if (!SignatureUtils::doesHintMatch(ByteSlice(h.data(), 4), sig.hint)) continue;
        Pending p;
        p.pk.ed25519() = s.key.key;
        p.sig = sig.signature;
        p.msg = s.key.payload;
        items_.push_back(std::move(p));
      }
    }
  }
}

void SignatureBatchPrefetch::run() {
  std::vector<PubKeyUtils::VerifyItem> items;
  items.reserve(items_.size());
  for (auto const& p : items_) items.push_back(PubKeyUtils::VerifyItem{&p.pk, &p.sig, ByteSlice(p.msg)});
  std::vector<bool> v = PubKeyUtils::verifySigBatch(items);
  verdicts_.reserve(items_.size());
  for (size_t i = 0; i < items_.size(); ++i)
    verdicts_[cacheKeyString(items_[i].pk.ed25519(), items_[i].sig, ByteSlice(items_[i].msg))] = v[i];
}

bool SignatureBatchPrefetch::lookup(uint256 const& pk, Signature const& sig, ByteSlice const& msg,
                                    bool& verdict) const {
  auto it = verdicts_.find(cacheKeyString(pk, sig, msg));
  if (it == verdicts_.end()) return false;
  verdict = it->second;
  return true;
}

// ---------------------------------------------------------------- checker
SignatureChecker::SignatureChecker(uint32_t protocolVersion, Hash const& contentsHash,
                                   std::vector<DecoratedSignature> const& signatures,
                                   SignatureBatchPrefetch const* prefetched)
    : mProtocolVersion(protocolVersion),
      mContentsHash(contentsHash),
      mSignatures(signatures),
      mUsedSignatures(signatures.size(), false),
      mPrefetched(prefetched) {}

bool SignatureChecker::verifyEd25519(DecoratedSignature const& sig, uint256 const& key, ByteSlice const& msg) const {
  if (mPrefetched && sig.signature.size() == 64) {
    bool v;
    if (mPrefetched->lookup(key, sig.signature, msg, v)) return v;
  }
  PublicKey pk;
  pk.ed25519() = key;
  return PubKeyUtils::verifySig(pk, sig.signature, msg);
}

bool SignatureChecker::checkSignature(std::vector<Signer> const& signersV, int32_t neededWeight) {
  if (mProtocolVersion == 7) return true;  // SignatureChecker.cpp:38-41

  std::vector<Signer> byType[4];
  for (auto const& s : signersV) byType[s.key.type].push_back(s);

  int32_t totalWeight = 0;
  for (auto const& s : byType[SIGNER_KEY_TYPE_PRE_AUTH_TX]) {  // :54-69
    if (s.key.key == mContentsHash) {
      totalWeight += (int32_t)clampWeight(mProtocolVersion, s.weight);
      if (totalWeight >= neededWeight) return true;
    }
  }

  using VerifyT = std::function<bool(DecoratedSignature const&, Signer const&)>;
  auto verifyAll = [&](std::vector<Signer>& signers, VerifyT verify) {  // :73-102
    for (size_t i = 0; i < mSignatures.size(); i++) {
      auto const& sig = mSignatures[i];
      for (auto it = signers.begin(); it != signers.end(); ++it) {
        if (verify(sig, *it)) {
          mUsedSignatures[i] = true;
          totalWeight += (int32_t)clampWeight(mProtocolVersion, it->weight);
          if (totalWeight >= neededWeight) return true;
          signers.erase(it);
          break;
        }
      }
    }
    return false;
  };

  if (verifyAll(byType[SIGNER_KEY_TYPE_HASH_X], [&](DecoratedSignature const& sig, Signer const& s) {
        // SignatureUtils::verifyHashX, SignatureUtils.cpp:86-93
        if (!SignatureUtils::doesHintMatch(ByteSlice(s.key.key.data(), 32), sig.hint)) return false;
        auto h = hostcrypto::sha256(sig.signature.data(), sig.signature.size());
        return std::memcmp(h.data(), s.key.key.data(), 32) == 0;
      }))
    return true;

  if (verifyAll(byType[SIGNER_KEY_TYPE_ED25519], [&](DecoratedSignature const& sig, Signer const& s) {
        // SignatureUtils::verify, SignatureUtils.cpp:38-46
        if (!SignatureUtils::doesHintMatch(ByteSlice(s.key.key.data(), 32), sig.hint)) return false;
        return verifyEd25519(sig, s.key.key, ByteSlice(mContentsHash.data(), 32));
      }))
    return true;

  if (verifyAll(byType[SIGNER_KEY_TYPE_ED25519_SIGNED_PAYLOAD], [&](DecoratedSignature const& sig, Signer const& s) {
        // SignatureUtils::verifyEd25519SignedPayload, SignatureUtils.cpp:48-61
        SignatureHint h = SignatureUtils::getSignedPayloadHint(s.key);
        if (!SignatureUtils::doesHintMatch(ByteSlice(h.data(), 4), sig.hint)) return false;
        return verifyEd25519(sig, s.key.key, ByteSlice(s.key.payload.data(), s.key.payload.size()));
      }))
    return true;

  return false;
}

bool SignatureChecker::checkAllSignaturesUsed() const {  // :138-158
  if (mProtocolVersion == 7) return true;
  for (bool used : mUsedSignatures)
    if (!used) return false;
  return true;
}

}  // namespace stellar
