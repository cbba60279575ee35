// See SignatureChecker.h.  Logic restated from
// /root/reference/src/transactions/SignatureChecker.cpp:30-158 and
// /root/reference/src/transactions/SignatureUtils.cpp:30-136.
#include "SignatureChecker.h"

#include <algorithm>
#include <cstring>
#include <exception>
#include <mutex>
#include <thread>

#include "HostPool.h"
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

// SignatureUtils.cpp:38-46
bool verify(DecoratedSignature const& sig, SignerKey const& signerKey, Hash const& hash) {
  if (!doesHintMatch(ByteSlice(signerKey.key.data(), 32), sig.hint)) return false;
  PublicKey pk;
  pk.ed25519() = signerKey.key;
  return PubKeyUtils::verifySig(pk, sig.signature, ByteSlice(hash.data(), hash.size()));
}

// SignatureUtils.cpp:86-93
bool verifyHashX(DecoratedSignature const& sig, SignerKey const& signerKey) {
  if (!doesHintMatch(ByteSlice(signerKey.key.data(), 32), sig.hint)) return false;
  auto h = hostcrypto::sha256(sig.signature.data(), sig.signature.size());
  return std::memcmp(h.data(), signerKey.key.data(), 32) == 0;
}

// SignatureUtils.cpp:48-61
bool verifyEd25519SignedPayload(DecoratedSignature const& sig, SignerKey const& signer) {
  SignatureHint h = getSignedPayloadHint(signer);
  if (!doesHintMatch(ByteSlice(h.data(), 4), sig.hint)) return false;
  PublicKey pk;
  pk.ed25519() = signer.key;
  return PubKeyUtils::verifySig(pk, sig.signature, ByteSlice(signer.payload.data(), signer.payload.size()));
}

}  // namespace SignatureUtils

namespace {
uint32_t clampWeight(uint32_t protocol, uint32_t w) { return (protocol >= 10 && w > 255) ? 255 : w; }
}  // namespace

// ---------------------------------------------------------------- prefetch
void SignatureBatchPrefetch::Storage::clear() {
  pk.clear();
  sig.clear();
  msg.clear();
  off.clear();
  len.clear();
  verdict.clear();
  table.clear();
  txBegin.clear();
}

// A few spares per thread: a call that holds several prefetches at once (the
// pipelined tx-set pre-pass holds two) reuses the storage of each.
std::vector<SignatureBatchPrefetch::Storage>& SignatureBatchPrefetch::spares() {
  thread_local std::vector<Storage> s;
  return s;
}

SignatureBatchPrefetch::SignatureBatchPrefetch() {
  auto& sp = spares();
  if (!sp.empty()) {
    std::swap(st_, sp.back());
    sp.pop_back();
  }
  st_.clear();
}

SignatureBatchPrefetch::~SignatureBatchPrefetch() {
  auto& sp = spares();
  if (sp.size() < kSpares) sp.push_back(std::move(st_));
}
uint64_t SignatureBatchPrefetch::hashOf(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, size_t len) {
  // signatures and keys are uniformly distributed bytes: a few words of each
  // (plus the message's) make a good table hash; lookups compare all bytes
  uint64_t a, b, c = 0;
  std::memcpy(&a, sig, 8);
  std::memcpy(&b, pk + 24, 8);
  if (len >= 8) std::memcpy(&c, msg + len - 8, 8);
  else if (len) std::memcpy(&c, msg, len);
  uint64_t h = a ^ (b * 0x9e3779b97f4a7c15ull) ^ ((c + len) * 0xc2b2ae3d27d4eb4full);
  return h ^ (h >> 29);
}

namespace {
uint32_t hint32(const uint8_t* p) {
  uint32_t h;
  std::memcpy(&h, p, 4);
  return h;
}

// Small vector on the stack (spills to the heap past N): the per-tx scratch
// of add() and checkSignature().  Not thread_local: in a shared library every
// access to a thread_local goes through __tls_get_addr, which inside these
// loops cost more than the work (measured on MI355X hosts: add() 2.3 -> 3.9 ms
// on a 30k-pair set when its scratch was made thread_local).
template <typename T, size_t N>
class InlineVec {
 public:
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T* begin() { return data(); }
  T* end() { return data() + n_; }
  T& operator[](size_t i) { return data()[i]; }
  void push_back(T const& v) {
    if (heap_.empty() && n_ < N) {
      buf_[n_++] = v;
      return;
    }
    if (heap_.empty()) heap_.assign(buf_, buf_ + N);
    heap_.push_back(v);
    ++n_;
  }
  T* erase(T* it) {
    T* d = data();
    std::copy(it + 1, d + n_, it);
    --n_;
    if (!heap_.empty()) heap_.pop_back();
    return it;
  }

 private:
  T* data() { return heap_.empty() ? buf_ : heap_.data(); }
  T buf_[N];
  size_t n_ = 0;
  std::vector<T> heap_;
};
}  // namespace

namespace {
// A tx's ed25519 / signed-payload signers with their hints as 32-bit words
// (the signers' hints are formed once per tx and compared as words).
struct TxSigners {
  InlineVec<uint32_t, 48> hints;
  InlineVec<const Signer*, 48> eds;
  explicit TxSigners(std::vector<Signer> const& signers) {
    for (auto const& s : signers) {
      if (s.key.type == SIGNER_KEY_TYPE_ED25519) {
        hints.push_back(hint32(s.key.key.data() + 28));
        eds.push_back(&s);
      } else if (s.key.type == SIGNER_KEY_TYPE_ED25519_SIGNED_PAYLOAD) {
        const SignatureHint h = SignatureUtils::getSignedPayloadHint(s.key);
        hints.push_back(hint32(h.data()));
        eds.push_back(&s);
      }
    }
  }
};

// Visits the pairs SignatureChecker would verify for one tx, in its order
// per signature: hint-matching ED25519 signers (SignatureUtils::verify) and
// ED25519_SIGNED_PAYLOAD signers (verifyEd25519SignedPayload) --
// fn(signature, signer index k in eds).
template <class F>
void forEachPair(TxSigners& ts, std::vector<DecoratedSignature> const& signatures, F fn) {
  if (ts.eds.empty()) return;
  for (auto const& sig : signatures) {
    if (sig.signature.size() != 64) continue;  // verifySig rejects before verifying
    const uint32_t h = hint32(sig.hint.data());
    for (size_t k = 0; k < ts.eds.size(); ++k)
      if (ts.hints[k] == h) fn(sig, k);
  }
}
}  // namespace

void SignatureBatchPrefetch::enumerate(Storage& st, Hash const& contentsHash,
                                       std::vector<DecoratedSignature> const& signatures,
                                       std::vector<Signer> const& signers) {
  TxSigners ts(signers);
  if (ts.eds.empty()) return;
  auto pushMsg = [&](const uint8_t* msg, size_t msgLen) {
    const uint64_t off = st.msg.size();
    st.msg.resize(off + msgLen);
    if (msgLen) std::memcpy(&st.msg[off], msg, msgLen);
    return off;
  };
  // message bytes are stored once per tx (contents hash) / per payload signer
  uint64_t hashOff = ~0ull;
  InlineVec<uint64_t, 48> payOff;
  for (size_t k = 0; k < ts.eds.size(); ++k) payOff.push_back(~0ull);
  forEachPair(ts, signatures, [&](DecoratedSignature const& sig, size_t k) {
    Signer const& s = *ts.eds[k];
    uint64_t mo;
    size_t ml;
    if (s.key.type == SIGNER_KEY_TYPE_ED25519) {
      if (hashOff == ~0ull) hashOff = pushMsg(contentsHash.data(), 32);
      mo = hashOff;
      ml = 32;
    } else {
      if (payOff[k] == ~0ull) payOff[k] = pushMsg(s.key.payload.data(), s.key.payload.size());
      mo = payOff[k];
      ml = s.key.payload.size();
    }
    const size_t i = st.len.size();
    st.pk.resize(32 * (i + 1));
    st.sig.resize(64 * (i + 1));
    std::memcpy(&st.pk[32 * i], s.key.key.data(), 32);
    std::memcpy(&st.sig[64 * i], sig.signature.data(), 64);
    st.off.push_back(mo);
    st.len.push_back((uint32_t)ml);
  });
}

void SignatureBatchPrefetch::add(Hash const& contentsHash, std::vector<DecoratedSignature> const& signatures,
                                 std::vector<Signer> const& signers) {
  enumerate(st_, contentsHash, signatures, signers);
}

void SignatureBatchPrefetch::addBatch(std::vector<TxRef> const& txs, std::function<void(size_t)> const& prepare) {
  const size_t ntx = txs.size();
  if (txBegin_.empty()) txBegin_.push_back((uint32_t)len_.size());
  constexpr size_t kGrain = 256;
  // one contiguous range of txs per thread (the pool's helpers and this one):
  // equal ranges balance well at this grain, where more parts than threads
  // left some threads two parts and the others one (profiles/r06/config3/)
  const size_t parts = std::min(hostPoolThreads(), std::max<size_t>(1, ntx / kGrain));
  if (parts == 1) {
    for (size_t k = 0; k < ntx; ++k) {
      if (prepare) prepare(k);
      enumerate(st_, *txs[k].contentsHash, *txs[k].signatures, *txs[k].signers);
      txBegin_.push_back((uint32_t)len_.size());
    }
    return;
  }
  // Two passes over the set, each one contiguous range of txs per part, and
  // no scratch copy between them: pass 1 prepares (marshals) each tx and
  // counts its pairs and message bytes; after a prefix sum, pass 2 writes
  // every pair straight to its final place.  (The previous single pass
  // enumerated into per-part scratch and then copied it: ~30 % of the phase.)
  // An exception must not leave a pool thread: the first is kept and
  // rethrown here once every part has finished.
  std::exception_ptr failed;
  std::mutex failMu;
  const size_t t0base = txBegin_.size() - 1;  // (this batch's first tx index)
  const size_t pair0 = len_.size(), msg0 = msg_.size();
  std::vector<uint32_t> npairs(ntx), nbytes(ntx);
  std::vector<uint64_t> partPairs(parts + 1, 0), partBytes(parts + 1, 0);
  hostParallelFor(parts, 1, [&](size_t a, size_t b) {
    for (size_t p = a; p < b; ++p) {
      const size_t t0 = ntx * p / parts, t1 = ntx * (p + 1) / parts;
      uint64_t pp = 0, pb = 0;
      try {
        for (size_t t = t0; t < t1; ++t) {
          if (prepare) prepare(t);
          TxSigners ts(*txs[t].signers);
          uint32_t np = 0, nb = 0, hashUsed = 0;
          InlineVec<uint8_t, 48> payUsed;
          for (size_t k = 0; k < ts.eds.size(); ++k) payUsed.push_back(0);
          forEachPair(ts, *txs[t].signatures, [&](DecoratedSignature const&, size_t k) {
            ++np;
            if (ts.eds[k]->key.type == SIGNER_KEY_TYPE_ED25519) {
              if (!hashUsed) nb += 32;
              hashUsed = 1;
            } else if (!payUsed[k]) {
              nb += (uint32_t)ts.eds[k]->key.payload.size();
              payUsed[k] = 1;
            }
          });
          npairs[t] = np;
          nbytes[t] = nb;
          pp += np;
          pb += nb;
        }
      } catch (...) {
        std::lock_guard<std::mutex> g(failMu);
        if (!failed) failed = std::current_exception();
      }
      partPairs[p + 1] = pp;
      partBytes[p + 1] = pb;
    }
  });
  if (failed) std::rethrow_exception(failed);
  for (size_t p = 0; p < parts; ++p) {
    partPairs[p + 1] += partPairs[p];
    partBytes[p + 1] += partBytes[p];
  }
  const size_t n = pair0 + partPairs[parts];
  pk_.resize(32 * n);
  sig_.resize(64 * n);
  off_.resize(n);
  len_.resize(n);
  msg_.resize(msg0 + partBytes[parts]);
  txBegin_.resize(t0base + 1 + ntx);
  hostParallelFor(parts, 1, [&](size_t a, size_t b) {
    for (size_t p = a; p < b; ++p) {
      const size_t t0 = ntx * p / parts, t1 = ntx * (p + 1) / parts;
      size_t i = pair0 + partPairs[p];
      uint64_t mpos = msg0 + partBytes[p];
      for (size_t t = t0; t < t1; ++t) {
        TxSigners ts(*txs[t].signers);
        uint64_t hashOff = ~0ull;
        InlineVec<uint64_t, 48> payOff;
        for (size_t k = 0; k < ts.eds.size(); ++k) payOff.push_back(~0ull);
        Hash const& ch = *txs[t].contentsHash;
        forEachPair(ts, *txs[t].signatures, [&](DecoratedSignature const& sig, size_t k) {
          Signer const& s = *ts.eds[k];
          uint64_t mo;
          uint32_t ml;
          if (s.key.type == SIGNER_KEY_TYPE_ED25519) {
            if (hashOff == ~0ull) {
              hashOff = mpos;
              std::memcpy(&msg_[mpos], ch.data(), 32);
              mpos += 32;
            }
            mo = hashOff;
            ml = 32;
          } else {
            ml = (uint32_t)s.key.payload.size();
            if (payOff[k] == ~0ull) {
              payOff[k] = mpos;
              if (ml) std::memcpy(&msg_[mpos], s.key.payload.data(), ml);
              mpos += ml;
            }
            mo = payOff[k];
          }
          std::memcpy(&pk_[32 * i], s.key.key.data(), 32);
          std::memcpy(&sig_[64 * i], sig.signature.data(), 64);
          off_[i] = mo;
          len_[i] = ml;
          ++i;
        });
        txBegin_[t0base + 1 + t] = (uint32_t)i;
      }
    }
  });
}

void SignatureBatchPrefetch::buildTable() {
  const size_t n = len_.size();
  const uint8_t* msg = msg_.empty() ? nullptr : msg_.data();
  size_t cap = 16;
  while (cap < 2 * n) cap <<= 1;
  mask_ = cap - 1;
  table_.assign(cap, 0u);
  for (size_t i = 0; i < n; ++i) {
    size_t s = hashOf(&pk_[32 * i], &sig_[64 * i], msg ? msg + off_[i] : nullptr, len_[i]) & mask_;
    while (table_[s] != 0) s = (s + 1) & mask_;
    table_[s] = (uint32_t)(i + 1);
  }
}

void SignatureBatchPrefetch::run(bool seedCache) {
  const size_t n = len_.size();
  verdict_.assign(n, 0);
#ifdef FUZZING_BUILD_MODE_UNSAFE_FOR_PRODUCTION
  (void)seedCache;
  return;  // the checkers accept without looking (checkSignature): nothing to verify
#endif
  if (n == 0) return;
  const uint8_t* msg = msg_.empty() ? nullptr : msg_.data();
  // the lookup table needs only the pairs' bytes: it is built on a helper
  // thread while the engine verifies (large batches only)
  std::thread tb;
  if (n >= kAsyncTableMin) tb = std::thread([this] { buildTable(); });
  struct Join {
    std::thread& t;
    ~Join() {
      if (t.joinable()) t.join();
    }
  } join{tb};
  if (seedCache) {
    std::vector<PublicKey> keys(n);
    std::vector<PubKeyUtils::VerifyItem> items(n);
    for (size_t i = 0; i < n; ++i) {
      std::memcpy(keys[i].ed25519().data(), &pk_[32 * i], 32);
      items[i] = PubKeyUtils::VerifyItem{&keys[i], ByteSlice(&sig_[64 * i], 64),
                                         ByteSlice(msg ? msg + off_[i] : nullptr, len_[i])};
    }
    std::vector<bool> v = PubKeyUtils::verifySigBatch(items);
    for (size_t i = 0; i < n; ++i) verdict_[i] = v[i] ? 1 : 0;
  } else {
    static const uint8_t dummy = 0;
    PubKeyUtils::verifyBatchUncached(pk_.data(), sig_.data(), msg ? msg : &dummy, off_.data(), len_.data(), n,
                                     verdict_.data());
  }
  if (tb.joinable()) tb.join();
  else buildTable();
}

bool SignatureBatchPrefetch::lookup(uint256 const& pk, Signature const& sig, ByteSlice const& msg, bool& verdict,
                                    size_t tx) const {
  if (sig.size() != 64) return false;
  auto same = [&](size_t i) {
    return len_[i] == msg.size() && std::memcmp(&sig_[64 * i], sig.data(), 64) == 0 &&
           std::memcmp(&pk_[32 * i], pk.data(), 32) == 0 &&
           (msg.size() == 0 || std::memcmp(&msg_[off_[i]], msg.data(), msg.size()) == 0);
  };
  if (tx != kNoTx && tx + 1 < txBegin_.size()) {  // the tx's own pairs, contiguous (addBatch)
    for (size_t i = txBegin_[tx]; i < txBegin_[tx + 1]; ++i)
      if (same(i)) {
        verdict = verdict_[i] != 0;
        return true;
      }
  }
  if (table_.empty()) return false;
  for (size_t s = hashOf(pk.data(), sig.data(), msg.data(), msg.size()) & mask_;; s = (s + 1) & mask_) {
    const uint32_t t = table_[s];
    if (t == 0) return false;
    const size_t i = t - 1;
    if (same(i)) {
      verdict = verdict_[i] != 0;
      return true;
    }
  }
}

// ---------------------------------------------------------------- checker
SignatureChecker::SignatureChecker(uint32_t protocolVersion, Hash const& contentsHash,
                                   std::vector<DecoratedSignature> const& signatures,
                                   SignatureBatchPrefetch const* prefetched, size_t prefetchTx)
    : mProtocolVersion(protocolVersion),
      mContentsHash(contentsHash),
      mSignatures(signatures),
      mUsedSignatures(signatures.size()),
      mPrefetched(prefetched),
      mPrefetchTx(prefetchTx) {}

bool SignatureChecker::verifyEd25519(DecoratedSignature const& sig, uint256 const& key, ByteSlice const& msg) const {
  if (mPrefetched && sig.signature.size() == 64) {
    bool v;
    if (mPrefetched->lookup(key, sig.signature, msg, v, mPrefetchTx)) return v;
  }
  PublicKey pk;
  pk.ed25519() = key;
  return PubKeyUtils::verifySig(pk, sig.signature, msg);
}

bool SignatureChecker::checkSignature(std::vector<Signer> const& signersV, int32_t neededWeight) {
#ifdef FUZZING_BUILD_MODE_UNSAFE_FOR_PRODUCTION
  return true;  // SignatureChecker.cpp:34-36: fuzz builds accept every signature
#endif
  if (mProtocolVersion == 7) return true;  // SignatureChecker.cpp:38-41

  // the reference copies the signers into per-type vectors; the same order
  // and erase semantics over pointers (stack scratch, no allocation)
  using Ptrs = InlineVec<const Signer*, 24>;
  Ptrs byType[4];
  for (auto const& s : signersV) byType[s.key.type].push_back(&s);

  int32_t totalWeight = 0;
  for (const Signer* s : byType[SIGNER_KEY_TYPE_PRE_AUTH_TX]) {  // :54-69
    if (s->key.key == mContentsHash) {
      totalWeight += (int32_t)clampWeight(mProtocolVersion, s->weight);
      if (totalWeight >= neededWeight) return true;
    }
  }

  auto verifyAll = [&](Ptrs& signers, auto&& verify) {  // :73-102
    for (size_t i = 0; i < mSignatures.size(); i++) {
      auto const& sig = mSignatures[i];
      for (auto it = signers.begin(); it != signers.end(); ++it) {
        if (verify(sig, **it)) {
          mUsedSignatures.set(i);
          totalWeight += (int32_t)clampWeight(mProtocolVersion, (*it)->weight);
          if (totalWeight >= neededWeight) return true;
          signers.erase(it);
          break;
        }
      }
    }
    return false;
  };

  if (verifyAll(byType[SIGNER_KEY_TYPE_HASH_X], [&](DecoratedSignature const& sig, Signer const& s) {
        return SignatureUtils::verifyHashX(sig, s.key);
      }))
    return true;

  if (verifyAll(byType[SIGNER_KEY_TYPE_ED25519], [&](DecoratedSignature const& sig, Signer const& s) {
        // SignatureUtils::verify, SignatureUtils.cpp:38-46
        if (std::memcmp(s.key.key.data() + 28, sig.hint.data(), 4) != 0) return false;
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
#ifdef FUZZING_BUILD_MODE_UNSAFE_FOR_PRODUCTION
  return true;  // :141-143
#endif
  if (mProtocolVersion == 7) return true;
  return mUsedSignatures.all();
}

}  // namespace stellar
