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
// verdict before it is used.  The side table is keyed by the (pk, sig, msg)
// bytes themselves (a cheap hash of them, full compare on lookup), not by the
// BLAKE2b cache key, so a checker's lookup costs no hashing.
#pragma once

#include <array>
#include <cstdint>
#include <functional>
#include <memory>
#include <utility>
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
// SignatureUtils::verify / verifyHashX / verifyEd25519SignedPayload
bool verify(DecoratedSignature const& sig, SignerKey const& signerKey, Hash const& hash);
bool verifyHashX(DecoratedSignature const& sig, SignerKey const& signerKey);
bool verifyEd25519SignedPayload(DecoratedSignature const& sig, SignerKey const& signer);
}  // namespace SignatureUtils

// Verdicts computed ahead of the checkers.
class SignatureBatchPrefetch {
 public:
  // Storage is taken from (and on destruction returned to) per-thread
  // spares, so a node building one prefetch per ledger reuses mapped pages
  // instead of faulting in fresh ones every time (measured: page faults of
  // freshly grown buffers were most of the cost of add() on a 30k-pair set).
  SignatureBatchPrefetch();
  ~SignatureBatchPrefetch();
  SignatureBatchPrefetch(SignatureBatchPrefetch const&) = delete;
  SignatureBatchPrefetch& operator=(SignatureBatchPrefetch const&) = delete;
  // Enumerate the hint-matching ed25519 / signed-payload pairs of one tx.
  void add(Hash const& contentsHash, std::vector<DecoratedSignature> const& signatures,
           std::vector<Signer> const& signers);
  // The same for a whole set of transactions, enumerated in parallel on the
  // host pool (pairs in tx order, as add() per tx would give them).  The
  // pairs of batch tx k are then also found by their position: a checker
  // constructed with prefetchTx = k (the index in txs, counted over every
  // addBatch call of this prefetch) searches them before the table.
  struct TxRef {
    Hash const* contentsHash;
    std::vector<DecoratedSignature> const* signatures;
    std::vector<Signer> const* signers;
  };
  // prepare (optional): called as prepare(k) for batch tx k on the thread that
  // enumerates it, just before, to build the tx's objects in place (the
  // tx-set entry point marshals its C structs there: one pass over each tx,
  // its objects still in that core's cache).  An exception thrown by it is
  // rethrown here once every part has finished.
  void addBatch(std::vector<TxRef> const& txs, std::function<void(size_t)> const& prepare = {});
  // One engine batch over everything added.  seedCache = false: the verdicts
  // go to the side table only (the engine is called directly, no cache
  // interaction); true: through PubKeyUtils::verifySigBatch, which also fills
  // the global verify cache (a later verifySig then hits).  An engine error
  // re-runs the batch on the CPU path.
  void run(bool seedCache = false);
  // verdict for (pk, sig, msg) if prefetched (tx: see addBatch)
  static constexpr size_t kNoTx = ~size_t(0);
  bool lookup(uint256 const& pk, Signature const& sig, ByteSlice const& msg, bool& verdict,
              size_t tx = kNoTx) const;
  size_t pairs() const { return len_.size(); }

 private:
  void buildTable();
  static constexpr size_t kAsyncTableMin = 4096;
  static uint64_t hashOf(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, size_t len);
  // (growth without zero-filling: every byte of the pair arrays is written
  // right after the resize that makes room for it)
  template <typename T>
  struct NoInit : std::allocator<T> {
    template <typename U>
    struct rebind {
      using other = NoInit<U>;
    };
    NoInit() = default;
    template <typename U>
    NoInit(NoInit<U> const&) {}
    template <typename U>
    void construct(U* p) {
      ::new ((void*)p) U;
    }
    template <typename U, typename... A>
    void construct(U* p, A&&... a) {
      ::new ((void*)p) U(std::forward<A>(a)...);
    }
  };
  template <typename T>
  using RawVec = std::vector<T, NoInit<T>>;
  struct Storage {
    RawVec<uint8_t> pk, sig, msg;
    RawVec<uint64_t> off;
    RawVec<uint32_t> len;
    std::vector<uint8_t> verdict;
    std::vector<uint32_t> table;    // open addressing: pair index + 1, 0 = empty
    std::vector<uint32_t> txBegin;  // addBatch: first pair of batch tx k (k + 1 entries)
    void clear();
  };
  static void enumerate(Storage& st, Hash const& contentsHash, std::vector<DecoratedSignature> const& signatures,
                        std::vector<Signer> const& signers);
  static std::vector<Storage>& spares();
  static constexpr size_t kSpares = 4;
  Storage st_;
  RawVec<uint8_t>& pk_ = st_.pk;
  RawVec<uint8_t>& sig_ = st_.sig;
  RawVec<uint8_t>& msg_ = st_.msg;
  RawVec<uint64_t>& off_ = st_.off;
  RawVec<uint32_t>& len_ = st_.len;
  std::vector<uint8_t>& verdict_ = st_.verdict;
  std::vector<uint32_t>& table_ = st_.table;
  std::vector<uint32_t>& txBegin_ = st_.txBegin;
  size_t mask_ = 0;
};

class SignatureChecker {
 public:
  // prefetchTx: the tx's index in the prefetch's addBatch order (its pairs
  // are then found by position), or kNoTx
  SignatureChecker(uint32_t protocolVersion, Hash const& contentsHash,
                   std::vector<DecoratedSignature> const& signatures,
                   SignatureBatchPrefetch const* prefetched = nullptr,
                   size_t prefetchTx = SignatureBatchPrefetch::kNoTx);
  bool checkSignature(std::vector<Signer> const& signersV, int32_t neededWeight);
  bool checkAllSignaturesUsed() const;

 private:
  bool verifyEd25519(DecoratedSignature const& sig, uint256 const& key, ByteSlice const& msg) const;

  uint32_t mProtocolVersion;
  Hash const& mContentsHash;
  std::vector<DecoratedSignature> const& mSignatures;
  // which signatures a match used (the reference's std::vector<bool>); a tx
  // carries at most 20 (xvector<DecoratedSignature, 20>), so the bits live
  // inline and a checker allocates nothing -- one malloc per tx was ~15 % of
  // the pre-passed checkers' time (profiles/r06/config3/)
  class UsedBits {
   public:
    explicit UsedBits(size_t n) : n_(n) {
      if (n > kInline) heap_.assign((n + 63) / 64, 0);
    }
    void set(size_t i) { words()[i >> 6] |= 1ull << (i & 63); }
    bool all() const {
      const uint64_t* w = heap_.empty() ? inline_ : heap_.data();
      for (size_t i = 0; i < n_; i += 64) {
        const size_t k = n_ - i < 64 ? n_ - i : 64;
        const uint64_t want = k == 64 ? ~0ull : ((1ull << k) - 1);
        if ((w[i >> 6] & want) != want) return false;
      }
      return true;
    }

   private:
    static constexpr size_t kInline = 128;
    uint64_t* words() { return heap_.empty() ? inline_ : heap_.data(); }
    size_t n_;
    uint64_t inline_[kInline / 64] = {0, 0};
    std::vector<uint64_t> heap_;
  };
  UsedBits mUsedSignatures;
  SignatureBatchPrefetch const* mPrefetched;
  size_t mPrefetchTx;
};

}  // namespace stellar
