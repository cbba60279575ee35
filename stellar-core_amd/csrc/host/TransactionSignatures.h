// Transaction-level signature validation restated over the checker
// (SURVEY.md §8 a13): the sequence of SignatureChecker calls stellar-core
// makes for one transaction envelope, with everything that is not a
// signature (fees, sequence numbers, balances, operation semantics) left out.
//
// Reference (TransactionFrame::checkValidWithOptionallyChargedFee path):
//   one SignatureChecker per envelope over getContentsHash()
//       /root/reference/src/transactions/TransactionFrame.cpp:1441-1443
//   source account at its LOW threshold -> txBAD_AUTH       :1247-1254 (commonValid)
//   extra signers (protocol >= 19), weight 1 each, all needed -> txBAD_AUTH
//                                                            :1256-1262, :297-321
//   every operation: its source account (op source or tx source) at the
//   operation's threshold level (OperationFrame.cpp:173-209, getNeededThreshold
//   :47-62); a missing op-source account checks the op source key alone with
//   weight 1, needed 0 (checkSignatureNoAccount :286-295); failure -> opBAD_AUTH
//   / opNO_ACCOUNT and txFAILED                              :1461-1474
//   checkAllSignaturesUsed -> txBAD_AUTH_EXTRA               :1477-1480
//   account signer list = master key (weight thresholds[0], if non-zero) +
//   account signers                                          :268-284
// Fee bump (FeeBumpTransactionFrame.cpp:138-153, :173-197, :267-287): its own
//   checker over the fee-bump contents hash and the OUTER signatures; fee source
//   at LOW -> txBAD_AUTH; unused outer signatures -> txBAD_AUTH_EXTRA; then the
//   inner transaction as above -> txFEE_BUMP_INNER_SUCCESS / _FAILED.
//
// All of a transaction's checks accumulate into ONE checker (its
// mUsedSignatures), as in the reference.  prefetchTransaction() enumerates
// every (signature, signer) pair those checks can reach, so a whole tx set is
// verified in one engine batch before the checkers run (f1).
#pragma once

#include <cstdint>
#include <cstring>
#include <optional>
#include <unordered_map>
#include <vector>

#include "SignatureChecker.h"

namespace stellar {

// TransactionResultCode / OperationResultCode values (Stellar-transaction.x)
enum TxResultCode : int32_t {
  txFEE_BUMP_INNER_SUCCESS = 1,
  txSUCCESS = 0,
  txFAILED = -1,
  txBAD_AUTH = -6,
  txNO_ACCOUNT = -8,
  txBAD_AUTH_EXTRA = -10,
  txNOT_SUPPORTED = -12,
  txFEE_BUMP_INNER_FAILED = -13,
};
enum OpResultCode : int32_t { opINNER = 0, opBAD_AUTH = -1, opNO_ACCOUNT = -2 };
enum ThresholdLevel : int32_t { THRESHOLD_LOW_LEVEL = 1, THRESHOLD_MED_LEVEL = 2, THRESHOLD_HIGH_LEVEL = 3 };

// The signature-relevant part of an AccountEntry: thresholds[0] is the master
// key weight, [1..3] the LOW / MEDIUM / HIGH thresholds.
struct AccountSigState {
  uint256 accountID{};
  uint8_t thresholds[4] = {1, 0, 0, 0};
  std::vector<Signer> signers;
};

struct Uint256Hash {
  size_t operator()(uint256 const& k) const {
    size_t v;
    std::memcpy(&v, k.data(), sizeof v);
    return v;
  }
};
using AccountSnapshot = std::unordered_map<uint256, AccountSigState, Uint256Hash>;

struct OperationSigInfo {
  std::optional<uint256> sourceAccount;  // none: the transaction's source
  ThresholdLevel level = THRESHOLD_MED_LEVEL;
};

struct TransactionSigInfo {
  Hash contentsHash{};
  uint256 sourceAccount{};
  std::vector<DecoratedSignature> signatures;
  std::vector<OperationSigInfo> operations;
  std::vector<SignerKey> extraSigners;  // PreconditionsV2::extraSigners
};

struct FeeBumpSigInfo {
  Hash contentsHash{};  // of the fee-bump envelope
  uint256 feeSource{};
  std::vector<DecoratedSignature> signatures;  // outer
  TransactionSigInfo inner;
};

struct TxSigResult {
  int32_t code = txSUCCESS;
  int32_t innerCode = txSUCCESS;  // fee bump: the inner transaction's code
  int32_t failedOp = -1;          // txFAILED: first failing operation
  int32_t opCode = opINNER;
};

// forApply = false: the validation path (checkValid: operations fast-fail on
// the first invalid one).  forApply = true: the apply path
// (TransactionFrame::apply -> processSignatures, TransactionFrame.cpp:1091-1156:
// no operation checks before protocol 10, then every operation checked, no
// fast fail).  Both paths check operations with OperationFrame::checkSignature's
// forApply = false rule (processSignatures passes false, :1130-1131): a missing
// op-source account named by the operation is checked by its key alone
// (checkSignatureNoAccount), and only a missing transaction source -- no
// op source set -- is opNO_ACCOUNT (OperationFrame.cpp:186-207).
TxSigResult checkTransactionSignatures(TransactionSigInfo const& tx, AccountSnapshot const& accounts,
                                       uint32_t protocol, SignatureBatchPrefetch const* prefetched = nullptr,
                                       bool forApply = false);
TxSigResult checkFeeBumpSignatures(FeeBumpSigInfo const& tx, AccountSnapshot const& accounts, uint32_t protocol,
                                   SignatureBatchPrefetch const* prefetched = nullptr, bool forApply = false);

// Adds every (signature, signer) pair the checks of `tx` can reach.
void prefetchTransaction(SignatureBatchPrefetch& pre, TransactionSigInfo const& tx,
                         AccountSnapshot const& accounts);
void prefetchFeeBump(SignatureBatchPrefetch& pre, FeeBumpSigInfo const& tx, AccountSnapshot const& accounts);

}  // namespace stellar
