// See TransactionSignatures.h.  Restates the signature checks of
// /root/reference/src/transactions/TransactionFrame.cpp:268-321 (checkSignature,
// checkSignatureNoAccount, checkExtraSigners), :1247-1262 (commonValid),
// :1416-1486 (checkValidWithOptionallyChargedFee),
// OperationFrame.cpp:47-62,173-209 and FeeBumpTransactionFrame.cpp:138-197,267-287.
#include "TransactionSignatures.h"

namespace stellar {
namespace {

// TransactionFrame::checkSignature: master key (if its weight is non-zero)
// then the account's signers
std::vector<Signer> accountSigners(AccountSigState const& acc) {
  std::vector<Signer> signers;
  if (acc.thresholds[0]) {
    Signer m;
    m.key.type = SIGNER_KEY_TYPE_ED25519;
    m.key.key = acc.accountID;
    m.weight = acc.thresholds[0];
    signers.push_back(m);
  }
  signers.insert(signers.end(), acc.signers.begin(), acc.signers.end());
  return signers;
}

AccountSigState const* find(AccountSnapshot const& accounts, uint256 const& id) {
  auto it = accounts.find(id);
  return it == accounts.end() ? nullptr : &it->second;
}

std::vector<Signer> extraSignerList(std::vector<SignerKey> const& keys) {
  std::vector<Signer> signers;
  for (auto const& k : keys) {
    Signer s;
    s.key = k;
    s.weight = 1;
    signers.push_back(s);
  }
  return signers;
}

Signer noAccountSigner(uint256 const& id) {
  Signer s;
  s.key.type = SIGNER_KEY_TYPE_ED25519;
  s.key.key = id;
  s.weight = 1;
  return s;
}

}  // namespace

TxSigResult checkTransactionSignatures(TransactionSigInfo const& tx, AccountSnapshot const& accounts,
                                       uint32_t protocol, SignatureBatchPrefetch const* prefetched, bool forApply) {
  TxSigResult r;
  SignatureChecker checker(protocol, tx.contentsHash, tx.signatures, prefetched);
  AccountSigState const* src = find(accounts, tx.sourceAccount);
  if (!src) {  // commonValidPreSeqNum
    r.code = txNO_ACCOUNT;
    return r;
  }
  if (!checker.checkSignature(accountSigners(*src), src->thresholds[THRESHOLD_LOW_LEVEL])) {
    r.code = txBAD_AUTH;
    return r;
  }
  if (protocol >= 19 && !tx.extraSigners.empty() &&
      !checker.checkSignature(extraSignerList(tx.extraSigners), (int32_t)tx.extraSigners.size())) {
    r.code = txBAD_AUTH;
    return r;
  }
  if (forApply && protocol < 10) return r;  // processSignatures, TransactionFrame.cpp:1100-1103
  for (size_t i = 0; i < tx.operations.size(); ++i) {
    auto const& op = tx.operations[i];
    uint256 const& id = op.sourceAccount ? *op.sourceAccount : tx.sourceAccount;
    AccountSigState const* acc = find(accounts, id);
    bool ok;
    int32_t opc = opINNER;
    if (acc) {
      ok = checker.checkSignature(accountSigners(*acc), acc->thresholds[op.level]);
      if (!ok) opc = opBAD_AUTH;
    } else if (!op.sourceAccount) {
      // (processSignatures calls OperationFrame::checkSignature with
      // forApply = false, TransactionFrame.cpp:1130-1131: a missing op-source
      // account is checked by its key alone in BOTH modes; only a missing
      // transaction source gives opNO_ACCOUNT, OperationFrame.cpp:194-198)
      ok = false;
      opc = opNO_ACCOUNT;
    } else {
      ok = checker.checkSignature({noAccountSigner(id)}, 0);
      if (!ok) opc = opBAD_AUTH;
    }
    if (!ok && r.code != txFAILED) {
      r.code = txFAILED;
      r.failedOp = (int32_t)i;
      r.opCode = opc;
      if (!forApply) return r;  // checkValid fast-fails on the first invalid operation
    }
  }
  if (r.code == txFAILED) return r;
  if (!checker.checkAllSignaturesUsed()) r.code = txBAD_AUTH_EXTRA;
  return r;
}

TxSigResult checkFeeBumpSignatures(FeeBumpSigInfo const& tx, AccountSnapshot const& accounts, uint32_t protocol,
                                   SignatureBatchPrefetch const* prefetched, bool forApply) {
  TxSigResult r;
  if (protocol < 13) {
    r.code = txNOT_SUPPORTED;
    return r;
  }
  SignatureChecker checker(protocol, tx.contentsHash, tx.signatures, prefetched);
  AccountSigState const* fee = find(accounts, tx.feeSource);
  if (!fee) {
    r.code = txNO_ACCOUNT;
    return r;
  }
  if (!checker.checkSignature(accountSigners(*fee), fee->thresholds[THRESHOLD_LOW_LEVEL])) {
    r.code = txBAD_AUTH;
    return r;
  }
  if (!checker.checkAllSignaturesUsed()) {
    r.code = txBAD_AUTH_EXTRA;
    return r;
  }
  TxSigResult inner = checkTransactionSignatures(tx.inner, accounts, protocol, prefetched, forApply);
  r.code = inner.code == txSUCCESS ? txFEE_BUMP_INNER_SUCCESS : txFEE_BUMP_INNER_FAILED;
  r.innerCode = inner.code;
  r.failedOp = inner.failedOp;
  r.opCode = inner.opCode;
  return r;
}

void prefetchTransaction(SignatureBatchPrefetch& pre, TransactionSigInfo const& tx, AccountSnapshot const& accounts) {
  std::vector<Signer> all;
  auto addAccount = [&](uint256 const& id, bool noAccountKey) {
    if (AccountSigState const* a = find(accounts, id)) {
      auto s = accountSigners(*a);
      all.insert(all.end(), s.begin(), s.end());
    } else if (noAccountKey) {
      all.push_back(noAccountSigner(id));
    }
  };
  addAccount(tx.sourceAccount, false);
  for (auto const& op : tx.operations)
    if (op.sourceAccount) addAccount(*op.sourceAccount, true);
  auto extra = extraSignerList(tx.extraSigners);
  all.insert(all.end(), extra.begin(), extra.end());
  // the same (key, payload) reached twice would only duplicate pairs
  std::vector<Signer> uniq;
  for (auto const& s : all) {
    bool dup = false;
    for (auto const& u : uniq)
      if (u.key.type == s.key.type && u.key.key == s.key.key && u.key.payload == s.key.payload) {
        dup = true;
        break;
      }
    if (!dup) uniq.push_back(s);
  }
  pre.add(tx.contentsHash, tx.signatures, uniq);
}

void prefetchFeeBump(SignatureBatchPrefetch& pre, FeeBumpSigInfo const& tx, AccountSnapshot const& accounts) {
  if (AccountSigState const* a = find(accounts, tx.feeSource)) pre.add(tx.contentsHash, tx.signatures, accountSigners(*a));
  prefetchTransaction(pre, tx.inner, accounts);
}

}  // namespace stellar
