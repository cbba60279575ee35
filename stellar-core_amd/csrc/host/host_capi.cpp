// extern "C" surface of libstellar_host.so (the C++ PubKeyUtils /
// SignatureChecker / transaction-signature mirror), for bindings and tests.
// Declared in include/stellar_host.h.  C++ exceptions never cross this
// boundary.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <atomic>
#include <exception>
#include <future>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/stellar_host.h"
#include "HostPool.h"
#include "PubKeyUtils.h"
#include "SignatureChecker.h"
#include "TransactionSignatures.h"
#include "VerifyMicroBatcher.h"
#include "hashes.h"

using namespace stellar;

namespace {

// SV_HOST_TRACE: phase timings of the tx-set entry points to stderr
const bool gPhaseTrace = getenv("SV_HOST_TRACE") != nullptr;
struct PhaseClock {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  // returns the lap in ms
  double lap(const char* what) {
    const auto now = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(now - t).count();
    if (gPhaseTrace) fprintf(stderr, "[svh] %-28s %8.3f ms\n", what, ms);
    t = now;
    return ms;
  }
};
// phases of this thread's last svh_check_txset (svh_txset_last_phases)
thread_local double t_txset_phases[4] = {0, 0, 0, 0};
thread_local std::string t_err;
int guard_exc(std::exception const& e) {
  t_err = e.what();
  return SVH_ERR_INVALID_ARG;
}

// hostParallelFor whose pieces may throw: the first exception is rethrown on
// this thread once every piece has returned (an exception must not leave a
// pool thread)
void parallelOrThrow(size_t n, size_t grain, std::function<void(size_t, size_t)> const& range) {
  std::exception_ptr first;
  std::mutex mu;
  hostParallelFor(n, grain, [&](size_t a, size_t b) {
    try {
      range(a, b);
    } catch (...) {
      std::lock_guard<std::mutex> g(mu);
      if (!first) first = std::current_exception();
    }
  });
  if (first) std::rethrow_exception(first);
}

// (in place: the tx-set marshal builds ~30k of each per call)
void decoratedInto(DecoratedSignature& d, svh_decorated_sig const& s) {
  if (s.sig_len > 64) throw std::invalid_argument("signature longer than 64 bytes");
  std::memcpy(d.hint.data(), s.hint, 4);
  d.signature.assign(s.sig, s.sig + s.sig_len);
}
void signerInto(Signer& g, svh_signer const& s) {
  if (s.type > 3 || s.payload_len > 64) throw std::invalid_argument("bad signer");
  g.key.type = (SignerKeyType)s.type;
  std::memcpy(g.key.key.data(), s.key, 32);
  g.key.payload.assign(s.payload, s.payload + s.payload_len);
  g.weight = s.weight;
}
Signer signer(svh_signer const& s) {
  Signer g;
  signerInto(g, s);
  return g;
}

std::vector<DecoratedSignature> sigRange(const svh_decorated_sig* sigs, uint32_t off, uint32_t n) {
  std::vector<DecoratedSignature> v(n);
  for (uint32_t k = 0; k < n; ++k) decoratedInto(v[k], sigs[off + k]);
  return v;
}

uint256 u256(const uint8_t* p) {
  uint256 u;
  std::memcpy(u.data(), p, 32);
  return u;
}
}  // namespace

extern "C" {

const char* svh_last_error_string(void) { return t_err.c_str(); }

void svh_blake2b256(uint8_t out[32], const uint8_t* p, size_t n) {
  auto h = hostcrypto::blake2b256(p, n);
  std::memcpy(out, h.data(), 32);
}

void svh_sha256(uint8_t out[32], const uint8_t* p, size_t n) {
  auto h = hostcrypto::sha256(p, n);
  std::memcpy(out, h.data(), 32);
}

int svh_verify_sig(const uint8_t pk[32], const uint8_t* sig, size_t sig_len, const uint8_t* msg, size_t msg_len) {
  try {
    // (verifySig rejects any size but 64 before touching the cache,
    // SecretKey.cpp:441-444; an XDR opaque<64> cannot hold more)
    if (sig_len > Signature::kMax) return 0;
    PublicKey k;
    std::memcpy(k.ed25519().data(), pk, 32);
    Signature s(sig, sig + sig_len);
    return PubKeyUtils::verifySig(k, s, ByteSlice(msg, msg_len)) ? 1 : 0;
  } catch (std::exception const& e) {
    return guard_exc(e);
  }
}

int svh_bench_verify_hits(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, size_t msg_len, size_t n,
                          int passes, int threads, double* hits_per_s, double* fill_s) {
  try {
    if (!pk || !sig || (!msg && msg_len) || !hits_per_s || passes < 2 || threads < 1) return SVH_ERR_INVALID_ARG;
    std::vector<PublicKey> keys(n);
    std::vector<Signature> sigs(n);
    for (size_t i = 0; i < n; ++i) {
      std::memcpy(keys[i].ed25519().data(), pk + 32 * i, 32);
      sigs[i] = Signature(sig + 64 * i, sig + 64 * i + 64);
    }
    auto one = [&](size_t i) {
      return PubKeyUtils::verifySig(keys[i], sigs[i], ByteSlice(msg + i * msg_len, msg_len));
    };
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    bool ok = true;
    for (size_t i = 0; i < n; ++i) ok = one(i) && ok;  // pass 0: misses (SecretKey.cpp:221-225)
    const auto t1 = clk::now();
    if (fill_s) *fill_s = std::chrono::duration<double>(t1 - t0).count();
    std::atomic<bool> all{ok};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] {
        bool good = true;
        const size_t start = n * (size_t)t / (size_t)threads;
        for (int pass = 1; pass < passes; ++pass)
          for (size_t k = 0; k < n; ++k) good = one((start + k) % n) && good;
        if (!good) all.store(false);
      });
    for (auto& x : th) x.join();
    const double dt = std::chrono::duration<double>(clk::now() - t1).count();
    *hits_per_s = (double)n * (double)(passes - 1) * (double)threads / dt;
    return all.load() ? 0 : SVH_ERR_INVALID_ARG;
  } catch (std::exception const& e) {
    return guard_exc(e);
  }
}

int svh_verify_sig_batch(const uint8_t* pk, const uint8_t* sig, const uint32_t* sig_len, const uint8_t* msg,
                         const uint64_t* msg_off, const uint32_t* msg_len, size_t n, uint8_t* verdict) {
  try {
    std::vector<PublicKey> keys(n);
    std::vector<PubKeyUtils::VerifyItem> items(n);
    for (size_t i = 0; i < n; ++i) {
      std::memcpy(keys[i].ed25519().data(), pk + 32 * i, 32);
      const uint32_t sl = sig_len ? sig_len[i] : 64;
      if (sl > 64) throw std::invalid_argument("signature longer than 64 bytes");
      items[i] = PubKeyUtils::VerifyItem{&keys[i], ByteSlice(sig + 64 * i, sl), ByteSlice(msg + msg_off[i], msg_len[i])};
    }
    auto v = PubKeyUtils::verifySigBatch(items);
    for (size_t i = 0; i < n; ++i) verdict[i] = v[i] ? 1 : 0;
    return SVH_OK;
  } catch (std::exception const& e) {
    return guard_exc(e);
  }
}

int svh_verify_uncached(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                        const uint32_t* msg_len, size_t n, uint8_t* verdict) {
  try {
    PubKeyUtils::verifyBatchUncached(pk, sig, msg, msg_off, msg_len, n, verdict);
    return SVH_OK;
  } catch (std::exception const& e) {
    return guard_exc(e);
  }
}

void svh_cache_clear(void) { PubKeyUtils::clearVerifySigCache(); }
void svh_cache_seed(unsigned int seed) { PubKeyUtils::maybeSeedVerifySigCache(seed); }
void svh_cache_counts(uint64_t* hits, uint64_t* misses) {
  uint64_t h, m;
  PubKeyUtils::flushVerifySigCacheCounts(h, m);
  if (hits) *hits = h;
  if (misses) *misses = m;
}
size_t svh_cache_keys(uint8_t* out, size_t max_keys) {
  auto keys = PubKeyUtils::cacheKeysForTesting();
  const size_t n = std::min(max_keys, keys.size());
  for (size_t i = 0; i < n; ++i) std::memcpy(out + 32 * i, keys[i].data(), 32);
  return keys.size();
}
void svh_engine_counts(uint64_t* sigs, uint64_t* batches) {
  uint64_t s, b;
  PubKeyUtils::flushEngineCounts(s, b);
  if (sigs) *sigs = s;
  if (batches) *batches = b;
}
void svh_engine_counts_ex(svh_engine_stats* out) {
  auto c = PubKeyUtils::flushEngineCounts();
  if (out) {
    out->gpu_signatures = c.gpuSignatures;
    out->gpu_batches = c.gpuBatches;
    out->cpu_signatures = c.cpuSignatures;
    out->fallbacks = c.fallbacks;
  }
}
void svh_engine_histograms(uint64_t out[4 * 32]) {
  const auto h = PubKeyUtils::flushEngineHistograms();
  static_assert(PubKeyUtils::EngineHistograms::kBuckets == 32, "svh_engine_histograms layout");
  if (!out) return;
  for (int b = 0; b < 32; ++b) {
    out[b] = h.gpuBatchSize[b];
    out[32 + b] = h.gpuLatencyUs[b];
    out[64 + b] = h.cpuBatchSize[b];
    out[96 + b] = h.cpuLatencyUs[b];
  }
}
void svh_set_test_verifier(svh_batch_verify_fn fn) { PubKeyUtils::setBatchVerifierForTesting(fn); }
void svh_set_test_keyed_verifier(svh_keyed_verify_fn fn) { PubKeyUtils::setKeyedBatchVerifierForTesting(fn); }
void svh_set_keyed_threshold(size_t min_items) { PubKeyUtils::setKeyedBatchThreshold(min_items); }
void svh_set_cpu_threshold(size_t max_misses) { PubKeyUtils::setCpuBatchThreshold(max_misses); }

// Below this many transactions the pipelined pre-pass (use_prefetch 4) runs
// as one batch: its halves would leave the engine's lane and the pool idle.
constexpr size_t kPipelineMinTxs = 1024;

// One helper thread per calling thread, kept for that thread's life: the
// pipelined pre-pass runs its engine calls on it (a thread created per call
// cost tens of microseconds on a loaded host).  start() hands it one task;
// wait() returns when it is done and rethrows what it threw.
class CallHelper {
 public:
  CallHelper() : thread_([this] { loop(); }) {}
  ~CallHelper() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    thread_.join();
  }
  void start(std::function<void()> f) {
    std::lock_guard<std::mutex> g(mu_);
    task_ = std::move(f);
    err_ = nullptr;
    pending_ = true;
    done_ = false;
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return done_; });
    if (err_) std::rethrow_exception(err_);
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || pending_; });
      if (stop_) return;
      std::function<void()> f = std::move(task_);
      pending_ = false;
      lk.unlock();
      std::exception_ptr e;
      try {
        f();
      } catch (...) {
        e = std::current_exception();
      }
      lk.lock();
      err_ = e;
      done_ = true;
      cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::function<void()> task_;
  std::exception_ptr err_;
  bool pending_ = false, done_ = true, stop_ = false;
  std::thread thread_;  // (last: started once the state above exists)
};

int svh_check_txset(const svh_tx* txs, size_t ntx, const svh_decorated_sig* sigs, const svh_signer* signers,
                    int use_prefetch, uint8_t* ok, uint8_t* all_used, uint64_t* prefetched_pairs) {
  try {
    PhaseClock pc;
    // the mirror's tx objects, kept per thread from call to call: a node
    // holds them anyway, and building then freeing ~10k small vectors per set
    // measured ~1 ms of the call on this container (their destructors ran
    // after the last phase)
    thread_local std::vector<Hash> tlHashes;
    thread_local std::vector<std::vector<DecoratedSignature>> tlSigs;
    thread_local std::vector<std::vector<Signer>> tlSigners;
    // (local references: a lambda names a thread_local directly, so on the
    // pool's threads it would see their own, empty, instances)
    std::vector<Hash>& hashes = tlHashes;
    std::vector<std::vector<DecoratedSignature>>& dsigs = tlSigs;
    std::vector<std::vector<Signer>>& sgn = tlSigners;
    if (hashes.size() < ntx) {
      hashes.resize(ntx);
      dsigs.resize(ntx);
      sgn.resize(ntx);
    }
    // the C structs -> the mirror's C++ objects (a node already holds these
    // objects; the tx set is independent per tx from here on)
    auto marshal = [&](size_t t) {
      // (a tx holds at most 20 signatures and 20 + 1 + 2 signers: with that
      // capacity kept, a new set's objects are built in place, never
      // reallocated -- fresh allocations on the pool's threads, first-touch
      // faults included, were most of this phase for sets seen once:
      // profiles/r06/config3/)
      if (dsigs[t].capacity() < 20) dsigs[t].reserve(20);
      if (sgn[t].capacity() < 24) sgn[t].reserve(24);
      // the C structs of a later tx of this range, on their way from memory
      if (t + 2 < ntx) {
        const svh_tx& nx = txs[t + 2];
        const char* a = (const char*)(sigs + nx.sig_off);
        for (size_t b = 0; b < sizeof(svh_decorated_sig) * nx.nsigs; b += 64) __builtin_prefetch(a + b);
        const char* g = (const char*)(signers + nx.signer_off);
        for (size_t b = 0; b < sizeof(svh_signer) * nx.nsigners; b += 64) __builtin_prefetch(g + b);
      }
      std::memcpy(hashes[t].data(), txs[t].contents_hash, 32);
      dsigs[t].resize(txs[t].nsigs);
      for (uint32_t k = 0; k < txs[t].nsigs; ++k) decoratedInto(dsigs[t][k], sigs[txs[t].sig_off + k]);
      sgn[t].resize(txs[t].nsigners);
      for (uint32_t k = 0; k < txs[t].nsigners; ++k) signerInto(sgn[t][k], signers[txs[t].signer_off + k]);
    };
    double ph[4] = {0, 0, 0, 0};
    // use_prefetch 4: the side-table pre-pass in two halves, pipelined -- the
    // engine verifies half 0's pairs while half 1 is enumerated, and half 1's
    // while half 0's checkers run (each half its own prefetch, so neither's
    // storage moves under the other's engine call).  Same pairs, verdicts and
    // checker outcomes as mode 1; smaller sets run as mode 1.
    if (use_prefetch == 4 && ntx >= kPipelineMinTxs) {
      const size_t half = ntx / 2, lo[2] = {0, half}, hi[2] = {half, ntx};
      SignatureBatchPrefetch pres[2];
      std::vector<SignatureBatchPrefetch::TxRef> refs(ntx);
      for (size_t t = 0; t < ntx; ++t) refs[t] = {&hashes[t], &dsigs[t], &sgn[t]};
      ph[0] = pc.lap("txset: marshal (alloc)");
      auto enumerate = [&](int h) {
        std::vector<SignatureBatchPrefetch::TxRef> part(refs.begin() + (ptrdiff_t)lo[h],
                                                        refs.begin() + (ptrdiff_t)hi[h]);
        pres[h].addBatch(part, [&, h](size_t k) { marshal(lo[h] + k); });
      };
      auto checkers = [&](int h) {
        parallelOrThrow(hi[h] - lo[h], 128, [&, h](size_t a, size_t b) {
          for (size_t t = lo[h] + a; t < lo[h] + b; ++t) {
            SignatureChecker c(txs[t].protocol, hashes[t], dsigs[t], &pres[h], t - lo[h]);
            ok[t] = c.checkSignature(sgn[t], txs[t].needed_weight) ? 1 : 0;
            all_used[t] = c.checkAllSignaturesUsed() ? 1 : 0;
          }
        });
      };
      // the engine calls run on this thread's helper; an exception in either
      // is rethrown by wait(), after this thread's own part has finished
      thread_local CallHelper helper;
      enumerate(0);
      ph[1] = pc.lap("txset: half 0 marshal + prefetch add");
      helper.start([&] { pres[0].run(false); });
      std::exception_ptr failed;
      try {
        enumerate(1);
      } catch (...) {
        failed = std::current_exception();
      }
      helper.wait();
      if (failed) std::rethrow_exception(failed);
      helper.start([&] { pres[1].run(false); });
      try {
        checkers(0);
      } catch (...) {
        failed = std::current_exception();
      }
      helper.wait();
      if (failed) std::rethrow_exception(failed);
      ph[2] = pc.lap("txset: engine 0 | half 1 add, engine 1 | half 0 checkers");
      checkers(1);
      ph[3] = pc.lap("txset: half 1 checkers");
      if (prefetched_pairs) *prefetched_pairs = pres[0].pairs() + pres[1].pairs();
      std::memcpy(t_txset_phases, ph, sizeof ph);
      return SVH_OK;
    }
    if (use_prefetch == 4) use_prefetch = 1;
    SignatureBatchPrefetch pre;
    if (use_prefetch) {
      // with the pre-pass each tx is marshalled by the pool thread that
      // enumerates its pairs, just before (one parallel pass; phase 0 is
      // then only the allocation, phase 1 both)
      std::vector<SignatureBatchPrefetch::TxRef> refs(ntx);
      for (size_t t = 0; t < ntx; ++t) refs[t] = {&hashes[t], &dsigs[t], &sgn[t]};
      ph[0] = pc.lap("txset: marshal (alloc)");
      pre.addBatch(refs, marshal);
      ph[1] = pc.lap("txset: marshal + prefetch add");
      pre.run(use_prefetch == 2);
      ph[2] = pc.lap("txset: prefetch run");
    } else {
      parallelOrThrow(ntx, 256, [&](size_t a, size_t b) {
        for (size_t t = a; t < b; ++t) marshal(t);
      });
      ph[0] = pc.lap("txset: marshal");
    }
    if (prefetched_pairs) *prefetched_pairs = pre.pairs();
    auto check = [&](size_t a, size_t b) {
      for (size_t t = a; t < b; ++t) {
        SignatureChecker c(txs[t].protocol, hashes[t], dsigs[t], use_prefetch ? &pre : nullptr,
                           use_prefetch == 1 || use_prefetch == 2 ? t : SignatureBatchPrefetch::kNoTx);
        ok[t] = c.checkSignature(sgn[t], txs[t].needed_weight) ? 1 : 0;
        all_used[t] = c.checkAllSignaturesUsed() ? 1 : 0;
      }
    };
    // With the pre-pass every checker only reads the side table, independent
    // of the others: they run on the host pool.  Without it (the reference's
    // flow: one verifySig per signature) they run in tx order on this thread.
    if (use_prefetch) parallelOrThrow(ntx, 128, check);
    else check(0, ntx);
    ph[3] = pc.lap("txset: checkers");
    std::memcpy(t_txset_phases, ph, sizeof ph);
    return SVH_OK;
  } catch (std::exception const& e) {
    return guard_exc(e);
  }
}

void svh_txset_last_phases(double out[4]) { std::memcpy(out, t_txset_phases, sizeof t_txset_phases); }

int svh_check_envelopes(const svh_envelope* env, size_t n, const svh_decorated_sig* sigs, const svh_op* ops,
                        const svh_signer* signers, const svh_account* accounts, size_t naccounts,
                        uint32_t protocol, int prefetch, int for_apply, svh_tx_result* results,
                        uint64_t* prefetched_pairs) {
  try {
    AccountSnapshot snap;
    snap.reserve(naccounts);
    for (size_t a = 0; a < naccounts; ++a) {
      AccountSigState st;
      st.accountID = u256(accounts[a].account_id);
      std::memcpy(st.thresholds, accounts[a].thresholds, 4);
      for (uint32_t k = 0; k < accounts[a].nsigners; ++k)
        st.signers.push_back(signer(signers[accounts[a].signer_off + k]));
      snap[st.accountID] = std::move(st);
    }
    std::vector<FeeBumpSigInfo> txs(n);
    for (size_t t = 0; t < n; ++t) {
      svh_envelope const& e = env[t];
      TransactionSigInfo& in = txs[t].inner;
      std::memcpy(in.contentsHash.data(), e.contents_hash, 32);
      in.sourceAccount = u256(e.source);
      in.signatures = sigRange(sigs, e.sig_off, e.nsigs);
      for (uint32_t k = 0; k < e.nops; ++k) {
        svh_op const& o = ops[e.op_off + k];
        if (o.level < 1 || o.level > 3) throw std::invalid_argument("bad threshold level");
        OperationSigInfo op;
        if (o.has_source) op.sourceAccount = u256(o.source);
        op.level = (ThresholdLevel)o.level;
        in.operations.push_back(op);
      }
      for (uint32_t k = 0; k < e.nextra; ++k) in.extraSigners.push_back(signer(signers[e.extra_off + k]).key);
      if (e.fee_bump) {
        std::memcpy(txs[t].contentsHash.data(), e.fee_bump_hash, 32);
        txs[t].feeSource = u256(e.fee_source);
        txs[t].signatures = sigRange(sigs, e.outer_off, e.nouter);
      }
    }
    SignatureBatchPrefetch pre;
    if (prefetch) {
      for (size_t t = 0; t < n; ++t) {
        if (env[t].fee_bump) prefetchFeeBump(pre, txs[t], snap);
        else prefetchTransaction(pre, txs[t].inner, snap);
      }
      pre.run(prefetch == 2);
    }
    if (prefetched_pairs) *prefetched_pairs = pre.pairs();
    SignatureBatchPrefetch const* p = prefetch ? &pre : nullptr;
    auto check = [&](size_t a, size_t b) {
      for (size_t t = a; t < b; ++t) {
        TxSigResult r = env[t].fee_bump ? checkFeeBumpSignatures(txs[t], snap, protocol, p, for_apply != 0)
                                        : checkTransactionSignatures(txs[t].inner, snap, protocol, p, for_apply != 0);
        results[t].code = r.code;
        results[t].inner_code = r.innerCode;
        results[t].failed_op = r.failedOp;
        results[t].op_code = r.opCode;
      }
    };
    // (as svh_check_txset: with the pre-pass the checkers only read the side
    // table and the account snapshot, so they run on the host pool)
    if (prefetch) parallelOrThrow(n, 128, check);
    else check(0, n);
    return SVH_OK;
  } catch (std::exception const& e) {
    return guard_exc(e);
  }
}

int svh_mb_run_ex(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                  const uint32_t* msg_len, size_t n, int producers, int workers, uint32_t max_batch,
                  uint32_t max_delay_us, uint32_t inter_arrival_us, int fire_and_forget, uint8_t* verdict,
                  svh_mb_stats* stats) {
  try {
    if (producers < 1) producers = 1;
    if (workers < 1) workers = 1;
    std::vector<int> err(producers, 0);
    std::vector<std::string> msgs(producers);
    // (the round-2 deadline policy: these entry points' callers and tests
    // count size and deadline flushes; svh_scp_run drives the WhenIdle default)
    VerifyMicroBatcher mb(max_batch, std::chrono::microseconds(max_delay_us), (unsigned)workers,
                          /*recordLatency=*/!fire_and_forget, VerifyMicroBatcher::FlushPolicy::Deadline);
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int p = 0; p < producers; ++p) {
      th.emplace_back([&, p] {
        std::vector<std::pair<size_t, std::future<bool>>> futs;
        PublicKey k;
        for (size_t i = (size_t)p; i < n; i += (size_t)producers) {
          std::memcpy(k.ed25519().data(), pk + 32 * i, 32);
          const ByteSlice s(sig + 64 * i, 64);
          const ByteSlice m(msg + msg_off[i], msg_len[i]);
          if (fire_and_forget) mb.post(k, s, m);
          else futs.emplace_back(i, mb.submit(k, s, m));
          if (inter_arrival_us) std::this_thread::sleep_for(std::chrono::microseconds(inter_arrival_us));
        }
        try {
          for (auto& f : futs) verdict[f.first] = f.second.get() ? 1 : 0;
        } catch (std::exception const& e) {
          err[p] = 1;
          msgs[p] = e.what();
        }
      });
    }
    for (auto& t : th) t.join();
    // futures resolve before their worker books the batch in the stats: drain in
    // both modes so the stats below cover every item
    mb.drain();
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int p = 0; p < producers; ++p)
      if (err[p]) {
        t_err = msgs[p];
        return SVH_ERR_ENGINE;
      }
    if (fire_and_forget && verdict) {
      // the verdicts were only cached: read them back like the reference's
      // later verifyEnvelope would (cache hits)
      for (size_t i = 0; i < n; ++i) {
        PublicKey k;
        std::memcpy(k.ed25519().data(), pk + 32 * i, 32);
        Signature s(sig + 64 * i, sig + 64 * i + 64);
        verdict[i] = PubKeyUtils::verifySig(k, s, ByteSlice(msg + msg_off[i], msg_len[i])) ? 1 : 0;
      }
    }
    if (stats) {
      auto s = mb.stats();
      stats->items = s.items;
      stats->batches = s.batches;
      stats->flushed_by_size = s.flushedBySize;
      stats->flushed_by_deadline = s.flushedByDeadline;
      stats->max_batch = s.maxBatchSeen;
      std::vector<double> lat = mb.latencies();
      std::sort(lat.begin(), lat.end());
      stats->lat_p50_us = lat.empty() ? 0 : lat[lat.size() / 2];
      stats->lat_p99_us = lat.empty() ? 0 : lat[std::min(lat.size() - 1, (size_t)(lat.size() * 0.99))];
      stats->wall_s = wall;
    }
    return SVH_OK;
  } catch (std::exception const& e) {
    return guard_exc(e);
  }
}

int svh_scp_run(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                const uint32_t* msg_len, size_t n, const svh_scp_params* prm, uint8_t* verdict, svh_scp_result* res) {
  try {
    if (!prm || !res || prm->struct_size < offsetof(svh_scp_params, batch_post) || n == 0 || !pk || !sig ||
        !msg_off || !msg_len)
      throw std::invalid_argument("svh_scp_run: bad arguments");
    const bool batchPost = prm->struct_size >= sizeof(svh_scp_params) && prm->batch_post != 0;
    using Clk = std::chrono::steady_clock;
    const unsigned P = std::max(1u, prm->producers);
    const size_t B = prm->burst ? prm->burst : n;
    VerifyMicroBatcher::Options o;
    o.maxBatch = prm->max_batch ? prm->max_batch : 8192;
    o.maxDelay = std::chrono::microseconds(prm->max_delay_us);
    o.workers = std::max(1u, prm->workers);
    o.policy = prm->policy == 1 ? VerifyMicroBatcher::FlushPolicy::Deadline : VerifyMicroBatcher::FlushPolicy::WhenIdle;
    o.idleInFlight = std::max(1u, prm->idle_in_flight);
    o.linger = std::chrono::microseconds(prm->linger_us);
    o.quiet = std::chrono::microseconds(prm->quiet_us);
    o.maxLinger = std::chrono::microseconds(prm->max_linger_us);
    o.recordLatency = true;  // (submit -> the batch's verdicts are in the cache, before its continuations run)
    std::vector<Clk::time_point> tSub(n), tVer(n), tMain(n);
    std::vector<uint8_t> cbVerdict(n, 2);
    // the main thread's queue (Peer::recvMessage posted by the continuation)
    // (as an event loop's post: the waiting thread is woken only when it
    // sleeps; a busy one finds the new items on its next pass -- a wake-up
    // per item costs each continuation a futex call)
    std::mutex qm;
    std::condition_variable qcv;
    std::vector<size_t> q;
    bool mainWaiting = false;
    q.reserve(n);
    (void)PubKeyUtils::flushEngineCounts();  // (the run's own counts are read at the end)
    std::vector<uint8_t> out(n, 2);
    uint64_t hits = 0, misses = 0, mismatches = 0;
    std::vector<double> mainCallUs;
    mainCallUs.reserve(n);
    const Clk::time_point T0 = Clk::now() + std::chrono::milliseconds(2);
    VerifyMicroBatcher::Stats st;
    if (batchPost)  // one main-thread post per verified batch (the envelopes in batch order)
      o.onBatch = [&](const uint64_t* tags, const uint8_t* v, size_t m) {
        const auto t = Clk::now();
        for (size_t j = 0; j < m; ++j) {
          tVer[tags[j]] = t;
          cbVerdict[tags[j]] = v[j];
        }
        bool wake;
        {
          std::lock_guard<std::mutex> g(qm);
          q.insert(q.end(), tags, tags + m);
          wake = mainWaiting;
        }
        if (wake) qcv.notify_one();
      };
    {
      VerifyMicroBatcher mb(o);
      // the main thread: HerderImpl::verifyEnvelope per envelope, in the order
      // the continuations posted them (HerderImpl.cpp:2414-2432)
      std::thread mainThr([&] {
        uint64_t h0, m0;
        PubKeyUtils::flushThreadVerifySigCounts(h0, m0);
        size_t doneN = 0, head = 0;
        std::vector<size_t> local;
        while (doneN < n) {
          {
            std::unique_lock<std::mutex> lk(qm);
            while (q.size() <= head) {
              mainWaiting = true;
              qcv.wait(lk);
            }
            mainWaiting = false;
            local.assign(q.begin() + (ptrdiff_t)head, q.end());
            head = q.size();
          }
          for (size_t i : local) {
            PublicKey k;
            std::memcpy(k.ed25519().data(), pk + 32 * i, 32);
            Signature s(sig + 64 * i, sig + 64 * i + 64);
            const auto a = Clk::now();
            const bool v = PubKeyUtils::verifySig(k, s, ByteSlice(msg + msg_off[i], msg_len[i]));
            const auto b = Clk::now();
            tMain[i] = b;
            mainCallUs.push_back(std::chrono::duration<double, std::micro>(b - a).count());
            out[i] = v ? 1 : 0;
            if ((uint8_t)v != cbVerdict[i]) ++mismatches;
            ++doneN;
          }
        }
        PubKeyUtils::flushThreadVerifySigCounts(hits, misses);
      });
      std::vector<std::thread> th;
      for (unsigned p = 0; p < P; ++p) {
        th.emplace_back([&, p] {
          PublicKey k;
          for (size_t b0 = 0, burst = 0; b0 < n; b0 += B, ++burst) {
            if (prm->interval_us) std::this_thread::sleep_until(T0 + std::chrono::microseconds((uint64_t)prm->interval_us * burst));
            const size_t b1 = std::min(n, b0 + B);
            for (size_t i = b0 + p; i < b1; i += P) {
              std::memcpy(k.ed25519().data(), pk + 32 * i, 32);
              tSub[i] = Clk::now();
              if (batchPost) {
                mb.submitTagged(k, ByteSlice(sig + 64 * i, 64), ByteSlice(msg + msg_off[i], msg_len[i]), i);
                continue;
              }
              mb.submit(k, ByteSlice(sig + 64 * i, 64), ByteSlice(msg + msg_off[i], msg_len[i]), [&, i](bool v) {
                tVer[i] = Clk::now();
                cbVerdict[i] = v ? 1 : 0;
                bool wake;
                {
                  std::lock_guard<std::mutex> g(qm);
                  q.push_back(i);
                  wake = mainWaiting;
                }
                if (wake) qcv.notify_one();
              });
            }
          }
        });
      }
      for (auto& t : th) t.join();
      mainThr.join();
      mb.drain();
      st = mb.stats();
      std::vector<double> ready = mb.latencies();
      std::sort(ready.begin(), ready.end());
      if (!ready.empty()) {
        res->ready_p50_us = ready[ready.size() / 2];
        res->ready_p99_us = ready[std::min(ready.size() - 1, (size_t)(0.99 * (double)ready.size()))];
      }
    }
    auto eng = PubKeyUtils::flushEngineCounts();
    std::vector<double> lv(n), lm(n);
    Clk::time_point first = tSub[0], last = tMain[0];
    for (size_t i = 0; i < n; ++i) {
      lv[i] = std::chrono::duration<double, std::micro>(tVer[i] - tSub[i]).count();
      lm[i] = std::chrono::duration<double, std::micro>(tMain[i] - tSub[i]).count();
      first = std::min(first, tSub[i]);
      last = std::max(last, tMain[i]);
    }
    auto pct = [](std::vector<double> v, double q) {
      std::sort(v.begin(), v.end());
      return v[std::min(v.size() - 1, (size_t)(q * (double)v.size()))];
    };
    double mean = 0;
    for (double x : lv) mean += x;
    res->verdict_p50_us = pct(lv, 0.5);
    res->verdict_p90_us = pct(lv, 0.9);
    res->verdict_p99_us = pct(lv, 0.99);
    res->verdict_max_us = pct(lv, 1.0);
    res->verdict_mean_us = mean / (double)n;
    res->main_p50_us = pct(lm, 0.5);
    res->main_p99_us = pct(lm, 0.99);
    res->main_call_p50_us = pct(mainCallUs, 0.5);
    double busy = 0;
    for (double x : mainCallUs) busy += x;
    res->main_busy_s = busy * 1e-6;
    res->main_call_mean_us = mainCallUs.empty() ? 0 : busy / (double)mainCallUs.size();
    res->main_hits = hits;
    res->main_misses = misses;
    res->main_mismatches = mismatches;
    res->batches = st.batches;
    res->flushed_by_size = st.flushedBySize;
    res->flushed_by_deadline = st.flushedByDeadline;
    res->flushed_idle = st.flushedIdle;
    res->max_batch = st.maxBatchSeen;
    res->burst_waits = st.burstWaits;
    res->mean_batch = st.batches ? (double)st.items / (double)st.batches : 0;
    res->gpu_batches = eng.gpuBatches;
    res->gpu_signatures = eng.gpuSignatures;
    res->cpu_signatures = eng.cpuSignatures;
    res->fallbacks = eng.fallbacks;
    res->wall_s = std::chrono::duration<double>(last - first).count();
    if (verdict) std::memcpy(verdict, out.data(), n);
    return SVH_OK;
  } catch (std::exception const& e) {
    return guard_exc(e);
  }
}

int svh_mb_run_workers(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                       const uint32_t* msg_len, size_t n, int producers, int workers, uint32_t max_batch,
                       uint32_t max_delay_us, uint32_t inter_arrival_us, uint8_t* verdict, svh_mb_stats* stats) {
  return svh_mb_run_ex(pk, sig, msg, msg_off, msg_len, n, producers, workers, max_batch, max_delay_us,
                       inter_arrival_us, 0, verdict, stats);
}

int svh_mb_run(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
               const uint32_t* msg_len, size_t n, int producers, uint32_t max_batch, uint32_t max_delay_us,
               uint32_t inter_arrival_us, uint8_t* verdict, svh_mb_stats* stats) {
  return svh_mb_run_ex(pk, sig, msg, msg_off, msg_len, n, producers, 2, max_batch, max_delay_us, inter_arrival_us, 0,
                       verdict, stats);
}

}  // extern "C"
