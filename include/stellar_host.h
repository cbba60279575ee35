/*
 * stellar_host.h — C surface of libstellar_host.so, the C++ mirror of
 * stellar-core's verification callers re-targeted at the MI355X engine
 * (stellar-core_amd/csrc/host/).  C++ integrators use the C++ headers
 * (PubKeyUtils.h, SignatureChecker.h) directly; this surface exists for
 * bindings and tests.
 *
 *   svh_verify_sig          == PubKeyUtils::verifySig
 *                              (/root/reference/src/crypto/SecretKey.cpp:435-468)
 *   svh_verify_sig_batch    == PubKeyUtils::verifySigBatch (new)
 *   svh_cache_*             == clearVerifySigCache / maybeSeedVerifySigCache /
 *                              flushVerifySigCacheCounts (SecretKey.cpp:317-339)
 *   svh_check_txset         == SignatureChecker::checkSignature +
 *                              checkAllSignaturesUsed per tx
 *                              (/root/reference/src/transactions/SignatureChecker.cpp:30-158),
 *                              optionally after one GPU batch pre-pass over the
 *                              whole set
 *   svh_check_envelopes     == the signature checks of TransactionFrame::checkValid /
 *                              apply and FeeBumpTransactionFrame::checkValid over ONE
 *                              checker per envelope: source account at LOW, extra
 *                              signers, every operation at its threshold, all
 *                              signatures used (TransactionFrame.cpp:268-321,
 *                              1091-1156, 1185-1301, 1416-1486; OperationFrame.cpp:
 *                              173-209; FeeBumpTransactionFrame.cpp:138-197), optionally
 *                              after one batch pre-pass over every envelope (a tx set,
 *                              f1, or a whole catchup checkpoint, f3: verdicts in a
 *                              side table, the 0xffff cache bypassed)
 *   svh_mb_run              == VerifyMicroBatcher driven by `producers` threads: the
 *                              SCP/overlay pre-verify (/root/reference/src/overlay/
 *                              Peer.cpp:963-970) turned into size/deadline-flushed
 *                              GPU batches
 *
 * Nothing here reports an engine (GPU) error: the mirror re-runs a failed
 * batch on the engine's CPU path (sv_ed25519_verify_batch_cpu), like the
 * reference's verifySig, which never fails.  svh_engine_counts_ex reports how
 * often that happened.
 */
#ifndef STELLAR_HOST_H
#define STELLAR_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SVH_OK 0
#define SVH_ERR_INVALID_ARG (-1)
#define SVH_ERR_ENGINE (-2) /* (kept for ABI stability; engine errors are absorbed by the CPU path) */

typedef struct svh_signer {
  uint8_t type; /* 0 ED25519, 1 PRE_AUTH_TX, 2 HASH_X, 3 ED25519_SIGNED_PAYLOAD */
  uint8_t key[32];
  uint32_t weight;
  uint32_t payload_len; /* signed payload only, <= 64 */
  uint8_t payload[64];
} svh_signer;

typedef struct svh_decorated_sig {
  uint8_t hint[4];
  uint32_t sig_len; /* <= 64; != 64 never verifies */
  uint8_t sig[64];
} svh_decorated_sig;

typedef struct svh_tx {
  uint8_t contents_hash[32];
  uint32_t protocol;
  int32_t needed_weight;
  uint32_t nsigs, sig_off;       /* range in the svh_decorated_sig array */
  uint32_t nsigners, signer_off; /* range in the svh_signer array */
} svh_tx;

typedef int (*svh_batch_verify_fn)(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                                   const uint32_t* len, size_t n, uint8_t* verdict);

const char* svh_last_error_string(void);
void svh_blake2b256(uint8_t out[32], const uint8_t* p, size_t n);
void svh_sha256(uint8_t out[32], const uint8_t* p, size_t n);
/* 1 valid, 0 invalid, < 0 error */
int svh_verify_sig(const uint8_t pk[32], const uint8_t* sig, size_t sig_len, const uint8_t* msg, size_t msg_len);
int svh_verify_sig_batch(const uint8_t* pk, const uint8_t* sig /* n x 64 */, const uint32_t* sig_len /* NULL = 64 */,
                         const uint8_t* msg, const uint64_t* msg_off, const uint32_t* msg_len, size_t n,
                         uint8_t* verdict);
/* Verify-hit benchmark, the shape of the reference's "verify-hit benchmarking"
 * (/root/reference/src/crypto/test/CryptoTests.cpp:308-316 ->
 * SecretKey::benchmarkOpsPerSecond(.., 10000, 10), SecretKey.cpp:214-241):
 * n cases (pk n x 32, sig n x 64, messages n x msg_len), one untimed pass of
 * PubKeyUtils::verifySig over them (cache misses: verified and cached), then
 * passes - 1 timed passes, every call a cache hit, on `threads` threads each
 * walking all n cases from a different start (threads > 1: callers contending
 * for the cache's mutex).  *hits_per_s = timed calls / timed wall seconds over
 * all threads; *fill_s = the first pass's wall seconds.  Returns 0, or < 0 if
 * any call did not return 1 (the cases must be valid). */
int svh_bench_verify_hits(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, size_t msg_len, size_t n,
                          int passes, int threads, double* hits_per_s, double* fill_s);
void svh_cache_clear(void);
void svh_cache_seed(unsigned int seed);
void svh_cache_counts(uint64_t* hits, uint64_t* misses); /* flushes, like flushVerifySigCacheCounts */
/* the cache's keys in its insertion-order vector (the reference's mValuePtrs);
 * writes min(max_keys, size) keys of 32 bytes, returns the cache size */
size_t svh_cache_keys(uint8_t* out, size_t max_keys);
void svh_engine_counts(uint64_t* signatures, uint64_t* batches); /* GPU signatures / calls; flushes */
typedef struct svh_engine_stats {
  uint64_t gpu_signatures, gpu_batches, cpu_signatures, fallbacks;
} svh_engine_stats;
void svh_engine_counts_ex(svh_engine_stats* out); /* flushes all four */
/* Batch-size and latency histograms (PubKeyUtils::flushEngineHistograms):
 * out[0..31] GPU batch sizes, [32..63] GPU latencies (us), [64..95] CPU-path
 * batch sizes, [96..127] CPU-path latencies; bucket b counts values v with
 * floor(log2(v)) == b (v = 0 in bucket 0, the last bucket open-ended).
 * Flushes. */
void svh_engine_histograms(uint64_t out[128]);
/* batches with at most max_misses cache misses run on the CPU path (default 1) */
void svh_set_cpu_threshold(size_t max_misses);
/* engine-only batch, no cache (PubKeyUtils::verifyBatchUncached) */
int svh_verify_uncached(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                        const uint32_t* msg_len, size_t n, uint8_t* verdict);
/* test hook: route cache misses to fn instead of the GPU (NULL restores) */
void svh_set_test_verifier(svh_batch_verify_fn fn);
/* Keyed batches: verifySigBatch calls with >= min_items
 * eligible signatures get verdicts AND BLAKE2b cache keys from one engine pass
 * (sv_ed25519_verify_batch_gather with keys); 0 disables; default 256.  The
 * keyed test hook replaces that engine call (CPU tests). */
typedef int (*svh_keyed_verify_fn)(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                                   const uint32_t* len, size_t n, uint8_t* verdict, uint8_t* keys);
void svh_set_test_keyed_verifier(svh_keyed_verify_fn fn);
void svh_set_keyed_threshold(size_t min_items);
/* use_prefetch: 0 none; 1 one batch pre-pass into a side table (pairs
 * enumerated in parallel, each checker finds its tx's pairs by position); 2
 * the same through verifySigBatch (also seeds the verify cache); 3 as 1 with
 * the checkers looking their pairs up in the table only; 4 as 1 in two halves,
 * pipelined: the engine verifies half 0 while half 1 is enumerated and half 1
 * while half 0's checkers run (sets of at least 1024 transactions; smaller
 * ones run as 1).  Outcomes are the same in every mode. */
int svh_check_txset(const svh_tx* txs, size_t ntx, const svh_decorated_sig* sigs, const svh_signer* signers,
                    int use_prefetch, uint8_t* ok, uint8_t* all_used, uint64_t* prefetched_pairs);
/* Wall-clock phases (ms) of the calling thread's last svh_check_txset:
 * [0] C structs -> the mirror's objects, [1] pair enumeration (prefetch add),
 * [2] the engine pre-pass (prefetch run: one GPU batch + side table),
 * [3] the checkers.  [1] and [2] are 0 without the pre-pass.  Pipelined (use_prefetch 4): [1] half 0's
 * enumeration, [2] the overlapped middle (engine on half 0 beside half 1's enumeration, then engine on
 * half 1 beside half 0's checkers), [3] half 1's checkers. */
void svh_txset_last_phases(double out[4]);

/* ---- transaction-level checks (a13) ---- */
typedef struct svh_account {
  uint8_t account_id[32];
  uint8_t thresholds[4]; /* master weight, LOW, MEDIUM, HIGH */
  uint32_t nsigners, signer_off; /* range in the svh_signer array */
} svh_account;

typedef struct svh_op {
  uint8_t has_source; /* 0: the transaction's source account */
  uint8_t level;      /* 1 LOW, 2 MEDIUM, 3 HIGH */
  uint8_t source[32];
  uint8_t pad[2];
} svh_op;

typedef struct svh_envelope {
  uint8_t contents_hash[32]; /* of the (inner) transaction */
  uint8_t source[32];
  uint32_t nsigs, sig_off;   /* the transaction's signatures */
  uint32_t nops, op_off;
  uint32_t nextra, extra_off; /* extra signer keys (svh_signer, weight ignored) */
  uint32_t fee_bump;          /* 1: fee-bump envelope around the transaction */
  uint8_t fee_bump_hash[32];
  uint8_t fee_source[32];
  uint32_t nouter, outer_off; /* fee-bump (outer) signatures */
} svh_envelope;

typedef struct svh_tx_result {
  int32_t code;       /* TransactionResultCode: 0 txSUCCESS, 1 txFEE_BUMP_INNER_SUCCESS, -1 txFAILED,
                         -6 txBAD_AUTH, -8 txNO_ACCOUNT, -10 txBAD_AUTH_EXTRA, -12 txNOT_SUPPORTED,
                         -13 txFEE_BUMP_INNER_FAILED */
  int32_t inner_code; /* fee bump: the inner transaction's code */
  int32_t failed_op;  /* txFAILED: the first failing operation, else -1 */
  int32_t op_code;    /* 0 opINNER, -1 opBAD_AUTH, -2 opNO_ACCOUNT */
} svh_tx_result;

/* prefetch: 0 none, 1 side table (cache bypassed: the per-checkpoint catchup
 * form), 2 side table + verify cache.  for_apply: 0 checkValid path, 1 apply
 * path (processSignatures). */
int svh_check_envelopes(const svh_envelope* env, size_t n, const svh_decorated_sig* sigs, const svh_op* ops,
                        const svh_signer* signers, const svh_account* accounts, size_t naccounts,
                        uint32_t protocol, int prefetch, int for_apply, svh_tx_result* results,
                        uint64_t* prefetched_pairs);

typedef struct svh_mb_stats {
  uint64_t items, batches, flushed_by_size, flushed_by_deadline, max_batch;
  double lat_p50_us, lat_p99_us; /* submit -> verdict ready (submit mode) */
  double wall_s;                 /* first submission -> last verdict */
} svh_mb_stats;
/* Feed n signatures through a VerifyMicroBatcher (2 flush workers) from
 * `producers` threads (item i from thread i % producers, optional sleep
 * between submissions). */
int svh_mb_run(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
               const uint32_t* msg_len, size_t n, int producers, uint32_t max_batch, uint32_t max_delay_us,
               uint32_t inter_arrival_us, uint8_t* verdict, svh_mb_stats* stats);
/* Same with `workers` flush threads (VerifyMicroBatcher workers > 1: several
 * batches in flight, host work of one overlapping the engine call of another). */
/* fire_and_forget: producers post() (verdicts only warm the verify cache, as the
 * reference's pre-verify) instead of submit(); verdict[] is then read back
 * from the cache after the run */
int svh_mb_run_ex(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                  const uint32_t* msg_len, size_t n, int producers, int workers, uint32_t max_batch,
                  uint32_t max_delay_us, uint32_t inter_arrival_us, int fire_and_forget, uint8_t* verdict,
                  svh_mb_stats* stats);
int svh_mb_run_workers(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                       const uint32_t* msg_len, size_t n, int producers, int workers, uint32_t max_batch,
                       uint32_t max_delay_us, uint32_t inter_arrival_us, uint8_t* verdict, svh_mb_stats* stats);

/* Config 4 through the integration path (BASELINE config 4):
 * `producers` overlay threads submit the n envelopes (pk, sig, msg) in bursts
 * of `burst` (burst k starts interval_us * k after the run starts; interval_us
 * 0 = a flood, back to back) into ONE VerifyMicroBatcher with the continuation
 * form of submit(): each verdict's continuation posts the envelope to a "main
 * thread", which calls PubKeyUtils::verifySig on it as HerderImpl::
 * verifyEnvelope does (/root/reference/src/herder/HerderImpl.cpp:2414-2432)
 * -- the reference's order: the overlay thread's pre-verify (Peer.cpp:963-970)
 * completes before the message is posted to the main thread.
 * verdict[i]: the main thread's verifySig result.  policy 0 WhenIdle, 1
 * Deadline (VerifyMicroBatcher.h). */
typedef struct svh_scp_params {
  uint32_t struct_size; /* sizeof(svh_scp_params) */
  uint32_t producers, burst, interval_us;
  uint32_t max_batch, max_delay_us, workers;
  uint32_t policy, linger_us, idle_in_flight;
  uint32_t quiet_us, max_linger_us; /* WhenIdle burst wait (VerifyMicroBatcher::Options; quiet 0: off) */
  /* 1: the overlay posts one main-thread task per verified batch (submitTagged + Options::onBatch) instead of
   * one per envelope; older callers whose struct_size ends before this field get 0 */
  uint32_t batch_post;
} svh_scp_params;
typedef struct svh_scp_result {
  double verdict_p50_us, verdict_p90_us, verdict_p99_us, verdict_max_us, verdict_mean_us; /* submit -> continuation */
  double main_p50_us, main_p99_us;   /* submit -> the main thread's verifySig returned */
  double main_call_p50_us;           /* one verifySig call on the main thread */
  uint64_t main_hits, main_misses, main_mismatches; /* main-thread verifySig: cache hits / misses / != continuation */
  uint64_t batches, flushed_by_size, flushed_by_deadline, flushed_idle, max_batch;
  double mean_batch;
  uint64_t gpu_batches, gpu_signatures, cpu_signatures, fallbacks; /* engine counts over the run */
  double wall_s; /* first submission -> last main-thread verifySig */
  double ready_p50_us, ready_p99_us; /* submit -> the item's batch verified and cached (before its continuations) */
  uint64_t burst_waits;              /* idle flushes that first waited for a burst to end */
  double main_busy_s;                /* the main thread's time inside verifySig: n / main_busy_s is its ceiling */
  double main_call_mean_us;          /* mean of one main-thread verifySig call */
} svh_scp_result;
int svh_scp_run(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                const uint32_t* msg_len, size_t n, const svh_scp_params* params, uint8_t* verdict,
                svh_scp_result* result);

#ifdef __cplusplus
}
#endif
#endif /* STELLAR_HOST_H */
