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
 *   svh_mb_run              == VerifyMicroBatcher driven by `producers` threads: the
 *                              SCP/overlay pre-verify (/root/reference/src/overlay/
 *                              Peer.cpp:963-970) turned into size/deadline-flushed
 *                              GPU batches
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
#define SVH_ERR_ENGINE (-2) /* device error: the batch is unverified, never rejected */

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
void svh_cache_clear(void);
void svh_cache_seed(unsigned int seed);
void svh_cache_counts(uint64_t* hits, uint64_t* misses); /* flushes, like flushVerifySigCacheCounts */
void svh_engine_counts(uint64_t* signatures, uint64_t* batches);
/* test hook: route cache misses to fn instead of the GPU (NULL restores) */
void svh_set_test_verifier(svh_batch_verify_fn fn);
/* Keyed batches: verifySigBatch calls with >= min_items
 * eligible signatures get verdicts AND BLAKE2b cache keys from one engine pass
 * (sv_ed25519_verify_batch_keyed); 0 disables; default 4096.  The keyed test
 * hook replaces that engine call (CPU tests). */
typedef int (*svh_keyed_verify_fn)(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                                   const uint32_t* len, size_t n, uint8_t* verdict, uint8_t* keys);
void svh_set_test_keyed_verifier(svh_keyed_verify_fn fn);
void svh_set_keyed_threshold(size_t min_items);
int svh_check_txset(const svh_tx* txs, size_t ntx, const svh_decorated_sig* sigs, const svh_signer* signers,
                    int use_prefetch, uint8_t* ok, uint8_t* all_used, uint64_t* prefetched_pairs);

typedef struct svh_mb_stats {
  uint64_t items, batches, flushed_by_size, flushed_by_deadline, max_batch;
  double lat_p50_us, lat_p99_us; /* submit -> verdict ready */
} svh_mb_stats;
/* Feed n signatures through a VerifyMicroBatcher (2 flush workers) from
 * `producers` threads (item i from thread i % producers, optional sleep
 * between submissions). */
int svh_mb_run(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
               const uint32_t* msg_len, size_t n, int producers, uint32_t max_batch, uint32_t max_delay_us,
               uint32_t inter_arrival_us, uint8_t* verdict, svh_mb_stats* stats);
/* Same with `workers` flush threads (VerifyMicroBatcher workers > 1: several
 * batches in flight, host work of one overlapping the engine call of another). */
int svh_mb_run_workers(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                       const uint32_t* msg_len, size_t n, int producers, int workers, uint32_t max_batch,
                       uint32_t max_delay_us, uint32_t inter_arrival_us, uint8_t* verdict, svh_mb_stats* stats);

#ifdef __cplusplus
}
#endif
#endif /* STELLAR_HOST_H */
