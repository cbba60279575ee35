/*
 * stellar_sigverify.h — C-ABI of the MI355X (gfx950) batched ed25519
 * signature-verification engine for stellar-core.
 *
 * Drop-in boundary.  stellar-core verifies every ed25519 signature through one
 * synchronous function:
 *
 *   bool stellar::PubKeyUtils::verifySig(PublicKey const&, Signature const&,
 *                                        ByteSlice const&)
 *     declared  /root/reference/src/crypto/SecretKey.h:139-140
 *     defined   /root/reference/src/crypto/SecretKey.cpp:435-468
 *
 * which, on a verify-cache miss, calls libsodium
 *   crypto_sign_verify_detached(sig, msg, msg_len, pk)   (SecretKey.cpp:461-463)
 *
 * The entry points below replace that libsodium call for WHOLE BATCHES of
 * cache misses.  Verdicts are bit-identical to libsodium 1.0.18
 * crypto_sign_verify_detached (cofactorless, S < L, small-order R/A and
 * non-canonical A rejected) on every input.  The size-64 rule of
 * SecretKey.cpp:441-444 is the caller's job (a Signature is an XDR opaque<64>;
 * anything shorter never reaches this API), as is the verify cache
 * (SecretKey.cpp:446-457,464-466) — see the C++ host mirror
 * stellar-core_amd/csrc/host/PubKeyUtils.{h,cpp}.
 *
 * Conventions: plain pointers and sizes, caller-owned memory, no exceptions
 * cross the boundary, every call returns SV_OK (0) or a negative SV_ERR_*.
 * An error is NEVER a reject: on error the verdict buffer content is
 * unspecified and the caller must treat the whole batch as unverified.
 * All entry points are thread-safe; calls that target one device are
 * serialised on that device's internal stream (its per-lane table workspace).
 */
#ifndef STELLAR_SIGVERIFY_H
#define STELLAR_SIGVERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SV_OK 0
#define SV_ERR_INVALID_ARG (-1)
#define SV_ERR_NO_DEVICE (-2)
#define SV_ERR_HIP (-3)
#define SV_ERR_ALLOC (-4)
#define SV_ERR_NOT_INIT (-5)
#define SV_ERR_ALIGN (-6)
/* A kernel reported that it could not stand behind its verdicts (the
 * three-wave cold-key octet kernel when one of its bounded LDS hand-over waits
 * ran out).  Like every error: the verdict buffer is unspecified and the batch
 * must be re-verified (the C++ mirror re-runs it on the CPU path), never
 * cached as rejects. */
#define SV_ERR_KERNEL (-7)

/* Batch options.  A NULL opts pointer means "all defaults". */
typedef struct sv_opts {
  uint32_t struct_size; /* sizeof(sv_opts), for forward compatibility */
  int32_t device;       /* -1 (default): contiguous slices over the device slots, every slice at least the
                           minimum shard (sv_set_min_shard; smaller batches run on one slot); k >= 0: slot k only */
  uint32_t max_devices; /* 0 (default): no limit; else use at most this many slots when device == -1 */
  uint32_t flags;       /* 0 or one SV_FLAG_PATH_* (kernel path for this call); other bits must be 0 */
} sv_opts;

/* Kernel paths.  THROUGHPUT: one lane per signature, prep + main kernels per
 * 2^20-signature chunk (large batches).  LATENCY: one quad of lanes per
 * signature, every point operation split four ways (small, latency-bound
 * batches such as SCP envelope floods).  AUTO picks LATENCY for batches of at
 * most 12288 signatures (the sizes it runs in one pass over the GPU).
 * Verdicts are identical on every path. */
#define SV_PATH_AUTO 0
#define SV_PATH_THROUGHPUT 1
#define SV_PATH_LATENCY 2
#define SV_FLAG_PATH_THROUGHPUT 0x1u
#define SV_FLAG_PATH_LATENCY 0x2u
#define SV_FLAG_PATH_MASK 0x3u

/* Process-wide default path for calls that do not request one (the device
 * API never does).  Returns the previous default, or SV_ERR_INVALID_ARG. */
int sv_set_kernel_path(int path);

/* Enumerate the device slots (one per visible GPU unless a device map says
 * otherwise).  Idempotent; called implicitly by every entry point.  Per-slot
 * resources (streams, base-point tables, workspace, pinned staging) are
 * created on the slot's first use; the throughput-path workspace is sized to
 * the batch and grows on demand. */
int sv_init(void);
/* Device slots -> physical GPUs, e.g. {0, 0}: two logical slots on GPU 0
 * (tests of the multi-device path on one GPU).  Releases every slot's
 * resources first; count == 0 restores one slot per visible GPU.  The
 * environment variable SV_DEVICE_MAP="0,0" sets the same at first init. */
int sv_set_device_map(const int* physical, int count);
/* Minimum signatures per slot when a batch is sharded (default 65536). */
int sv_set_min_shard(size_t n);
/* Release all device resources.  Safe to call more than once. */
void sv_shutdown(void);
/* Number of usable devices (initialises on first use); negative on error. */
int sv_device_count(void);
/* Thread-local description of the last error on the calling thread. */
const char* sv_last_error_string(void);
const char* sv_version(void);

/*
 * Variable-length batch, host buffers (replaces n calls of
 * crypto_sign_verify_detached made by PubKeyUtils::verifySig, SecretKey.cpp:461-463).
 *   pk       n x 32 bytes   (PublicKey ed25519, uint256)
 *   sig      n x 64 bytes   (R || S)
 *   msg      message bytes; message i = msg[msg_off[i] .. msg_off[i] + msg_len[i])
 *   verdict  n bytes out, 1 = valid, 0 = invalid
 */
int sv_ed25519_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                            const uint64_t* msg_off, const uint32_t* msg_len, size_t n,
                            uint8_t* verdict, const sv_opts* opts);

/*
 * Gather form of sv_ed25519_verify_batch: item i is (pk[i] -> 32 bytes,
 * sig[i] -> 64 bytes, msg[i] -> msg_len[i] bytes), packed by the engine
 * straight into its pinned staging (no intermediate copy by the caller, e.g.
 * PubKeyUtils::verifySigBatch over VerifyItem pointers).  keys (optional, n x
 * 32) also receives each item's verify-cache key BLAKE2b-256(pk || sig ||
 * msg) from the same staging (SecretKey.cpp:50-61).
 */
int sv_ed25519_verify_batch_gather(const uint8_t* const* pk, const uint8_t* const* sig, const uint8_t* const* msg,
                                   const uint32_t* msg_len, size_t n, uint8_t* verdict, uint8_t* keys,
                                   const sv_opts* opts);

/*
 * Same, with a callback for overlapping the caller's work with the GPU:
 * keys_ready(ctx) is called exactly once on success, on the calling thread,
 * as soon as every key is in `keys` -- for a batch that fits one staging chunk
 * on one slot, while the verify kernels are still running -- and the call
 * returns once the verdicts are in `verdict`.  keys_ready must not call into
 * this library.  On an error return keys_ready may or may not have run.
 */
int sv_ed25519_verify_batch_gather_cb(const uint8_t* const* pk, const uint8_t* const* sig,
                                      const uint8_t* const* msg, const uint32_t* msg_len, size_t n, uint8_t* verdict,
                                      uint8_t* keys, void (*keys_ready)(void* ctx), void* ctx, const sv_opts* opts);

/*
 * As sv_ed25519_verify_batch_gather_cb, with the keys delivered in pieces:
 * keys_ready(ctx, ready) runs with keys [0, ready) in `keys`, for increasing
 * `ready`, the last time with ready == n.  For a one-chunk batch of >= 8192
 * signatures the engine packs, copies up and hashes the batch in pieces: the
 * first of 2048 rows, each later one twice the one before, at most 32768 rows,
 * and no runt last piece (a remainder under 1.5 pieces joins the one before;
 * a 100k batch is 6 pieces).  So a caller that walks its cache in item order
 * (verifySigBatch, /root/reference/src/crypto/SecretKey.cpp:446-466 per item)
 * starts on the first rows while the rest is still on its way.  Same threading
 * rules.
 */
int sv_ed25519_verify_batch_gather_progress(const uint8_t* const* pk, const uint8_t* const* sig,
                                            const uint8_t* const* msg, const uint32_t* msg_len, size_t n,
                                            uint8_t* verdict, uint8_t* keys,
                                            void (*keys_ready)(void* ctx, size_t ready), void* ctx,
                                            const sv_opts* opts);

/*
 * CPU path: the engine's own per-signature algorithm (csrc/verify_core.h,
 * the half-size equation of csrc/lattice.h) compiled for the host, on
 * `threads` threads (0: the machine's hardware concurrency, capped at 16).
 * Same verdicts as every GPU path.  It is what a caller runs when a GPU entry
 * point returns an error (an error is never a reject) and what the C++ mirror
 * uses for single-signature verifySig calls, where a GPU round trip costs more
 * than the verification itself.  Message layout as in sv_ed25519_verify_batch.
 */
int sv_ed25519_verify_batch_cpu(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                                const uint32_t* msg_len, size_t n, uint8_t* verdict, int threads);
/* single-signature form (returns 1 valid, 0 invalid) */
int sv_ed25519_verify_cpu(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, size_t msg_len);

/*
 * Fixed-length batch, host buffers: message i = msg[i*msg_len .. (i+1)*msg_len).
 * msg_len == 32 (transaction contents hashes, TransactionFrame.cpp:90-117)
 * takes the single-SHA-512-block fast path.
 */
int sv_ed25519_verify_batch_fixed(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                                  uint32_t msg_len, size_t n, uint8_t* verdict, const sv_opts* opts);

/*
 * Device-resident batch on one device: every pointer is device memory on
 * `device` (16-byte aligned pk/sig; for fixed_msg_len == 32 also msg).
 * If fixed_msg_len != 0, message i = d_msg[i*fixed_msg_len ..] and
 * d_msg_off/d_msg_len are ignored (may be NULL).  d_bitmap (optional, may be
 * NULL) receives one bit per signature, 64 per word, bit (i % 64) of word
 * i / 64 (wave-level ballot compaction of the verdicts); it must hold
 * ceil(n / 64) words, and the bits past n in the last word are written 0.
 * `stream` is a hipStream_t (NULL = legacy default stream): the work is
 * ordered after prior work on `stream` and later work on `stream` is ordered
 * after it; the call itself does not block.
 */
int sv_ed25519_verify_device(int device, const void* d_pk, const void* d_sig, const void* d_msg,
                             const uint64_t* d_msg_off, const uint32_t* d_msg_len,
                             uint32_t fixed_msg_len, size_t n, void* d_verdict, void* d_bitmap,
                             void* stream);

/*
 * Synthetic-workload generator (device-resident): for i in [0, n) derive the
 * keypair from seed i (RFC 8032, == crypto_sign_seed_keypair) and sign the
 * 32-byte message i (== crypto_sign_detached).  Used by the bench to build
 * the 1M..64M-signature datasets on the GPU box; its output is checked
 * against libsodium-generated digests (tests/golden/digests.json).
 */
int sv_ed25519_sign_device(int device, const void* d_seed, const void* d_msg32, size_t n, void* d_pk,
                           void* d_sig, void* stream);

/* ---- Batch hashing on the device ----------------------
 * Verify-cache keys: keys[32*i..] = BLAKE2b-256(pk_i || sig_i || msg_i), the key
 * PubKeyUtils::verifySig computes per call before consulting the cache
 * (/root/reference/src/crypto/SecretKey.cpp:50-61, verifySigCacheKey).
 * Message layout as in sv_ed25519_verify_batch. */
int sv_verify_cache_keys(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                         const uint32_t* msg_len, size_t n, uint8_t* keys /* n x 32 */, const sv_opts* opts);

/* Verdicts AND cache keys from one staging of the batch (one H2D, two kernels
 * on one stream, one sync): the verifySigBatch miss path without any
 * per-signature host hashing. */
int sv_ed25519_verify_batch_keyed(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                                  const uint64_t* msg_off, const uint32_t* msg_len, size_t n, uint8_t* verdict,
                                  uint8_t* keys /* n x 32 */, const sv_opts* opts);

/* SHA-256 of n byte strings (data + off[i], len[i]): digests[32*i..].  Batch
 * form of the transaction contents hash, sha256(xdr(networkID, ENVELOPE_TYPE_TX,
 * tx)) at /root/reference/src/transactions/TransactionFrame.cpp:90-117. */
int sv_sha256_batch(const uint8_t* data, const uint64_t* off, const uint32_t* len, size_t n,
                    uint8_t* digests /* n x 32 */, const sv_opts* opts);

/* Device-resident forms (stream semantics as sv_ed25519_verify_device; pk, sig
 * and output buffers 4-byte aligned; fixed_len != 0 means item i's message is
 * d_msg + i * fixed_len and d_off / d_len are ignored). */
int sv_verify_cache_keys_device(int device, const void* d_pk, const void* d_sig, const void* d_msg,
                                const uint64_t* d_msg_off, const uint32_t* d_msg_len, uint32_t fixed_msg_len,
                                size_t n, void* d_keys, void* stream);
int sv_sha256_device(int device, const void* d_data, const uint64_t* d_off, const uint32_t* d_len,
                     uint32_t fixed_len, size_t n, void* d_digests, void* stream);

/* ---- Warm-key latency path (csrc/comb.h, csrc/sv_comb.hip) ---------------
 * Each device slot keeps a bounded cache of per-public-key tables
 * ({0..8} * 16^j * (-A), 108 KiB per key) in HBM.  A latency-path host batch
 * whose keys are all cached runs the comb kernel: libsodium's equation
 * [S]B + [h](-A) == R evaluated as a sum of 96 table entries, no scalar
 * multiplication.  Any other batch runs the octet kernel, after which its
 * keys (on their second sighting) are built on a low-priority stream for the
 * next batch.  Verdicts are identical on both kernels; the cache holds only
 * data derived from public keys.  Default capacity 1024 keys (or the
 * SV_KEY_CACHE environment variable); 0 disables the warm path.  Drains and
 * clears every slot's cache. */
int sv_set_key_cache(size_t capacity);
/* Blocks until every key-table build queued on `device` has finished. */
int sv_key_cache_wait(int device);
typedef struct sv_key_cache_stats {
  uint64_t capacity;     /* keys the cache holds at most */
  uint64_t keys;         /* keys cached or being built */
  uint64_t warm_batches; /* latency-lane batches served by the comb kernel */
  uint64_t cold_batches; /* latency-lane batches served by the octet kernel */
  uint64_t keys_built;   /* key-table builds queued */
  uint64_t evictions;
  uint64_t shared_launches; /* bulk (throughput-path) launches that ran in shared
                               mode because latency batches were live: they leave
                               one workgroup slot per CU to the latency lane
                               (window SV_LAT_SHARE_MS, default 1000; 0: off) */
  uint64_t table_launches;  /* throughput-path launches that used the per-key tables */
  uint64_t table_keys;      /* keys claimed in them since the tables were last cleared
                               (as of the last launch whose counters came back) */
  uint64_t table_clears;    /* times the claim words were cleared (claims reached half the slots) */
  uint64_t table_slots;     /* slots of the per-key tables */
} sv_key_cache_stats;
int sv_key_cache_get_stats(int device, sv_key_cache_stats* out);

/* Host-side stages of the calling thread's last latency-lane batch (a batch of
 * at most one staging chunk on one slot), in microseconds: out[0] plan + pack,
 * [1] the H2D call (0 while the kernels read the image in place), [2] the kernel launch, [3] the D2H / event record calls,
 * [4] key-table build queueing, [5] the wait for the device (H2D + kernel +
 * verdicts), [6] the whole batch inside the engine, [7] 1 if it ran the
 * warm-key comb kernel, 0 the octet kernel.  Zeros before the first batch.
 * For tail-latency diagnosis (bench.py latency_1k.slow_iterations). */
int sv_lat_last_trace(double out[8]);

/* Per-key tables of the throughput path (replaces, for repeated signers, the
 * per-signature decode of A that libsodium's verify does,
 * /root/reference/src/crypto/SecretKey.cpp:461-463 per call; catchup replays
 * ~16 signatures per account, LedgerManagerImpl.cpp:1546-1609): each key's
 * decoded -A and its 9-entry table are built once on the device and reused
 * by every later signature of that key.  mode 0: off; 1: every throughput-
 * path launch; 2 (default): host-buffer batches whose keys repeat (a sampled
 * estimate; device-resident batches only with 1); -1: the SV_KEY_TABLES
 * environment variable.  slots: table size (0: SV_KEY_TABLE_SLOTS or 2^19,
 * ~1.5 KB of HBM each; claims stop at half, then the tables are cleared).
 * Verdicts never depend on the tables.  Returns the previous mode. */
int sv_set_key_tables(int mode, size_t slots);

/* Test knobs (0 in production).  TRIVIAL_PAIR: every lane verifies through the
 * fallback pair (h, 1) of the half-size equation (lattice.h), i.e. the
 * full-length scalar; MAX_WINDOWS: every wave runs all 64 windows (both only
 * select code paths; verdicts are unchanged).  FAIL: every GPU entry point
 * returns SV_ERR_HIP without touching the device (callers' CPU fallback
 * tests); PREP_ONLY (profiling): throughput-path launches run the
 * per-signature prep kernel only (verdicts are NOT written).  FAIL and
 * PREP_ONLY are refused (SV_ERR_INVALID_ARG) unless the process environment
 * has SV_TEST_KNOBS=1.  Returns the previous flags, or SV_ERR_INVALID_ARG. */
#define SV_DBG_TRIVIAL_PAIR 0x1u
#define SV_DBG_MAX_WINDOWS 0x2u
#define SV_DBG_FAIL 0x4u
#define SV_DBG_PREP_ONLY 0x8u
#define SV_DBG_KEY_COLLIDE 0x10u /* every key gets the same per-key-table fingerprint (collision path) */
/* throughput-path geometry: QUAD runs every throughput-path launch one signature
 * per quad of lanes (the medium-batch kernel), NO_QUAD none (one per lane);
 * by default launches of at most SV_QUAD_MAX signatures (env; default in
 * DESIGN.md) that use no per-key tables take the quad geometry.  Code paths
 * only: verdicts are unchanged. */
#define SV_DBG_QUAD 0x20u
#define SV_DBG_NO_QUAD 0x40u
/* DROP_HANDOVER (needs SV_TEST_KNOBS=1): the three-wave cold-key octet kernel
 * never raises its tables' hand-over flag, so its verify wave's bounded wait
 * (~0.5 s) runs out: the kernel writes fail-closed rejects and raises its
 * failure word, and the call returns SV_ERR_KERNEL (the error path of a lost
 * hand-over). */
#define SV_DBG_DROP_HANDOVER 0x80u
int sv_set_debug_flags(uint32_t flags);

/* Host-feed probe (multi-GPU sizing).  Runs the host
 * side of sv_ed25519_verify_batch_fixed(device = -1, max_devices) over n
 * signatures -- the contiguous slices, each slot's own staging workers
 * (pinned to the GPU's NUMA node), the pack into the slot's two pinned
 * staging slots and, with upload != 0, the H2D copies -- and launches no
 * kernel: no verdicts.  What the G slots' host side can feed, against the
 * rate G GPUs verify at. */
typedef struct sv_feed_stats {
  uint32_t struct_size;      /* sizeof(sv_feed_stats) */
  uint32_t slots;            /* slots the batch was sliced over */
  uint32_t threads_per_slot; /* pack threads per slot (1 slot: the shared pool + caller) */
  uint32_t usable_cpus;      /* affinity limited by the cgroup CPU quota */
  double seconds;            /* wall time of the whole feed */
  int32_t gpu_numa[16];      /* NUMA node of slot g's GPU (-1: unknown) */
  int32_t staging_numa[16];  /* NUMA node of slot g's first pinned staging page (-1: unknown) */
  uint32_t pinned_cpus[16];  /* CPUs slot g's workers are pinned to (0: not pinned) */
} sv_feed_stats;
int sv_host_feed_probe(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t msg_len, size_t n,
                       uint32_t max_devices, int upload, sv_feed_stats* out);

/* Bytes of the slot's kernel workspace / pinned staging currently allocated. */
int sv_workspace_bytes(int device, size_t* bytes);
int sv_pinned_bytes(int device, size_t* bytes);

/* Kernel-time accounting for profiling: when enabled, every verify launch is
 * bracketed by HIP events on the device's internal stream and the elapsed
 * times are accumulated (read back with sv_kernel_time). */
int sv_timing_enable(int enable);
int sv_kernel_time(int device, double* total_ms, uint64_t* launches, uint64_t* signatures);
int sv_kernel_time_reset(void);
int sv_device_synchronize(int device);

#ifdef __cplusplus
}
#endif
#endif /* STELLAR_SIGVERIFY_H */
