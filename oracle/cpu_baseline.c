/*
 * CPU BASELINE HARNESS — test/bench infrastructure only (bench.py's
 * cpu_baseline leg).  Never part of the product path.
 *
 * Times the CPU path stellar-core uses today: libsodium
 * crypto_sign_verify_detached, the call PubKeyUtils::verifySig makes on a cache
 * miss (/root/reference/src/crypto/SecretKey.cpp:461-463), over n fixed-length
 * messages on `threads` pthreads with a static contiguous partition (SURVEY.md
 * §8 d8).  libsodium is dlopen'd from `sodium_path`; with sodium_path == NULL
 * the oracle restatement (ed25519_oracle.c) is timed instead ("port").
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <time.h>

#include "oracle.h"

typedef int (*verify_fn)(const unsigned char*, const unsigned char*, unsigned long long, const unsigned char*);

struct job {
  verify_fn sodium;
  const uint8_t *pk, *sig, *msg;
  uint32_t mlen;
  size_t lo, hi;
  uint8_t* out;
};

static void* worker(void* arg) {
  struct job* j = (struct job*)arg;
  for (size_t i = j->lo; i < j->hi; ++i) {
    int rc = j->sodium ? j->sodium(j->sig + 64 * i, j->msg + (size_t)j->mlen * i, j->mlen, j->pk + 32 * i)
                       : oracle_ed25519_verify(j->sig + 64 * i, j->msg + (size_t)j->mlen * i, j->mlen, j->pk + 32 * i);
    j->out[i] = rc == 0;
  }
  return 0;
}

/* Returns wall seconds (< 0 on error: -1 dlopen, -2 dlsym/init, -3 threads). */
double cpubase_run(const char* sodium_path, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t mlen,
                   size_t n, int threads, uint8_t* out) {
  verify_fn f = 0;
  if (sodium_path) {
    void* h = dlopen(sodium_path, RTLD_NOW | RTLD_LOCAL);
    if (!h) return -1.0;
    int (*init)(void) = (int (*)(void))dlsym(h, "sodium_init");
    f = (verify_fn)dlsym(h, "crypto_sign_verify_detached");
    if (!init || !f || init() < 0) return -2.0;
  }
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  struct job jobs[256];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; ++t) {
    jobs[t].sodium = f;
    jobs[t].pk = pk; jobs[t].sig = sig; jobs[t].msg = msg; jobs[t].mlen = mlen;
    jobs[t].lo = (size_t)t * n / threads;
    jobs[t].hi = (size_t)(t + 1) * n / threads;
    jobs[t].out = out;
    if (pthread_create(&th[t], 0, worker, &jobs[t]) != 0) return -3.0;
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], 0);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* libsodium-backed batch verifier with the svh_batch_verify_fn signature
 * (include/stellar_host.h), so the C++ SignatureChecker mirror can be timed
 * on the reference's own CPU path (one libsodium call per signature, on
 * `g_threads` threads).  Set up with cpubase_set_sodium(path, threads). */
static verify_fn g_sodium_fn = 0;
static int g_threads = 1;

int cpubase_set_sodium(const char* sodium_path, int threads) {
  void* h = dlopen(sodium_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return -1;
  int (*init)(void) = (int (*)(void))dlsym(h, "sodium_init");
  g_sodium_fn = (verify_fn)dlsym(h, "crypto_sign_verify_detached");
  if (!init || !g_sodium_fn || init() < 0) return -2;
  g_threads = threads < 1 ? 1 : (threads > 256 ? 256 : threads);
  return 0;
}

struct vjob {
  const uint8_t *pk, *sig, *msg;
  const uint64_t* off;
  const uint32_t* len;
  size_t lo, hi;
  uint8_t* out;
};

static void* vworker(void* arg) {
  struct vjob* j = (struct vjob*)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->out[i] = g_sodium_fn(j->sig + 64 * i, j->msg + j->off[i], j->len[i], j->pk + 32 * i) == 0;
  return 0;
}

int cpubase_sodium_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                         const uint32_t* len, size_t n, uint8_t* verdict) {
  if (!g_sodium_fn) return -1;
  int T = g_threads;
  if ((size_t)T > n) T = n ? (int)n : 1;
  if (T == 1) {  /* inline: a per-call thread would dominate single-signature calls */
    struct vjob j = {pk, sig, msg, off, len, 0, n, verdict};
    vworker(&j);
    return 0;
  }
  pthread_t th[256];
  struct vjob jobs[256];
  for (int t = 0; t < T; ++t) {
    jobs[t].pk = pk; jobs[t].sig = sig; jobs[t].msg = msg; jobs[t].off = off; jobs[t].len = len;
    jobs[t].lo = (size_t)t * n / T;
    jobs[t].hi = (size_t)(t + 1) * n / T;
    jobs[t].out = verdict;
    if (pthread_create(&th[t], 0, vworker, &jobs[t]) != 0) return -3;
  }
  for (int t = 0; t < T; ++t) pthread_join(th[t], 0);
  return 0;
}

/* The reference's verifySig on every core: `threads` pthreads, each calling
 * `verify_sig` (the C++ PubKeyUtils::verifySig mirror, svh_verify_sig:
 * BLAKE2b cache key, global cache under its mutex, then the batch verifier --
 * set to cpubase_sodium_batch with one thread, i.e. one libsodium call per
 * miss, as SecretKey.cpp:435-468 does) for its contiguous slice.  Returns
 * wall seconds (< 0 on error). */
typedef int (*verifysig_fn)(const uint8_t*, const uint8_t*, size_t, const uint8_t*, size_t);
struct sjob {
  verifysig_fn f;
  const uint8_t *pk, *sig, *msg;
  const uint64_t* off;
  const uint32_t* len;
  size_t lo, hi;
  uint8_t* out;
};

static void* sworker(void* arg) {
  struct sjob* j = (struct sjob*)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->out[i] = j->f(j->pk + 32 * i, j->sig + 64 * i, 64, j->msg + j->off[i], j->len[i]) == 1;
  return 0;
}

double cpubase_verifysig_threads(verifysig_fn f, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                                 const uint64_t* off, const uint32_t* len, size_t n, int threads, uint8_t* out) {
  if (!f) return -2.0;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  struct sjob jobs[256];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; ++t) {
    struct sjob j = {f, pk, sig, msg, off, len, (size_t)t * n / threads, (size_t)(t + 1) * n / threads, out};
    jobs[t] = j;
    if (pthread_create(&th[t], 0, sworker, &jobs[t]) != 0) return -3.0;
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], 0);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
