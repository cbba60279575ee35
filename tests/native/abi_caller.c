/* TEST INFRASTRUCTURE (tests/test_callers.py): a plain C99 caller of the
 * engine's C-ABI (include/stellar_sigverify.h), written the way a maintainer
 * binds it in place of the loop of crypto_sign_verify_detached calls at
 * /root/reference/src/crypto/SecretKey.cpp:461-463.
 *
 * It checks that the header compiles as C, that the entry points link from C,
 * and the contract a caller relies on:
 *   - the CPU path (sv_ed25519_verify_batch_cpu / sv_ed25519_verify_cpu) gives
 *     the RFC 8032 section 7.1 verdicts (tests 1-3 valid; each with one bit
 *     flipped in R, S or the key invalid);
 *   - the GPU entry point either returns SV_OK with the same verdicts or a
 *     negative SV_ERR_*, and on an error the caller re-runs the whole batch
 *     on the CPU path: an error is never a reject.
 * Prints "gpu_rc=<rc>" and "ok"; exit status 0 on success.
 */
#include <stdio.h>
#include <string.h>

#include "stellar_sigverify.h"

#define N 6

static const char* PK[3] = {
    "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a",
    "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c",
    "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025",
};
static const char* SIG[3] = {
    "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e06522490155"
    "5fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b",
    "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da"
    "085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00",
    "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac"
    "18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28dc027beceea1ec40a",
};
static const char* MSG[3] = {"", "72", "af82"};

static size_t unhex(uint8_t* out, const char* s) {
  size_t n = strlen(s) / 2;
  for (size_t i = 0; i < n; ++i) {
    unsigned v;
    sscanf(s + 2 * i, "%2x", &v);
    out[i] = (uint8_t)v;
  }
  return n;
}

int main(void) {
  uint8_t pk[N * 32], sig[N * 64], msg[16];
  uint64_t off[N];
  uint32_t len[N];
  uint8_t want[N], got[N];
  size_t mpos = 0;
  for (int i = 0; i < N; ++i) {
    const int v = i % 3;
    unhex(pk + 32 * i, PK[v]);
    unhex(sig + 64 * i, SIG[v]);
    off[i] = mpos;
    len[i] = (uint32_t)unhex(msg + mpos, MSG[v]);
    mpos += len[i];
    want[i] = i < 3;
  }
  sig[64 * 3 + 5] ^= 0x01;   /* R */
  sig[64 * 4 + 40] ^= 0x10;  /* S */
  pk[32 * 5 + 7] ^= 0x02;    /* A */

  printf("engine %s\n", sv_version());
  memset(got, 0xff, sizeof got);
  if (sv_ed25519_verify_batch_cpu(pk, sig, msg, off, len, N, got, 2) != SV_OK || memcmp(got, want, N) != 0) {
    printf("cpu path: wrong verdicts\n");
    return 1;
  }
  for (int i = 0; i < N; ++i)
    if (sv_ed25519_verify_cpu(pk + 32 * i, sig + 64 * i, msg + off[i], len[i]) != want[i]) {
      printf("cpu single %d: wrong verdict\n", i);
      return 1;
    }

  /* the call site of INTEGRATION.md section 2: the GPU batch, and on any
   * error the same batch on the CPU path */
  sv_opts o;
  memset(&o, 0, sizeof o);
  o.struct_size = sizeof o;
  o.device = -1;
  memset(got, 0xff, sizeof got);
  const int rc = sv_ed25519_verify_batch(pk, sig, msg, off, len, N, got, &o);
  printf("gpu_rc=%d\n", rc);
  if (rc != SV_OK) {
    printf("engine error (%s): batch re-run on the CPU path\n", sv_last_error_string());
    if (sv_ed25519_verify_batch_cpu(pk, sig, msg, off, len, N, got, 0) != SV_OK) return 1;
  }
  if (memcmp(got, want, N) != 0) {
    printf("batch: wrong verdicts\n");
    return 1;
  }
  sv_shutdown();
  printf("ok\n");
  return 0;
}
