/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see ed25519_oracle.c header).
 * C restatement of libsodium 1.0.18 crypto_sign_verify_detached semantics as
 * called by stellar-core PubKeyUtils::verifySig (src/crypto/SecretKey.cpp:461-463).
 */
#ifndef STELLAR_AMD_ORACLE_H
#define STELLAR_AMD_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 0 iff valid, -1 otherwise (libsodium return convention). */
int oracle_ed25519_verify(const uint8_t sig[64], const uint8_t* m, size_t mlen, const uint8_t pk[32]);

/* verdict[i] = 1 iff signature i verifies (message i = msg[msg_off[i] .. +msg_len[i]]). */
void oracle_ed25519_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                                 const uint64_t* msg_off, const uint32_t* msg_len, size_t n,
                                 uint8_t* verdict);

/* RFC 8032 deterministic key generation and signing (== libsodium crypto_sign_seed_keypair,
 * crypto_sign_detached). sk = seed || pk. */
void oracle_ed25519_seed_keypair(uint8_t pk[32], uint8_t sk[64], const uint8_t seed[32]);
void oracle_ed25519_sign(uint8_t sig[64], const uint8_t* m, size_t mlen, const uint8_t sk[64]);

void oracle_sha512(uint8_t out[64], const uint8_t* m, size_t n);
void oracle_sc_reduce64(uint8_t out[32], const uint8_t in[64]);
const char* oracle_version(void);

#ifdef __cplusplus
}
#endif
#endif
