// CPU path of the engine (include/stellar_sigverify.h sv_ed25519_verify_batch_cpu).
//
// The same per-signature algorithm as the GPU kernels -- checks (1)-(5) of
// libsodium's crypto_sign_verify_detached, SHA-512(R || A || M) mod L, the
// half-size equation [c1 S mod L] B + [c0](-A) + [c1](-R) == O of lattice.h --
// compiled from the same headers for the host (g++: SV_HD = static inline).
// Two things differ: the base-point digit radix is 2^8 instead of 2^16, so the
// two host tables (e B and e 2^128 B, e <= 128) are 2 x 129 entries built in a
// few milliseconds at first use instead of the GPU's 2 x 32769; and the field
// elements are 5 x 51-bit limbs (fe51_host.h) instead of the device's 10 x
// 25.5-bit ones, behind the same interface.
//
// Role: an engine error is never a reject -- the
// caller re-runs the batch here -- and a single verifySig is cheaper here than
// a GPU round trip.  Reference semantics: libsodium 1.0.18
// crypto_sign_verify_detached as called by PubKeyUtils::verifySig
// (/root/reference/src/crypto/SecretKey.cpp:461-463).  Not the oracle: nothing
// under oracle/ is compiled or linked here.
#define SV_LB_BITS 8
// field arithmetic in radix 2^51 with 128-bit products (fe51_host.h): what
// x86-64 multiplies fastest; the device form's 10 x 32-bit limbs would cost 4x
// the multiplications here
#define SV_HOST_FE51 1
#include "verify_core.h"

#include <algorithm>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/stellar_sigverify.h"

namespace {

std::vector<sv_u4> g_tab;  // table t entry e at (t * SV_LBTAB_ENTRIES + e) * SV_BTAB_QUADS
std::once_flag g_once;

void build_tables() {
  g_tab.assign((size_t)2 * SV_LBTAB_ENTRIES * SV_BTAB_QUADS, sv_u4{0, 0, 0, 0});
  const unsigned T = 4;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; ++t)
    th.emplace_back([t] {
      for (int k = (int)t; k < 2 * SV_LBTAB_ENTRIES; k += (int)T) {
        const int tab = k / SV_LBTAB_ENTRIES, e = k % SV_LBTAB_ENTRIES;
        sv_btab_entry_shift((uint32_t*)&g_tab[(size_t)k * SV_BTAB_QUADS], e, 128 * tab);
      }
    });
  for (auto& x : th) x.join();
}

inline void words(uint32_t w[8], const uint8_t* b) { std::memcpy(w, b, 32); }

bool verify_one(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t len, sv_u4* slot) {
  uint32_t A[8], R[8], S[8], hram[16];
  words(A, pk);
  words(R, sig);
  words(S, sig + 32);
  sha512_ram_var(hram, R, A, msg, len);
  sv_u4* tabA = slot;
  sv_u4* tabR = slot + SV_ATAB_ENTRIES * SV_LTAB_QUADS;
  sv_lat lat;
  const bool ok = sv_lat_pre(lat, A, R, S, hram, tabA, tabR);
  const int W = sv_lat_windows(lat.bits);
  sv_lat_digits D;
  sv_lat_prepare(D, lat, S, W);
  ge_p3 P;
  const sv_u4* t0 = g_tab.data();
  const sv_u4* t1 = t0 + (size_t)SV_LBTAB_ENTRIES * SV_BTAB_QUADS;
  sv_lat_scalarmult(P, D, W, tabA, tabR, t0, t1);
  return ok && sv_is_identity(P);
}

}  // namespace

extern "C" {

int sv_ed25519_verify_batch_cpu(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                                const uint32_t* msg_len, size_t n, uint8_t* verdict, int threads) {
  if (n == 0) return SV_OK;
  if (!pk || !sig || !msg_off || !msg_len || !verdict) return SV_ERR_INVALID_ARG;
  if (!msg)
    for (size_t i = 0; i < n; ++i)
      if (msg_len[i]) return SV_ERR_INVALID_ARG;
  std::call_once(g_once, build_tables);
  size_t T = threads > 0 ? (size_t)threads : std::min<size_t>(16, std::max(1u, std::thread::hardware_concurrency()));
  T = std::max<size_t>(1, std::min(T, n / 8));
  auto work = [&](size_t t) {
    std::vector<sv_u4> slot(SV_SLOT_QUADS_L);
    const size_t a = n * t / T, b = n * (t + 1) / T;
    for (size_t i = a; i < b; ++i)
      verdict[i] = verify_one(pk + 32 * i, sig + 64 * i, msg ? msg + msg_off[i] : nullptr, msg_len[i], slot.data())
                       ? 1
                       : 0;
  };
  if (T == 1) {
    work(0);
    return SV_OK;
  }
  std::vector<std::thread> th;
  for (size_t t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  return SV_OK;
}

int sv_ed25519_verify_cpu(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, size_t msg_len) {
  if (!pk || !sig || (!msg && msg_len) || msg_len > 0xffffffffu) return SV_ERR_INVALID_ARG;
  std::call_once(g_once, build_tables);
  static thread_local std::vector<sv_u4> slot(SV_SLOT_QUADS_L);
  return verify_one(pk, sig, msg, (uint32_t)msg_len, slot.data()) ? 1 : 0;
}

}  // extern "C"
