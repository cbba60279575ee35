// Developer tool (CPU only, ThreadSanitizer): the C-ABI's slot-table lifetime
// under concurrent use.  Four threads call the verify,
// device-API, hashing and stats entry points on every slot while a fifth
// re-maps the slots (sv_set_device_map) and tears them down (sv_shutdown) in
// a loop.  The slots are stubs (SV_TEST_STUB_SLOTS, no GPU): every call that
// reaches a slot's HIP resources fails with SV_ERR_HIP, but it reads the slot
// table and the Device objects exactly as on a GPU, so a Device deleted under
// an in-flight call is a TSan report (or a crash).  Built and run by
// tools/tsan_host.sh; prints "ok <calls> <remaps>".
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/stellar_sigverify.h"

int main() {
  setenv("SV_TEST_KNOBS", "1", 1);
  setenv("SV_TEST_STUB_SLOTS", "3", 1);
  if (sv_device_count() != 3) {
    fprintf(stderr, "stub slots not created: %s\n", sv_last_error_string());
    return 1;
  }
  std::atomic<bool> stop{false};
  std::atomic<long> calls{0}, remaps{0}, bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t) {
    th.emplace_back([&, t] {
      uint8_t pk[32 * 4] = {0}, sig[64 * 4] = {0}, msg[32 * 4] = {0}, out[4], keys[32 * 4];
      uint64_t off[4] = {0, 32, 64, 96};
      uint32_t len[4] = {32, 32, 32, 32};
      long k = 0;
      while (!stop.load()) {
        sv_opts o;
        memset(&o, 0, sizeof(o));
        o.struct_size = sizeof(o);
        o.device = (int)((k + t) % 4) - 1;  // -1 (any slot) and each slot
        int rc;
        switch ((k + t) % 6) {
          case 0: rc = sv_ed25519_verify_batch(pk, sig, msg, off, len, 4, out, &o); break;
          case 1: rc = sv_ed25519_verify_batch_fixed(pk, sig, msg, 32, 4, out, &o); break;
          case 2: rc = sv_ed25519_verify_device((int)(k % 3), pk, sig, msg, nullptr, nullptr, 32, 4, out, nullptr,
                                                nullptr);
                  break;
          case 3: rc = sv_verify_cache_keys(pk, sig, msg, off, len, 4, keys, &o); break;
          case 4: {
            sv_key_cache_stats st;
            memset(&st, 0, sizeof(st));
            rc = sv_key_cache_get_stats((int)(k % 3), &st);
            break;
          }
          default: {
            size_t b = 0;
            rc = sv_workspace_bytes((int)(k % 3), &b);
            (void)sv_device_count();
            break;
          }
        }
        // stubs: SV_OK for pure bookkeeping, SV_ERR_HIP / SV_ERR_NO_DEVICE /
        // SV_ERR_INVALID_ARG (slot gone between remaps) otherwise; never a crash
        if (rc != SV_OK && rc != SV_ERR_HIP && rc != SV_ERR_NO_DEVICE && rc != SV_ERR_INVALID_ARG) bad.fetch_add(1);
        ++k;
        calls.fetch_add(1);
      }
    });
  }
  th.emplace_back([&] {
    for (int r = 0; r < 400; ++r) {
      if (r % 2) {
        sv_shutdown();
      } else {
        const int map[3] = {0, 0, 0};
        (void)sv_set_device_map(map, 1 + r % 3);
      }
      remaps.fetch_add(1);
      // (callers run between teardowns: the lock prefers the writer, so a
      // back-to-back remap loop would otherwise leave them no turn)
      std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
    stop.store(true);
  });
  for (auto& x : th) x.join();
  sv_shutdown();
  if (bad.load()) {
    fprintf(stderr, "unexpected return codes: %ld\n", bad.load());
    return 1;
  }
  if (calls.load() < 4 * remaps.load()) {
    fprintf(stderr, "callers starved: %ld calls over %ld remaps\n", calls.load(), remaps.load());
    return 1;
  }
  printf("ok %ld %ld\n", calls.load(), remaps.load());
  return 0;
}
