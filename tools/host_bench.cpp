// Host-side cost of the C++ mirror (PubKeyUtils / SignatureChecker /
// VerifyMicroBatcher) with the engine replaced by a stub (every signature
// valid; the keyed stub returns sig[0..32) as the cache key): what the
// integration layer costs on top of the engine, per signature.
//   g++ -O2 -std=c++17 tools/host_bench.cpp -Istellar-core_amd/csrc/host \
//       -Lstellar-core_amd -lstellar_host -lstellar_sigverify -Wl,-rpath,$PWD/stellar-core_amd -lpthread
#include <chrono>
#include <cstdio>
#include <cstring>
#include <future>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "PubKeyUtils.h"
#include "SignatureChecker.h"
#include "VerifyMicroBatcher.h"

using namespace stellar;
using clk = std::chrono::steady_clock;

static int stub_verify(const uint8_t*, const uint8_t*, const uint8_t*, const uint64_t*, const uint32_t*, size_t n,
                       uint8_t* v) {
  memset(v, 1, n);
  return 0;
}
static int stub_keyed(const uint8_t*, const uint8_t* sig, const uint8_t*, const uint64_t*, const uint32_t*, size_t n,
                      uint8_t* v, uint8_t* keys) {
  memset(v, 1, n);
  for (size_t i = 0; i < n; ++i) memcpy(keys + 32 * i, sig + 64 * i, 32);
  return 0;
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)atol(argv[1]) : 100000;
  std::mt19937_64 rng(1);
  std::vector<PublicKey> keys(n);
  std::vector<Signature> sigs(n, Signature(64));
  std::vector<std::vector<uint8_t>> msgs(n, std::vector<uint8_t>(32));
  for (size_t i = 0; i < n; ++i) {
    for (auto& b : keys[i].ed25519()) b = (uint8_t)rng();
    for (auto& b : sigs[i]) b = (uint8_t)rng();
    for (auto& b : msgs[i]) b = (uint8_t)rng();
  }
  std::vector<PubKeyUtils::VerifyItem> items(n);
  for (size_t i = 0; i < n; ++i) items[i] = PubKeyUtils::VerifyItem{&keys[i], ByteSlice(sigs[i]), ByteSlice(msgs[i])};

  auto time = [&](const char* what, auto fn, int reps = 3) {
    double best = 1e9;
    for (int r = 0; r < reps; ++r) {
      PubKeyUtils::clearVerifySigCache();
      auto t0 = clk::now();
      fn();
      best = std::min(best, std::chrono::duration<double>(clk::now() - t0).count());
    }
    printf("%-58s %8.2f ms  %7.1f ns/sig  %6.2f M sig/s\n", what, best * 1e3, best * 1e9 / n, n / best / 1e6);
  };

  const bool gpu = argc > 2 && std::string(argv[2]) == "gpu";
  if (gpu) {
    // the real engine (GPU); random bytes verify as invalid at the same cost
    PubKeyUtils::setKeyedBatchThreshold(256);
    PubKeyUtils::verifySigBatch(items);  // warm: device init, staging, workspace
    time("verifySigBatch keyed (GPU engine), cold cache", [&] { PubKeyUtils::verifySigBatch(items); }, 5);
    PubKeyUtils::setKeyedBatchThreshold(0);
    time("verifySigBatch host-hashed (GPU engine), cold cache", [&] { PubKeyUtils::verifySigBatch(items); }, 3);
    PubKeyUtils::setKeyedBatchThreshold(256);
  }
  PubKeyUtils::setKeyedBatchVerifierForTesting(stub_keyed);
  PubKeyUtils::setKeyedBatchThreshold(1);
  time("verifySigBatch keyed (stub engine), cold cache", [&] { PubKeyUtils::verifySigBatch(items); });
  PubKeyUtils::setKeyedBatchVerifierForTesting(nullptr);
  PubKeyUtils::setKeyedBatchThreshold(0);
  PubKeyUtils::setBatchVerifierForTesting(stub_verify);
  time("verifySigBatch host-hashed (stub engine), cold cache", [&] { PubKeyUtils::verifySigBatch(items); });

  // tx set pre-pass: n signatures as n / 10 txs of 10 signers each
  {
    const size_t ntx = n / 10;
    std::vector<Hash> hashes(ntx);
    std::vector<std::vector<DecoratedSignature>> ds(ntx);
    std::vector<std::vector<Signer>> sg(ntx);
    for (size_t t = 0; t < ntx; ++t) {
      for (auto& b : hashes[t]) b = (uint8_t)rng();
      for (int k = 0; k < 10; ++k) {
        Signer s;
        s.key.key = keys[10 * t + k].ed25519();
        s.weight = 1;
        sg[t].push_back(s);
        DecoratedSignature d;
        memcpy(d.hint.data(), s.key.key.data() + 28, 4);
        d.signature = sigs[10 * t + k];
        ds[t].push_back(d);
      }
    }
    if (gpu) PubKeyUtils::setBatchVerifierForTesting(nullptr);
    double tAdd = 1e9, tRun = 1e9, tChk = 1e9;
    time(gpu ? "tx set (GPU): prefetch add + run (side table) + checkers" : "tx set: prefetch add + run (side table) + 10-of-10 checkers", [&] {
      auto t0 = clk::now();
      SignatureBatchPrefetch pre;
      for (size_t t = 0; t < ntx; ++t) pre.add(hashes[t], ds[t], sg[t]);
      auto t1 = clk::now();
      pre.run(false);
      auto t2 = clk::now();
      size_t ok = 0;
      for (size_t t = 0; t < ntx; ++t) {
        SignatureChecker c(21, hashes[t], ds[t], &pre);
        ok += c.checkSignature(sg[t], 10) && c.checkAllSignaturesUsed();
      }
      auto t3 = clk::now();
      auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      tAdd = std::min(tAdd, ms(t0, t1));
      tRun = std::min(tRun, ms(t1, t2));
      tChk = std::min(tChk, ms(t2, t3));
      if (!gpu && ok != ntx) printf("unexpected: %zu of %zu\n", ok, ntx);
    });
    printf("  (best phases: add %.3f ms, run %.3f ms, checkers %.3f ms)\n", tAdd, tRun, tChk);
  }

  if (gpu) {
    // per-batch latency of the keyed path at micro-batcher sizes
    for (size_t b : {1024, 4096, 16384}) {
      std::vector<PubKeyUtils::VerifyItem> sub(items.begin(), items.begin() + b);
      PubKeyUtils::verifySigBatch(sub);
      double best = 1e9;
      for (int r = 0; r < 20; ++r) {
        PubKeyUtils::clearVerifySigCache();
        auto t0 = clk::now();
        PubKeyUtils::verifySigBatch(sub);
        best = std::min(best, std::chrono::duration<double>(clk::now() - t0).count());
      }
      printf("verifySigBatch keyed (GPU) one batch of %-6zu                  %8.3f ms\n", b, best * 1e3);
    }
    for (unsigned workers : {1u, 2u, 4u})
      for (size_t mb_size : {1024, 4096, 16384}) {
        char label[128];
        snprintf(label, sizeof label, "micro-batcher (GPU) post, 8 producers, %u workers, %zu/batch", workers, mb_size);
        time(label, [&] {
          VerifyMicroBatcher mb(mb_size, std::chrono::microseconds(1000), workers);
          std::vector<std::thread> th;
          for (int p = 0; p < 8; ++p)
            th.emplace_back([&, p] {
              for (size_t i = p; i < n; i += 8) mb.post(keys[i], ByteSlice(sigs[i]), ByteSlice(msgs[i]));
            });
          for (auto& t : th) t.join();
          mb.drain();
        });
      }
  }
  for (int post = 0; post < 2; ++post) {
    PubKeyUtils::setBatchVerifierForTesting(nullptr);
    PubKeyUtils::setKeyedBatchVerifierForTesting(gpu ? nullptr : stub_keyed);
    PubKeyUtils::setKeyedBatchThreshold(gpu ? 256 : 1);
    char label[128];
    snprintf(label, sizeof label, "micro-batcher%s 8 producers, 2 workers, 4096/batch (%s)", gpu ? " (GPU)" : "", post ? "post" : "submit");
    time(label, [&] {
      VerifyMicroBatcher mb(4096, std::chrono::microseconds(1000), 2);
      std::vector<std::thread> th;
      for (int p = 0; p < 8; ++p)
        th.emplace_back([&, p] {
          std::vector<std::future<bool>> f;
          for (size_t i = p; i < n; i += 8) {
            if (post) mb.post(keys[i], ByteSlice(sigs[i]), ByteSlice(msgs[i]));
            else f.push_back(mb.submit(keys[i], ByteSlice(sigs[i]), ByteSlice(msgs[i])));
          }
          for (auto& x : f) x.get();
        });
      for (auto& t : th) t.join();
      mb.drain();
    });
  }
  return 0;
}
