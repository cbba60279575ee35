// Micro-batcher for latency-bound single verifications.
//
// Reference pattern it replaces: the overlay thread pre-verifies every
// SCP_MESSAGE signature one by one and discards the result only to warm the
// global verify cache (/root/reference/src/overlay/Peer.cpp:963-970); the main
// thread's HerderImpl::verifyEnvelope (src/herder/HerderImpl.cpp:2414-2432)
// then hits the cache.  Here producers enqueue (pk, sig, msg) and get a
// future; a worker thread flushes the queue as ONE PubKeyUtils::verifySigBatch
// call (which also fills the cache) when it holds maxBatch items or when the
// oldest item has waited maxDelay -- whichever comes first.  With workers > 1
// several batches are in flight at once: one worker's host work (cache keys,
// cache lookups, packing, promise fulfilment) overlaps another's engine call.
// The engine and the verify cache are thread-safe, so verdicts do not depend
// on the worker count.  Default 2: with one worker a flood of 1k-item batches
// queued up behind the host work (p50 submit->verdict 229 ms at 0.31M/s); two
// measured 2.1 ms at 0.68M/s (tools/bench_configs.py configmb).
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <future>
#include <mutex>
#include <thread>
#include <vector>

#include "PubKeyUtils.h"

namespace stellar {

class VerifyMicroBatcher {
 public:
  VerifyMicroBatcher(size_t maxBatch, std::chrono::microseconds maxDelay, unsigned workers = 2);
  ~VerifyMicroBatcher();  // drains the queue, then stops the workers
  VerifyMicroBatcher(VerifyMicroBatcher const&) = delete;
  VerifyMicroBatcher& operator=(VerifyMicroBatcher const&) = delete;

  // Thread-safe.  The future carries the verdict, or VerifyEngineError.
  std::future<bool> submit(PublicKey const& key, Signature const& sig, ByteSlice const& msg);

  struct Stats {
    uint64_t items = 0;
    uint64_t batches = 0;
    uint64_t flushedBySize = 0;
    uint64_t flushedByDeadline = 0;
    uint64_t maxBatchSeen = 0;
  };
  Stats stats() const;
  // submit -> verdict-ready latencies in microseconds (recorded per item)
  std::vector<double> latencies() const;

 private:
  struct Item {
    PublicKey key;
    Signature sig;
    std::vector<uint8_t> msg;
    std::promise<bool> done;
    std::chrono::steady_clock::time_point t0;
  };
  void run();

  const size_t mMaxBatch;
  const std::chrono::microseconds mMaxDelay;
  mutable std::mutex mMu;
  std::condition_variable mCv;
  std::deque<Item> mQueue;
  bool mStop = false;
  Stats mStats;
  std::vector<double> mLatUs;
  std::vector<std::thread> mWorkers;
};

}  // namespace stellar
