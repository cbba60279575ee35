// Micro-batcher for latency-bound single verifications.
//
// Reference pattern it replaces: the overlay thread pre-verifies every
// SCP_MESSAGE signature one by one and discards the result only to warm the
// global verify cache (/root/reference/src/overlay/Peer.cpp:963-970); the main
// thread's HerderImpl::verifyEnvelope (src/herder/HerderImpl.cpp:2414-2432)
// then hits the cache.  Here producers enqueue (pk, sig, msg) -- post() when
// the result is only meant to warm the cache, exactly like the reference's
// pre-verify, or submit() for a future carrying the verdict -- and a worker
// thread flushes the queue as ONE PubKeyUtils::verifySigBatch call (which also
// fills the cache).  When a flush happens is the FlushPolicy:
//   WhenIdle (default): as soon as fewer than `idleInFlight` batches are being
//     verified, a worker flushes whatever is queued (after an optional
//     `linger` counted from the oldest item's arrival, to let a burst that is
//     still arriving join the batch); while batches are in flight items
//     accumulate and are flushed when one completes, at maxBatch items, or at
//     the oldest item's maxDelay deadline, whichever comes first.  A lone SCP
//     envelope is verified at once (a one-item batch takes the CPU path, no GPU
//     round trip), and under load the batches grow by themselves.
//   Deadline: flush at maxBatch items or when the oldest has waited maxDelay
//     (the round-2 policy: every sub-maxBatch batch pays the full maxDelay).
// With workers > 1 several batches are in flight at once: one worker's host
// work (cache walk, promise fulfilment) overlaps another's engine call.  The
// engine and the verify cache are thread-safe, so verdicts do not depend on
// the worker count or the policy.
//
// Queue layout: kShards sub-queues, each fixed records (key, signature
// bytes) plus one byte arena for the messages under its own mutex; a producer
// thread always appends to "its" shard (so concurrent producers rarely share a
// lock) and a flushing worker swaps whole sub-queues out, so enqueueing is one
// short uncontended critical section and no allocation per item (submit()
// allocates its promise).  Item order inside a batch follows the shards;
// verdicts do not depend on it.
//
// Engine errors never reach producers: verifySigBatch re-runs a failed batch
// on the CPU path (PubKeyUtils.h).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <future>
#include <mutex>
#include <thread>
#include <vector>

#include "PubKeyUtils.h"

namespace stellar {

class VerifyMicroBatcher {
 public:
  enum class FlushPolicy { WhenIdle, Deadline };
  struct Options {
    size_t maxBatch = 8192;
    std::chrono::microseconds maxDelay{2000};
    unsigned workers = 2;
    // keep submit -> verdict latencies of the most recent kLatencySamples
    // items (off by default: a long-running node keeps none)
    bool recordLatency = false;
    FlushPolicy policy = FlushPolicy::WhenIdle;
    // WhenIdle: a worker flushes at once while fewer than this many batches
    // are in flight (1: the engine's latency lane is never queued behind a
    // second small batch of ours)
    unsigned idleInFlight = 1;
    // WhenIdle: an idle flush waits until the oldest item is this old
    std::chrono::microseconds linger{0};
    // WhenIdle: while a burst is arriving (more than one item queued and the
    // newest less than `quiet` old) an idle flush waits for the burst to end,
    // at most until the oldest item is `maxLinger` old, so a burst becomes one
    // batch instead of a small first batch that the rest queues behind.  A
    // lone item is flushed at once.  0 (the default) disables: for SCP-shaped
    // bursts arriving over ~0.1-0.2 ms, verifying the early part while the
    // rest arrives measured faster (bursts of 1k every 5 ms, submit -> batch
    // verified p50 0.23-0.26 ms without the wait, 0.27-0.30 ms with it:
    // profiles/r05/config4_integrated/).  (The wait is a yield loop without
    // the queue lock: a condition-variable timeout this short oversleeps by
    // the timer slack.)
    std::chrono::microseconds quiet{0};
    std::chrono::microseconds maxLinger{200};
    // Batch continuation for submitTagged() items: one call per flushed batch,
    // onBatch(tags, verdicts, n) with the batch's tagged items in batch order,
    // on the flush worker once their verdicts are IN THE VERIFY CACHE (after the
    // batch's promises and per-item continuations).  What an overlay that posts
    // one main-thread task per batch of SCP messages needs: one post per batch
    // instead of one per envelope (Peer.cpp:977-981 posts each message).  Must
    // not throw; a batch that throws (a non-ed25519 key) delivers 0 verdicts.
    std::function<void(const uint64_t* tags, const uint8_t* verdicts, size_t n)> onBatch;
  };
  explicit VerifyMicroBatcher(Options const& opts);
  VerifyMicroBatcher(size_t maxBatch, std::chrono::microseconds maxDelay, unsigned workers = 2,
                     bool recordLatency = false, FlushPolicy policy = FlushPolicy::WhenIdle);
  ~VerifyMicroBatcher();  // drains the queue, then stops the workers
  VerifyMicroBatcher(VerifyMicroBatcher const&) = delete;
  VerifyMicroBatcher& operator=(VerifyMicroBatcher const&) = delete;

  // Thread-safe.  The future carries the verdict.
  std::future<bool> submit(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg);
  // Thread-safe, fire and forget: the verdict lands in the verify cache only.
  void post(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg);
  // Thread-safe continuation form: onVerdict(valid) runs on a flush worker
  // once the item's batch is verified and its verdict is IN THE VERIFY CACHE.
  // This keeps the reference's ordering at Peer.cpp:963-979, where the
  // overlay thread's pre-verify completes before the message is posted to the
  // main thread: post the message from onVerdict and HerderImpl::
  // verifyEnvelope's verifySig is a cache hit.  onVerdict must not throw and
  // should be short (it delays the batch's other continuations); if the batch
  // throws (a non-ed25519 key: the reference's releaseAssert) it gets false.
  void submit(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg, std::function<void(bool)> onVerdict);
  // Thread-safe batch-continuation form: the verdict reaches Options::onBatch
  // with `tag`, together with the rest of its batch (no allocation per item).
  void submitTagged(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg, uint64_t tag);
  // Blocks until every item enqueued before the call has been verified.
  void drain();

  struct Stats {
    uint64_t items = 0;
    uint64_t batches = 0;
    uint64_t flushedBySize = 0;
    uint64_t flushedByDeadline = 0;
    uint64_t flushedIdle = 0;  // WhenIdle: below maxBatch, before the deadline, engine idle
    uint64_t burstWaits = 0;   // WhenIdle: idle flushes that first waited for a burst to end (quiet)
    uint64_t maxBatchSeen = 0;
  };
  Stats stats() const;
  static constexpr size_t kLatencySamples = 1 << 16;
  // submit -> verdict-ready latencies in microseconds (recordLatency only;
  // the most recent kLatencySamples items)
  std::vector<double> latencies() const;

 private:
  using Clock = std::chrono::steady_clock;
  struct Rec {
    PublicKey key;
    uint8_t sig[64];
    uint32_t sigLen;
    uint32_t msgLen;
    uint64_t msgOff;           // into the arena
    std::promise<bool>* done;  // submit() only
    std::function<void(bool)>* cb;  // submit(.., onVerdict) only
    uint64_t tag;              // submitTagged() only (tagged)
    bool tagged;
    Clock::time_point t0;      // recordLatency only
    int64_t arrivalNs;         // deadline accounting (steady clock)
  };
  int64_t oldestQueuedNs();  // arrival of the oldest queued record (INT64_MAX: none)
  struct Queue {
    std::vector<Rec> recs;
    std::vector<uint8_t> arena;
  };
  static constexpr size_t kShards = 8;
  struct alignas(64) Shard {
    std::mutex mu;
    Queue q;
  };
  void enqueue(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg, std::promise<bool>* done,
               std::function<void(bool)>* cb, bool tagged = false, uint64_t tag = 0);
  void wake();
  // moves up to `want` of the oldest items of shard s into `into`; returns the count
  size_t takeFrom(size_t s, size_t want, Queue& into);
  void run();
  void deliverTagged(std::vector<Rec const*> const& recs, size_t take, std::vector<bool> const* v,
                     std::vector<uint64_t>& tags, std::vector<uint8_t>& verdicts);

  const size_t mMaxBatch;
  const std::chrono::microseconds mMaxDelay;
  const bool mRecordLatency;
  const FlushPolicy mPolicy;
  const unsigned mIdleInFlight;
  const std::chrono::microseconds mLinger;
  const std::chrono::microseconds mQuiet, mMaxLinger;
  const std::function<void(const uint64_t*, const uint8_t*, size_t)> mOnBatch;
  std::atomic<int64_t> mNewestNs{0};  // arrival of the newest queued item (a hint: WhenIdle's quiet period)
  unsigned mInFlight = 0;  // batches being verified (under mMu)
  Shard mShards[kShards];
  std::atomic<size_t> mQueued{0};
  std::atomic<uint64_t> mEnqueued{0};
  std::atomic<unsigned> mNextShard{0};
  mutable std::mutex mMu;  // worker wake-ups, stats, drain
  std::condition_variable mCv;
  std::condition_variable mDoneCv;
  bool mStop = false;
  uint64_t mCompleted = 0;
  Stats mStats;
  std::vector<double> mLatUs;  // ring of kLatencySamples
  size_t mLatNext = 0;
  std::vector<std::thread> mWorkers;
};

}  // namespace stellar
