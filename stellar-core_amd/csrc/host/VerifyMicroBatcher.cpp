// See VerifyMicroBatcher.h.
#include "VerifyMicroBatcher.h"

#include <algorithm>
#include <climits>
#include <cstring>
#include <exception>

namespace stellar {

namespace {
int64_t nowNs() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

VerifyMicroBatcher::VerifyMicroBatcher(Options const& o)
    : mMaxBatch(std::max<size_t>(1, o.maxBatch)),
      mMaxDelay(o.maxDelay),
      mRecordLatency(o.recordLatency),
      mPolicy(o.policy),
      mIdleInFlight(std::max(1u, o.idleInFlight)),
      mLinger(std::min(o.linger, o.maxDelay)),
      mQuiet(o.quiet),
      mMaxLinger(std::min(o.maxLinger, o.maxDelay)),
      mOnBatch(o.onBatch) {
  const unsigned w = std::max(1u, o.workers);
  mWorkers.reserve(w);
  for (unsigned i = 0; i < w; ++i) mWorkers.emplace_back([this] { run(); });
}

namespace {
VerifyMicroBatcher::Options makeOptions(size_t maxBatch, std::chrono::microseconds maxDelay, unsigned workers,
                                        bool recordLatency, VerifyMicroBatcher::FlushPolicy policy) {
  VerifyMicroBatcher::Options o;
  o.maxBatch = maxBatch;
  o.maxDelay = maxDelay;
  o.workers = workers;
  o.recordLatency = recordLatency;
  o.policy = policy;
  return o;
}
}  // namespace

VerifyMicroBatcher::VerifyMicroBatcher(size_t maxBatch, std::chrono::microseconds maxDelay, unsigned workers,
                                       bool recordLatency, FlushPolicy policy)
    : VerifyMicroBatcher(makeOptions(maxBatch, maxDelay, workers, recordLatency, policy)) {}

VerifyMicroBatcher::~VerifyMicroBatcher() {
  {
    std::lock_guard<std::mutex> g(mMu);
    mStop = true;
  }
  mCv.notify_all();
  for (auto& w : mWorkers) w.join();
}

void VerifyMicroBatcher::wake() {
  { std::lock_guard<std::mutex> g(mMu); }  // a worker between its check and its wait cannot miss this
  mCv.notify_one();
}

void VerifyMicroBatcher::enqueue(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg,
                                 std::promise<bool>* done, std::function<void(bool)>* cb, bool tagged, uint64_t tag) {
  // each producer thread keeps to one shard
  thread_local unsigned tShard = ~0u;
  if (tShard == ~0u) tShard = mNextShard.fetch_add(1) % kShards;
  Rec r;
  r.key = key;
  // anything but a 64-byte signature is rejected by verifySig before it is
  // read; keep at most 64 bytes and the size (clamped to 65)
  r.sigLen = (uint32_t)std::min<size_t>(sig.size(), 65);
  std::memcpy(r.sig, sig.data(), std::min<size_t>(sig.size(), 64));
  r.msgLen = (uint32_t)msg.size();
  r.done = done;
  r.cb = cb;
  r.tagged = tagged;
  r.tag = tag;
  if (mRecordLatency) r.t0 = Clock::now();
  r.arrivalNs = nowNs();
  mNewestNs.store(r.arrivalNs, std::memory_order_relaxed);
  size_t q;
  {
    Shard& sh = mShards[tShard];
    std::lock_guard<std::mutex> g(sh.mu);
    r.msgOff = sh.q.arena.size();
    sh.q.arena.insert(sh.q.arena.end(), msg.begin(), msg.end());
    sh.q.recs.push_back(r);
    // counted under the shard lock: a worker that takes this record (under
    // the same lock) always finds it counted, so its fetch_sub never wraps
    mEnqueued.fetch_add(1);
    q = mQueued.fetch_add(1) + 1;
  }
  if (q == 1 || q == mMaxBatch) wake();
}

int64_t VerifyMicroBatcher::oldestQueuedNs() {
  int64_t oldest = INT64_MAX;
  for (size_t s = 0; s < kShards; ++s) {
    Shard& sh = mShards[s];
    std::lock_guard<std::mutex> g(sh.mu);
    if (!sh.q.recs.empty()) oldest = std::min(oldest, sh.q.recs.front().arrivalNs);  // (FIFO per shard)
  }
  return oldest;
}

std::future<bool> VerifyMicroBatcher::submit(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg) {
  auto* p = new std::promise<bool>();
  std::future<bool> f = p->get_future();
  enqueue(key, sig, msg, p, nullptr);
  return f;
}

void VerifyMicroBatcher::submit(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg,
                                std::function<void(bool)> onVerdict) {
  enqueue(key, sig, msg, nullptr, onVerdict ? new std::function<void(bool)>(std::move(onVerdict)) : nullptr);
}

void VerifyMicroBatcher::submitTagged(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg,
                                      uint64_t tag) {
  enqueue(key, sig, msg, nullptr, nullptr, true, tag);
}

void VerifyMicroBatcher::post(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg) {
  enqueue(key, sig, msg, nullptr, nullptr);
}

void VerifyMicroBatcher::drain() {
  std::unique_lock<std::mutex> lk(mMu);
  const uint64_t target = mEnqueued.load();
  mCv.notify_all();
  mDoneCv.wait(lk, [&] { return mCompleted >= target; });
}

VerifyMicroBatcher::Stats VerifyMicroBatcher::stats() const {
  std::lock_guard<std::mutex> g(mMu);
  return mStats;
}

std::vector<double> VerifyMicroBatcher::latencies() const {
  std::lock_guard<std::mutex> g(mMu);
  return mLatUs;
}

size_t VerifyMicroBatcher::takeFrom(size_t s, size_t want, Queue& into) {
  Shard& sh = mShards[s];
  std::lock_guard<std::mutex> g(sh.mu);
  Queue& q = sh.q;
  const size_t n = q.recs.size();
  if (n == 0 || want == 0) return 0;
  into.recs.clear();
  into.arena.clear();
  if (n <= want) {
    std::swap(into, q);  // the whole sub-queue, no copy
    return n;
  }
  const uint64_t cut = q.recs[want].msgOff;  // the oldest `want` items; the rest stay (offsets rebased)
  into.recs.assign(q.recs.begin(), q.recs.begin() + want);
  into.arena.assign(q.arena.begin(), q.arena.begin() + cut);
  q.recs.erase(q.recs.begin(), q.recs.begin() + want);
  q.arena.erase(q.arena.begin(), q.arena.begin() + cut);
  for (Rec& r : q.recs) r.msgOff -= cut;
  return want;
}

// The batch's tagged items to Options::onBatch in one call (v == nullptr: the
// batch threw, every verdict 0).
void VerifyMicroBatcher::deliverTagged(std::vector<Rec const*> const& recs, size_t take, std::vector<bool> const* v,
                                       std::vector<uint64_t>& tags, std::vector<uint8_t>& verdicts) {
  tags.clear();
  verdicts.clear();
  for (size_t i = 0; i < take; ++i)
    if (recs[i]->tagged) {
      tags.push_back(recs[i]->tag);
      verdicts.push_back(v && (*v)[i] ? 1 : 0);
    }
  if (tags.empty() || !mOnBatch) return;
  try {
    mOnBatch(tags.data(), verdicts.data(), tags.size());
  } catch (...) {  // (a continuation must not take the worker down)
  }
}

void VerifyMicroBatcher::run() {
  std::vector<Queue> parts(kShards);
  std::vector<PubKeyUtils::VerifyItem> items;
  std::vector<Rec const*> recs;
  std::vector<double> lat;
  std::vector<uint64_t> tags;  // the batch's submitTagged() items, in batch order
  std::vector<uint8_t> tagVerdicts;
  size_t start = 0;
  std::unique_lock<std::mutex> lk(mMu);
  for (;;) {
    // wait for: stop, a full batch, an idle engine (WhenIdle) or the oldest
    // item's deadline
    while (!mStop && mQueued.load() == 0) mCv.wait(lk);
    if (mQueued.load() == 0) return;  // stop requested and every queue drained
    bool idle = false;
    if (mQueued.load() < mMaxBatch && !mStop) {
      // (read from the queues themselves: a count-based "first arrival" mark
      // can lag a concurrent take)
      const int64_t oldest = oldestQueuedNs();
      if (oldest == INT64_MAX) {  // another worker is taking everything
        mCv.wait_for(lk, std::chrono::microseconds(20));
        continue;
      }
      const int64_t now = nowNs();
      const int64_t deadline = oldest + (int64_t)mMaxDelay.count() * 1000;
      const bool whenIdle = mPolicy == FlushPolicy::WhenIdle;
      if (whenIdle && mInFlight < mIdleInFlight) {
        const int64_t lingerEnd = oldest + (int64_t)mLinger.count() * 1000;
        if (now < lingerEnd && now < deadline) {
          mCv.wait_for(lk, std::chrono::nanoseconds(lingerEnd - now),
                       [&] { return mStop || mQueued.load() >= mMaxBatch; });
          continue;
        }
        if (mQuiet.count() > 0 && mQueued.load() > 1) {
          // a burst: wait (unlocked, yielding) until it has been quiet for
          // mQuiet, the oldest item is mMaxLinger old, or a batch is full
          const int64_t cap = std::min(oldest + (int64_t)mMaxLinger.count() * 1000, deadline);
          const int64_t q = (int64_t)mQuiet.count() * 1000;
          if (now < cap && now - mNewestNs.load(std::memory_order_relaxed) < q) {
            lk.unlock();
            for (;;) {
              const int64_t t = nowNs();
              if (t >= cap || t - mNewestNs.load(std::memory_order_relaxed) >= q || mQueued.load() >= mMaxBatch)
                break;
              std::this_thread::yield();
            }
            lk.lock();
            ++mStats.burstWaits;
            continue;  // (re-evaluate: another worker may have flushed meanwhile)
          }
        }
        idle = now < deadline;
      } else if (now < deadline) {
        // (WhenIdle: a completing batch notifies, and the engine is idle again)
        mCv.wait_for(lk, std::chrono::nanoseconds(deadline - now), [&] {
          return mStop || mQueued.load() >= mMaxBatch || (whenIdle && mInFlight < mIdleInFlight);
        });
        continue;  // re-evaluate: another worker may have taken the queue meanwhile
      }
    }
    const bool bySize = mQueued.load() >= mMaxBatch;
    ++mInFlight;
    lk.unlock();
    // collect up to maxBatch items, starting from a rotating shard
    size_t take = 0;
    for (size_t k = 0; k < kShards; ++k) {
      const size_t s = (start + k) % kShards;
      const size_t got = takeFrom(s, mMaxBatch - take, parts[s]);
      if (got == 0) parts[s].recs.clear();
      take += got;
    }
    start = (start + 1) % kShards;
    const size_t left = mQueued.fetch_sub(take) - take;
    if (left >= mMaxBatch) wake();  // (the leftovers keep their own arrival times)
    if (take == 0) {
      lk.lock();
      --mInFlight;
      continue;
    }
    items.clear();
    recs.clear();
    for (size_t s = 0; s < kShards; ++s) {
      const uint8_t* arena = parts[s].arena.data();
      for (Rec const& r : parts[s].recs) {
        items.push_back(PubKeyUtils::VerifyItem{&r.key, ByteSlice(r.sig, r.sigLen), ByteSlice(arena + r.msgOff, r.msgLen)});
        recs.push_back(&r);
      }
    }
    bool ok = true;
    // The engine is free once verifySigBatch returns: the next batch may be
    // flushed (WhenIdle) while this one's promises and continuations run.
    bool released = false;
    auto release = [&] {
      if (released) return;
      released = true;
      std::lock_guard<std::mutex> g(mMu);
      --mInFlight;
      if (mPolicy == FlushPolicy::WhenIdle && mQueued.load() > 0) mCv.notify_all();
    };
    try {
      std::vector<bool> v = PubKeyUtils::verifySigBatch(items);
      release();
      if (mRecordLatency) {
        const auto now = Clock::now();
        lat.resize(take);
        for (size_t i = 0; i < take; ++i) lat[i] = std::chrono::duration<double, std::micro>(now - recs[i]->t0).count();
      }
      for (size_t i = 0; i < take; ++i) {
        if (std::promise<bool>* p = recs[i]->done) {
          p->set_value(v[i]);
          delete p;
        }
        if (std::function<void(bool)>* c = recs[i]->cb) {
          try {
            (*c)(v[i]);
          } catch (...) {  // (a continuation must not take the worker down)
          }
          delete c;
        }
      }
      deliverTagged(recs, take, &v, tags, tagVerdicts);
    } catch (...) {  // (only a non-ed25519 key: the reference's releaseAssert)
      release();
      ok = false;
      for (size_t i = 0; i < take; ++i) {
        if (std::promise<bool>* p = recs[i]->done) {
          p->set_exception(std::current_exception());
          delete p;
        }
        if (std::function<void(bool)>* c = recs[i]->cb) {
          try {
            (*c)(false);
          } catch (...) {
          }
          delete c;
        }
      }
      deliverTagged(recs, take, nullptr, tags, tagVerdicts);
    }
    lk.lock();
    ++mStats.batches;
    if (bySize) ++mStats.flushedBySize;
    else if (idle) ++mStats.flushedIdle;
    else ++mStats.flushedByDeadline;
    mStats.items += take;
    mStats.maxBatchSeen = std::max<uint64_t>(mStats.maxBatchSeen, take);
    if (ok && mRecordLatency) {
      for (size_t i = 0; i < take; ++i) {
        if (mLatUs.size() < kLatencySamples) mLatUs.push_back(lat[i]);
        else mLatUs[mLatNext] = lat[i];
        mLatNext = (mLatNext + 1) % kLatencySamples;
      }
    }
    mCompleted += take;
    mDoneCv.notify_all();
  }
}

}  // namespace stellar
