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

VerifyMicroBatcher::VerifyMicroBatcher(size_t maxBatch, std::chrono::microseconds maxDelay, unsigned workers,
                                       bool recordLatency)
    : mMaxBatch(std::max<size_t>(1, maxBatch)), mMaxDelay(maxDelay), mRecordLatency(recordLatency) {
  const unsigned w = std::max(1u, workers);
  mWorkers.reserve(w);
  for (unsigned i = 0; i < w; ++i) mWorkers.emplace_back([this] { run(); });
}

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
                                 std::promise<bool>* done) {
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
  if (mRecordLatency) r.t0 = Clock::now();
  r.arrivalNs = nowNs();
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
    if (q == 1) mOldestNs.store(r.arrivalNs);
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
  enqueue(key, sig, msg, p);
  return f;
}

void VerifyMicroBatcher::post(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg) {
  enqueue(key, sig, msg, nullptr);
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

void VerifyMicroBatcher::run() {
  std::vector<Queue> parts(kShards);
  std::vector<PubKeyUtils::VerifyItem> items;
  std::vector<Rec const*> recs;
  std::vector<double> lat;
  size_t start = 0;
  std::unique_lock<std::mutex> lk(mMu);
  for (;;) {
    // wait for: stop, a full batch, or the oldest item's deadline
    while (!mStop && mQueued.load() == 0) mCv.wait(lk);
    if (mQueued.load() == 0) return;  // stop requested and every queue drained
    if (mQueued.load() < mMaxBatch && !mStop) {
      const int64_t deadline = mOldestNs.load() + (int64_t)mMaxDelay.count() * 1000;
      const int64_t now = nowNs();
      if (now < deadline) {
        mCv.wait_for(lk, std::chrono::nanoseconds(deadline - now),
                     [&] { return mStop || mQueued.load() >= mMaxBatch; });
        continue;  // re-evaluate: another worker may have taken the queue meanwhile
      }
    }
    const bool bySize = mQueued.load() >= mMaxBatch;
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
    if (left > 0) {
      // the leftovers keep their own deadline: the oldest one's arrival
      const int64_t oldest = oldestQueuedNs();
      if (oldest != INT64_MAX) mOldestNs.store(oldest);
      if (left >= mMaxBatch) wake();
    }
    if (take == 0) {
      lk.lock();
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
    try {
      std::vector<bool> v = PubKeyUtils::verifySigBatch(items);
      if (mRecordLatency) {
        const auto now = Clock::now();
        lat.resize(take);
        for (size_t i = 0; i < take; ++i) lat[i] = std::chrono::duration<double, std::micro>(now - recs[i]->t0).count();
      }
      for (size_t i = 0; i < take; ++i)
        if (std::promise<bool>* p = recs[i]->done) {
          p->set_value(v[i]);
          delete p;
        }
    } catch (...) {  // (only a non-ed25519 key: the reference's releaseAssert)
      ok = false;
      for (size_t i = 0; i < take; ++i)
        if (std::promise<bool>* p = recs[i]->done) {
          p->set_exception(std::current_exception());
          delete p;
        }
    }
    lk.lock();
    ++mStats.batches;
    if (bySize) ++mStats.flushedBySize;
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
