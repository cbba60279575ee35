// See VerifyMicroBatcher.h.
#include "VerifyMicroBatcher.h"

#include <algorithm>
#include <cstring>
#include <exception>

namespace stellar {

VerifyMicroBatcher::VerifyMicroBatcher(size_t maxBatch, std::chrono::microseconds maxDelay, unsigned workers,
                                       bool recordLatency)
    : mMaxBatch(std::max<size_t>(1, maxBatch)), mMaxDelay(maxDelay), mRecordLatency(recordLatency) {
  mQ.recs.reserve(mMaxBatch);
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

void VerifyMicroBatcher::enqueue(PublicKey const& key, ByteSlice const& sig, ByteSlice const& msg,
                                 std::promise<bool>* done) {
  Rec r;
  r.key = key;
  // a signature longer than 64 bytes is not an XDR Signature; anything but 64
  // is rejected by verifySig before verification, so keep at most 64 bytes
  // and the real size
  r.sigLen = (uint32_t)std::min<size_t>(sig.size(), 65);
  std::memcpy(r.sig, sig.data(), std::min<size_t>(sig.size(), 64));
  r.msgLen = (uint32_t)msg.size();
  r.done = done;
  if (mRecordLatency) r.t0 = Clock::now();
  bool wake;
  {
    std::lock_guard<std::mutex> g(mMu);
    if (mQ.recs.empty()) mOldest = mRecordLatency ? r.t0 : Clock::now();
    r.msgOff = mQ.arena.size();
    mQ.arena.insert(mQ.arena.end(), msg.begin(), msg.end());
    mQ.recs.push_back(r);
    ++mStats.items;
    ++mEnqueued;
    wake = mQ.recs.size() == 1 || mQ.recs.size() == mMaxBatch;
  }
  if (wake) mCv.notify_one();
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
  const uint64_t target = mEnqueued;
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

void VerifyMicroBatcher::run() {
  std::unique_lock<std::mutex> lk(mMu);
  Queue batch;
  std::vector<PubKeyUtils::VerifyItem> items;
  std::vector<double> lat;
  for (;;) {
    // wait for: stop, a full batch, or the oldest item's deadline
    while (!mStop && mQ.recs.empty()) mCv.wait(lk);
    if (mQ.recs.empty()) return;  // stop requested and the queue is drained
    if (mQ.recs.size() < mMaxBatch && !mStop) {
      const auto deadline = mOldest + mMaxDelay;
      if (Clock::now() < deadline) {
        mCv.wait_until(lk, deadline, [&] { return mStop || mQ.recs.size() >= mMaxBatch; });
        continue;  // re-evaluate: another worker may have taken the queue meanwhile
      }
    }
    const bool bySize = mQ.recs.size() >= mMaxBatch;
    batch.recs.clear();
    batch.arena.clear();
    if (mQ.recs.size() <= mMaxBatch) {
      std::swap(batch, mQ);  // the whole queue, no copy
    } else {
      // the oldest maxBatch items; the rest stay queued (offsets rebased)
      const uint64_t cut = mQ.recs[mMaxBatch].msgOff;
      batch.recs.assign(mQ.recs.begin(), mQ.recs.begin() + mMaxBatch);
      batch.arena.assign(mQ.arena.begin(), mQ.arena.begin() + cut);
      mQ.recs.erase(mQ.recs.begin(), mQ.recs.begin() + mMaxBatch);
      mQ.arena.erase(mQ.arena.begin(), mQ.arena.begin() + cut);
      for (Rec& r : mQ.recs) r.msgOff -= cut;
      mOldest = Clock::now();  // (the remaining items arrived no earlier than the flush decision)
      mCv.notify_one();        // leftovers: another worker can take them
    }
    const size_t take = batch.recs.size();
    ++mStats.batches;
    if (bySize) ++mStats.flushedBySize;
    else ++mStats.flushedByDeadline;
    mStats.maxBatchSeen = std::max<uint64_t>(mStats.maxBatchSeen, take);
    lk.unlock();
    items.resize(take);
    const uint8_t* arena = batch.arena.data();
    for (size_t i = 0; i < take; ++i) {
      Rec const& r = batch.recs[i];
      items[i] = PubKeyUtils::VerifyItem{&r.key, ByteSlice(r.sig, r.sigLen), ByteSlice(arena + r.msgOff, r.msgLen)};
    }
    bool ok = true;
    try {
      std::vector<bool> v = PubKeyUtils::verifySigBatch(items);
      if (mRecordLatency) {
        const auto now = Clock::now();
        lat.resize(take);
        for (size_t i = 0; i < take; ++i)
          lat[i] = std::chrono::duration<double, std::micro>(now - batch.recs[i].t0).count();
      }
      for (size_t i = 0; i < take; ++i)
        if (std::promise<bool>* p = batch.recs[i].done) {
          p->set_value(v[i]);
          delete p;
        }
    } catch (...) {  // (only a non-ed25519 key: the reference's releaseAssert)
      ok = false;
      for (size_t i = 0; i < take; ++i)
        if (std::promise<bool>* p = batch.recs[i].done) {
          p->set_exception(std::current_exception());
          delete p;
        }
    }
    lk.lock();
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
