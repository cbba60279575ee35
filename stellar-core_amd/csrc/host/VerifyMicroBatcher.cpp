// See VerifyMicroBatcher.h.
#include "VerifyMicroBatcher.h"

#include <algorithm>
#include <exception>

namespace stellar {

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

void VerifyMicroBatcher::enqueue(Item&& it) {
  bool wake;
  {
    std::lock_guard<std::mutex> g(mMu);
    mQueue.push_back(std::move(it));
    ++mStats.items;
    ++mEnqueued;
    wake = mQueue.size() == 1 || mQueue.size() >= mMaxBatch;
  }
  if (wake) mCv.notify_one();
}

std::future<bool> VerifyMicroBatcher::submit(PublicKey const& key, Signature const& sig, ByteSlice const& msg) {
  Item it;
  it.key = key;
  it.sig = sig;
  it.msg.assign(msg.begin(), msg.end());
  it.done = std::make_unique<std::promise<bool>>();
  it.t0 = std::chrono::steady_clock::now();
  std::future<bool> f = it.done->get_future();
  enqueue(std::move(it));
  return f;
}

void VerifyMicroBatcher::post(PublicKey const& key, Signature const& sig, ByteSlice const& msg) {
  Item it;
  it.key = key;
  it.sig = sig;
  it.msg.assign(msg.begin(), msg.end());
  it.t0 = std::chrono::steady_clock::now();
  enqueue(std::move(it));
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
  std::vector<Item> batch;
  std::vector<PubKeyUtils::VerifyItem> items;
  std::vector<double> lat;
  for (;;) {
    // wait for: stop, a full batch, or the oldest item's deadline
    while (!mStop && mQueue.empty()) mCv.wait(lk);
    if (mQueue.empty()) return;  // stop requested and the queue is drained
    if (mQueue.size() < mMaxBatch && !mStop) {
      const auto deadline = mQueue.front().t0 + mMaxDelay;
      if (std::chrono::steady_clock::now() < deadline) {
        mCv.wait_until(lk, deadline, [&] { return mStop || mQueue.size() >= mMaxBatch; });
        continue;  // re-evaluate: another worker may have taken the queue meanwhile
      }
    }
    const bool bySize = mQueue.size() >= mMaxBatch;
    const size_t take = std::min(mQueue.size(), mMaxBatch);
    batch.clear();
    batch.reserve(take);
    for (size_t i = 0; i < take; ++i) {
      batch.push_back(std::move(mQueue.front()));
      mQueue.pop_front();
    }
    ++mStats.batches;
    if (bySize) ++mStats.flushedBySize;
    else ++mStats.flushedByDeadline;
    mStats.maxBatchSeen = std::max<uint64_t>(mStats.maxBatchSeen, take);
    if (!mQueue.empty()) mCv.notify_one();  // leftovers: another worker can take them
    lk.unlock();
    items.clear();
    items.reserve(take);
    for (auto& b : batch) items.push_back(PubKeyUtils::VerifyItem{&b.key, &b.sig, ByteSlice(b.msg)});
    bool ok = true;
    try {
      std::vector<bool> v = PubKeyUtils::verifySigBatch(items);
      const auto now = std::chrono::steady_clock::now();
      if (mRecordLatency) {
        lat.resize(take);
        for (size_t i = 0; i < take; ++i) lat[i] = std::chrono::duration<double, std::micro>(now - batch[i].t0).count();
      }
      for (size_t i = 0; i < take; ++i)
        if (batch[i].done) batch[i].done->set_value(v[i]);
    } catch (...) {  // (only a non-ed25519 key: the reference's releaseAssert)
      ok = false;
      for (auto& b : batch)
        if (b.done) b.done->set_exception(std::current_exception());
    }
    batch.clear();
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
