// Persistent helper-thread pool shared by the engine's host side (staging,
// multi-slot fan-out: sv_api.cpp) and the C++ mirror (parallel hashing and
// CPU-path batches: host/).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace sv {

// Persistent host threads for packing staging buffers and for driving several
// device slots at once.  run(k, fn) executes fn(0..k-1); the calling thread
// takes part and, while waiting, keeps executing queued tasks, so nested use
// (a device slice that packs in parallel) cannot deadlock.
class Pool {
 public:
  // init (optional) runs first on every helper thread (a device slot's
  // workers pin themselves to the GPU's NUMA node there: sv_api.cpp)
  explicit Pool(unsigned threads, const std::function<void()>& init = {}) {
    for (unsigned i = 0; i < threads; ++i)
      th_.emplace_back([this, init] {
        if (init) init();
        loop();
      });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  size_t size() const { return th_.size(); }
  // Queues fn on a helper thread and returns at once (the caller tracks its
  // completion itself); with no helper threads fn runs here.
  void post(std::function<void()> fn) {
    if (th_.empty()) {
      fn();
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.emplace_back(std::move(fn));
    }
    cv_.notify_one();
  }
  void run(size_t k, const std::function<void(size_t)>& fn) {
    if (k == 0) return;
    if (k == 1 || th_.empty()) {
      for (size_t i = 0; i < k; ++i) fn(i);
      return;
    }
    // The group is shared with the helpers (heap, reference-counted): a
    // helper's last touch of it -- decrement and notify under grp->mu --
    // can never reach memory this call has already released, and run()
    // returns only after seeing zero under grp->mu, i.e. after every fn(i).
    // (An earlier stack-allocated group let run() return while a helper was
    // still to lock its mutex; the helper then slept forever on dead stack
    // memory and ~Pool's join hung process exit.)
    struct Group {
      size_t left;
      std::mutex mu;
      std::condition_variable cv;
    };
    auto grp = std::make_shared<Group>();
    grp->left = k - 1;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t i = 1; i < k; ++i)
        q_.emplace_back([grp, &fn, i] {
          fn(i);
          std::lock_guard<std::mutex> gg(grp->mu);
          if (--grp->left == 0) grp->cv.notify_all();
        });
    }
    cv_.notify_all();
    fn(0);
    for (;;) {
      std::function<void()> task;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (!q_.empty()) {
          task = std::move(q_.front());
          q_.pop_front();
        }
      }
      if (task) {
        task();
        continue;
      }
      // (a bounded wait, so tasks queued meanwhile -- nested run() calls --
      // are picked up; system_clock: libstdc++ then uses the timed wait that
      // ThreadSanitizer models, tests of this pool run under it clean)
      std::unique_lock<std::mutex> lk(grp->mu);
      if (grp->cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::microseconds(200),
                             [&] { return grp->left == 0; }))
        return;
    }
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;
      auto task = std::move(q_.front());
      q_.pop_front();
      lk.unlock();
      task();
      lk.lock();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
};

}  // namespace sv
