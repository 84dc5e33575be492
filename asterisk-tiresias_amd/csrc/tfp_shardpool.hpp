// tfp_shardpool.hpp — the device group's fan-out (csrc/tfp_group.cpp): f(s) for every shard s
// in parallel, one worker thread per shard but the first (which runs on the caller).
// Header-only so tests/native/tsan_threads.cpp can drive it under ThreadSanitizer on the CPU.
#pragma once

#include <stdint.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/tiresias_fp.h"

namespace tfp {

// One worker thread per shard but the first (which runs on the caller); run() executes f(s) for
// every shard in parallel and returns when all are done. A batch-1 search is ~30 us of GPU work
// per shard, so the hand-off must cost less than a thread wake-up (~10-50 us through a futex):
// workers and the caller spin on atomics for a short while (kSpinNs) before they block, and the
// blocking side uses the mutex + condition variables (no lost wake-ups: the generation is bumped
// under the mutex, and the predicates are checked under it).
class ShardPool {
 public:
  explicit ShardPool(int n) : n_(n), rc_(n, 0) {
    for (int s = 1; s < n; s++) th_.emplace_back([this, s] { loop(s); });
  }
  ~ShardPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_.store(true, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // first nonzero return code (shard order), its shard in *bad
  int run(const std::function<int(int)>& f, int* bad = nullptr) {
    f_ = &f;
    pending_.store(n_ - 1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(m_);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    rc_[0] = call(f, 0);
    if (!spin_until([&] { return pending_.load(std::memory_order_acquire) == 0; })) {
      std::unique_lock<std::mutex> lk(m_);
      done_.wait(lk, [this] { return pending_.load(std::memory_order_acquire) == 0; });
    }
    f_ = nullptr;
    for (int s = 0; s < n_; s++)
      if (rc_[s]) {
        if (bad) *bad = s;
        return rc_[s];
      }
    return TFP_OK;
  }

 private:
  static constexpr int64_t kSpinNs = 50000;
  // f(s), with an exception (an allocation inside a shard's call) as that shard's error code: a
  // throw on a worker thread would otherwise end the process, and one on the caller would leave
  // the workers running f after run() unwound
  static int call(const std::function<int(int)>& f, int s) {
    try {
      return f(s);
    } catch (const std::bad_alloc&) {
      return TFP_E_NOMEM;
    } catch (...) {
      return TFP_E_HIP;
    }
  }
  template <class P>
  static bool spin_until(P ready) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0;; i++) {
      if (ready()) return true;
      if ((i & 63) == 63 &&
          std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() > kSpinNs)
        return false;
      __builtin_ia32_pause();
    }
  }
  void loop(int s) {
    uint64_t seen = 0;
    for (;;) {
      auto fresh = [&] { return stop_.load(std::memory_order_acquire) || gen_.load(std::memory_order_acquire) != seen; };
      if (!spin_until(fresh)) {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, fresh);
      }
      if (stop_.load(std::memory_order_acquire)) return;
      seen = gen_.load(std::memory_order_acquire);
      rc_[s] = call(*f_, s);
      if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        std::lock_guard<std::mutex> lk(m_);
        done_.notify_one();
      }
    }
  }
  int n_;
  std::vector<int> rc_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<int(int)>* f_ = nullptr;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> pending_{0};
  std::atomic<bool> stop_{false};
};

}  // namespace tfp
