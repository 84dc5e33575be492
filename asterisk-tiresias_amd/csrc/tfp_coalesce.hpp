// tfp_coalesce.hpp — one search launch for many concurrent callers (engines and device groups).
//
// The reference runs one fp_search_fingerprint_info per channel thread (application_handler.c:180)
// on one shared handle (fp_handler.c:1161-1169). Each call is a batch-1 search: ~30 us of mostly
// fixed cost (launches, a stream sync), while the batch vote does 4,096 queries in 0.36 ms. So
// concurrent callers are combined: a caller queues its request; if no batch is running it becomes
// the leader, takes every queued request that can share its search (same sample format, rate and
// parameters: the same SQL, fp_handler.c:287-374) up to kMaxQueries queries, runs them as one
// batch, hands every caller its own results and wakes them. Requests that arrive while a batch
// runs form the next batch, led by the oldest of their callers. No timer: a lone caller runs at once,
// and the batches grow with the load. Per-call results are unchanged: a query's result depends
// only on its own frames and the index ("an internal queue/batcher ... as long as
// per-call results are unchanged").
#pragma once

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/tiresias_fp.h"

namespace tfp {

// One caller's search: its queries as (host pointer, samples), and where its results go. The
// caller sleeps on its own condition variable (state: 0 queued, 1 done, 2 lead the next batch), so
// finishing a batch wakes exactly its callers and one next leader, not every waiting thread.
struct SearchReq {
  std::vector<const void*> ptrs;
  std::vector<int64_t> lens;
  bool f32 = false;
  int32_t sr = 0;
  tfp_search_params P{};
  tfp_result* out = nullptr;
  int rc = TFP_OK;
  std::string err;  // the failure's message (set on the leader's thread, noted on the caller's)
  std::mutex m;
  std::condition_variable cv;
  int state = 0;
};

// Two requests give the same SQL per query frame: tolerance < 0 is the default 0.001
// (fp_handler.c:252-256), compared bitwise otherwise (NaN stays its own class).
inline bool same_search(const SearchReq& a, const SearchReq& b) {
  if (a.f32 != b.f32 || a.sr != b.sr || a.P.coefs != b.P.coefs || a.P.freq_ignore_low != b.P.freq_ignore_low ||
      a.P.freq_ignore_high != b.P.freq_ignore_high)
    return false;
  const double ta = a.P.tolerance < 0 ? TFP_DEFAULT_TOLERANCE : a.P.tolerance;
  const double tb = b.P.tolerance < 0 ? TFP_DEFAULT_TOLERANCE : b.P.tolerance;
  return memcmp(&ta, &tb, sizeof ta) == 0;
}

class Coalescer {
 public:
  static constexpr int32_t kMaxQueries = 512;   // per combined batch
  static constexpr int32_t kMaxCallQueries = 16;  // larger calls run on their own

  // Runs *r, alone or with other callers' requests, through exec(std::vector<SearchReq*>&), which
  // sets every request's rc, results and (on failure) err; see exec_batch. Returns r->rc. An
  // exception out of exec (host allocations) fails that batch's requests; the lead always moves on.
  template <class Exec>
  int submit(SearchReq* r, Exec&& exec) {
    bool lead = false;
    try {
      std::lock_guard<std::mutex> lk(m_);
      calls_++;
      q_.push_back(r);
      if (!busy_) busy_ = lead = true;
    } catch (const std::bad_alloc&) {
      r->err = "out of host memory";
      return r->rc = TFP_E_NOMEM;
    }
    if (!lead && wait(r) == 1) return r->rc;
    // the leader: batches until its own request is done, then hands the lead to the oldest waiter
    for (;;) {
      std::vector<SearchReq*> batch;
      bool took = false;
      try {
        std::lock_guard<std::mutex> lk(m_);
        take(&batch);  // (q_ is only changed by its final swap)
        took = true;
      } catch (const std::bad_alloc&) {
      }
      if (!took) {  // no batch could be formed: this request fails alone, the lead passes on
        SearchReq* next = nullptr;
        {
          std::lock_guard<std::mutex> lk(m_);
          q_.erase(std::remove(q_.begin(), q_.end(), r), q_.end());
          if (q_.empty()) busy_ = false;
          else next = q_.front();
        }
        if (next) set_state(next, 2);
        r->err = "out of host memory";
        return r->rc = TFP_E_NOMEM;
      }
      try {
        exec(batch);
      } catch (const std::bad_alloc&) {
        for (SearchReq* b : batch) b->err = "out of host memory", b->rc = TFP_E_NOMEM;
      } catch (...) {
        for (SearchReq* b : batch) b->err = "internal error", b->rc = TFP_E_HIP;
      }
      const bool mine = std::find(batch.begin(), batch.end(), r) != batch.end();
      SearchReq* next = nullptr;
      {
        std::lock_guard<std::mutex> lk(m_);
        batches_++;
        if (q_.empty()) busy_ = false;
        else if (mine) next = q_.front();
      }
      // the next batch starts first, then this batch's callers wake (a wake-up is a few us; 25 of
      // them before the hand-off would idle the GPU for a whole batch-1 search)
      if (next) set_state(next, 2);
      for (SearchReq* b : batch)
        if (b != r) set_state(b, 1);
      if (!mine) continue;  // (its own request was not in this batch: the queue still holds it)
      return r->rc;
    }
  }

  void stats(int64_t* calls, int64_t* batches) {
    std::lock_guard<std::mutex> lk(m_);
    if (calls) *calls = calls_;
    if (batches) *batches = batches_;
  }

 private:
  // FIFO: the oldest request and every later one that shares its search, up to kMaxQueries
  void take(std::vector<SearchReq*>* batch) {
    SearchReq* first = q_.front();
    size_t n = 0;
    std::vector<SearchReq*> rest;
    for (SearchReq* r : q_) {
      if (same_search(*first, *r) && (batch->empty() || n + r->lens.size() <= (size_t)kMaxQueries)) {
        batch->push_back(r);
        n += r->lens.size();
      } else {
        rest.push_back(r);
      }
    }
    q_.swap(rest);
  }

  static int wait(SearchReq* r) {
    std::unique_lock<std::mutex> lk(r->m);
    r->cv.wait(lk, [r] { return r->state != 0; });
    return r->state;
  }
  static void set_state(SearchReq* r, int st) {
    std::lock_guard<std::mutex> lk(r->m);
    r->state = st;
    r->cv.notify_one();
  }

  std::mutex m_;
  std::vector<SearchReq*> q_;
  bool busy_ = false;
  int64_t calls_ = 0, batches_ = 0;
};

// A batch's queries end to end, and each request's results back from the combined array.
struct Combined {
  std::vector<const void*> ptrs;
  std::vector<int64_t> lens;
  std::vector<tfp_result> res;
  explicit Combined(const std::vector<SearchReq*>& batch) {
    for (const SearchReq* b : batch) {
      ptrs.insert(ptrs.end(), b->ptrs.begin(), b->ptrs.end());
      lens.insert(lens.end(), b->lens.begin(), b->lens.end());
    }
    res.resize(std::max<size_t>(lens.size(), 1));
  }
  void scatter(const std::vector<SearchReq*>& batch) {
    size_t at = 0;
    for (SearchReq* b : batch) {
      b->rc = TFP_OK;
      memcpy(b->out, res.data() + at, sizeof(tfp_result) * b->lens.size());
      at += b->lens.size();
    }
  }
};

// A coalesced batch through run(ptrs, lens, nq, f32, sr, P, out) -> rc (the handle's uncoalesced
// search); last_error() reads the message of run's failure on this (the leader's) thread. When the
// combined batch fails for want of memory (TFP_E_NOMEM: a device or host allocation sized for all
// of it, or one caller's query whose own allocation fails), every request is run again alone, so
// only a request that fails by itself reports an error, with its own message, and the others get
// their results. Any other failure (a kernel fault, a launch error: a device that is now broken) is
// not re-run N more times: every request of the batch gets the leader's code and message.
template <class Run, class LastError>
void exec_batch(std::vector<SearchReq*>& batch, Run&& run, LastError&& last_error) {
  auto alone = [&](SearchReq* b) {
    b->rc = run(b->ptrs.data(), b->lens.data(), (int32_t)b->lens.size(), b->f32, b->sr, &b->P, b->out);
    if (b->rc) b->err = last_error();
  };
  if (batch.size() == 1) {
    alone(batch[0]);
    return;
  }
  Combined c(batch);
  const SearchReq* b0 = batch[0];
  const int rc = run(c.ptrs.data(), c.lens.data(), (int32_t)c.lens.size(), b0->f32, b0->sr, &b0->P, c.res.data());
  if (rc == TFP_OK) {
    c.scatter(batch);
    return;
  }
  if (rc == TFP_E_NOMEM) {
    for (SearchReq* b : batch) alone(b);
    return;
  }
  const std::string msg = last_error();
  for (SearchReq* b : batch) {
    b->rc = rc;
    b->err = msg;
  }
}

}  // namespace tfp
