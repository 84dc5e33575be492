// TEST HARNESS (tests/test_sanitizers.py; not product code): the engine's host-side thread hand-offs
// under ThreadSanitizer, on the CPU, with no GPU calls:
//   - tfp::ShardPool (csrc/tfp_shardpool.hpp): the device group's fan-out, run() from one caller at a
//     time as tfp_group does under its mutex, with short and long (blocking) shard functions, so
//     both the spin and the condition-variable hand-offs are taken;
//   - tfp::Coalescer (csrc/tfp_coalesce.hpp): many threads submitting searches at once, the leader
//     running a combined batch (tfp::exec_batch) and handing each caller its own results; some
//     callers' requests fail, so failed combined batches are re-run request by request and each
//     failing caller gets its own message through the real per-thread error slots
//     (csrc/tfp_internal.hpp: tfp::ErrorSlot), read concurrently by every caller;
//   - a shard function that throws (std::bad_alloc) becomes that shard's TFP_E_NOMEM.
// Every result is checked; TSan (halt_on_error=1) turns any data race into a failing exit code.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include "../../asterisk-tiresias_amd/csrc/tfp_coalesce.hpp"
#include "../../asterisk-tiresias_amd/csrc/tfp_internal.hpp"
#include "../../asterisk-tiresias_amd/csrc/tfp_shardpool.hpp"

static int fails = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
      fails++;                                                        \
    }                                                                 \
  } while (0)

static void pool_test(int shards, int rounds) {
  tfp::ShardPool pool(shards);
  std::vector<int64_t> acc(shards, 0);  // each shard's slot, written by its own worker only
  std::mutex caller;                     // tfp_group's mutex: one run() at a time
  auto caller_thread = [&](int t) {
    for (int r = 0; r < rounds; r++) {
      std::lock_guard<std::mutex> lk(caller);
      const int64_t add = t * 1000 + r;
      const bool slow = (r % 17) == 0;  // past the spin: the blocking hand-off
      int bad = -1;
      const int rc = pool.run(
          [&](int s) {
            if (slow) std::this_thread::sleep_for(std::chrono::microseconds(200));
            acc[s] += add;
            if (r % 31 == 7 && s == 0) throw std::bad_alloc();  // (after its add: counted below)
            return (r % 29 == 5 && s == shards - 1) ? -2 : 0;
          },
          &bad);
      if (r % 31 == 7) CHECK(rc == TFP_E_NOMEM && bad == 0);
      else if (r % 29 == 5) CHECK(rc == -2 && bad == shards - 1);
      else CHECK(rc == 0);
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < 4; t++) th.emplace_back(caller_thread, t);
  for (auto& x : th) x.join();
  int64_t want = 0;
  for (int t = 0; t < 4; t++)
    for (int r = 0; r < rounds; r++) want += t * 1000 + r;
  for (int s = 0; s < shards; s++) CHECK(acc[s] == want);
}

// A fake search: query i's "result" is a function of its samples, so a caller that got another
// caller's slice would see it.
static void coalesce_test(int nthreads, int reps) {
  tfp::Coalescer coal;
  std::atomic<int64_t> exec_queries{0};
  std::vector<std::vector<int16_t>> data(nthreads);
  for (int t = 0; t < nthreads; t++) {
    data[t].resize(64 + t);
    for (size_t i = 0; i < data[t].size(); i++) data[t][i] = (int16_t)(t * 31 + i);
  }
  // the handle's uncoalesced search: fails for want of memory (a message naming the query's
  // length) when any query has a poisoned length, as a device allocation for it would
  tfp::ErrorSlot slot;
  auto run = [&](const void* const* ptrs, const int64_t* lens, int32_t nq, bool, int32_t, const tfp_search_params*,
                 tfp_result* out) {
    for (int32_t q = 0; q < nq; q++)
      if (lens[q] % 7 == 3) {
        char m[64];
        snprintf(m, sizeof m, "poisoned query of %lld samples", (long long)lens[q]);
        slot.note(&slot, m);
        return TFP_E_NOMEM;
      }
    for (int32_t q = 0; q < nq; q++) {
      const int16_t* x = static_cast<const int16_t*>(ptrs[q]);
      int64_t sum = 0;
      for (int64_t i = 0; i < lens[q]; i++) sum += x[i];
      memset(&out[q], 0, sizeof out[q]);
      out[q].found = 1;
      out[q].match_count = (int32_t)sum;
      out[q].frame_count = (int32_t)lens[q];
    }
    exec_queries += nq;
    if (nq > 1) std::this_thread::sleep_for(std::chrono::microseconds(50));
    return TFP_OK;
  };
  auto exec = [&](std::vector<tfp::SearchReq*>& batch) {
    tfp::exec_batch(batch, run, [&] { return std::string(slot.read(&slot)); });
  };
  auto caller = [&](int t) {
    for (int r = 0; r < reps; r++) {
      tfp::SearchReq req;
      const int nq = 1 + (t + r) % 3;
      for (int q = 0; q < nq; q++) {
        req.ptrs.push_back(data[(t + q) % nthreads].data());
        req.lens.push_back((int64_t)data[(t + q) % nthreads].size());
      }
      req.sr = 8000;
      req.P.coefs = 1 + (r % 2);  // two parameter sets: batches never mix them
      req.P.tolerance = -1.0;
      std::vector<tfp_result> out(nq);
      req.out = out.data();
      const int rc = coal.submit(&req, exec);
      bool poisoned = false;
      for (int q = 0; q < nq; q++) poisoned = poisoned || req.lens[q] % 7 == 3;
      if (poisoned) {  // this caller alone fails, with the message of its own request
        CHECK(rc == TFP_E_NOMEM);
        if (rc) slot.note(&slot, req.err.c_str());
        const char* m = slot.read(&slot);
        bool mine = false;
        for (int q = 0; q < nq; q++) {
          char want[64];
          snprintf(want, sizeof want, "poisoned query of %lld samples", (long long)req.lens[q]);
          mine = mine || strcmp(m, want) == 0;
        }
        CHECK(mine);
        continue;
      }
      CHECK(rc == 0);
      for (int q = 0; q < nq; q++) {
        const auto& d = data[(t + q) % nthreads];
        int64_t sum = 0;
        for (int16_t v : d) sum += v;
        CHECK(out[q].found == 1 && out[q].match_count == (int32_t)sum && out[q].frame_count == (int32_t)d.size());
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; t++) th.emplace_back(caller, t);
  for (auto& x : th) x.join();
  int64_t calls = 0, batches = 0, want = 0;
  coal.stats(&calls, &batches);
  for (int t = 0; t < nthreads; t++)
    for (int r = 0; r < reps; r++) {
      bool poisoned = false;
      for (int q = 0; q < 1 + (t + r) % 3; q++) poisoned = poisoned || (64 + (t + q) % nthreads) % 7 == 3;
      if (!poisoned) want += 1 + (t + r) % 3;
    }
  CHECK(calls == (int64_t)nthreads * reps);
  CHECK(exec_queries.load() >= want);  // (the good requests, some more than once after a failed batch)
  CHECK(batches >= 1 && batches <= calls);
  printf("coalescer: %lld calls in %lld batches\n", (long long)calls, (long long)batches);
}

// A combined batch that fails for another reason than memory (a kernel fault, a launch error) is not
// re-run request by request: every request gets the leader's code and message, and the run is
// called once.
static void sticky_failure_test() {
  tfp::ErrorSlot slot;
  int runs = 0;
  auto run = [&](const void* const*, const int64_t*, int32_t nq, bool, int32_t, const tfp_search_params*, tfp_result*) {
    runs++;
    if (nq > 1) {
      slot.note(&slot, "device fault");
      return TFP_E_HIP;
    }
    return TFP_OK;
  };
  std::vector<int16_t> x(300, 1);
  std::vector<tfp::SearchReq> reqs(3);
  std::vector<tfp_result> out(3);
  std::vector<tfp::SearchReq*> batch;
  for (int i = 0; i < 3; i++) {
    reqs[i].ptrs.push_back(x.data());
    reqs[i].lens.push_back(300);
    reqs[i].sr = 8000;
    reqs[i].P.coefs = 1;
    reqs[i].out = &out[i];
    batch.push_back(&reqs[i]);
  }
  tfp::exec_batch(batch, run, [&] { return std::string(slot.read(&slot)); });
  CHECK(runs == 1);
  for (auto& r : reqs) CHECK(r.rc == TFP_E_HIP && r.err == "device fault");
  printf("sticky failure: one run, every request failed\n");
}

int main() {
  sticky_failure_test();
  pool_test(3, 400);
  pool_test(8, 200);
  coalesce_test(32, 40);
  coalesce_test(64, 10);
  if (fails) {
    fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  printf("ok\n");
  return 0;
}
