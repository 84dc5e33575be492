// TEST HARNESS (tests/test_sanitizers.py; not product code): the engine's host-side thread hand-offs
// under ThreadSanitizer, on the CPU, with no GPU calls:
//   - tfp::ShardPool (csrc/tfp_shardpool.hpp): the device group's fan-out, run() from one caller at a
//     time as tfp_group does under its mutex, with short and long (blocking) shard functions, so
//     both the spin and the condition-variable hand-offs are taken;
//   - tfp::Coalescer (csrc/tfp_coalesce.hpp): many threads submitting searches at once, the leader
//     running a combined batch and handing each caller its own results.
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
            return (r % 29 == 5 && s == shards - 1) ? -2 : 0;
          },
          &bad);
      if (r % 29 == 5) CHECK(rc == -2 && bad == shards - 1);
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
  auto exec = [&](std::vector<tfp::SearchReq*>& batch) {
    tfp::Combined c(batch);
    for (size_t q = 0; q < c.lens.size(); q++) {
      const int16_t* x = static_cast<const int16_t*>(c.ptrs[q]);
      int64_t sum = 0;
      for (int64_t i = 0; i < c.lens[q]; i++) sum += x[i];
      memset(&c.res[q], 0, sizeof c.res[q]);
      c.res[q].found = 1;
      c.res[q].match_count = (int32_t)sum;
      c.res[q].frame_count = (int32_t)c.lens[q];
    }
    exec_queries += (int64_t)c.lens.size();
    if (batch.size() > 1) std::this_thread::sleep_for(std::chrono::microseconds(50));
    c.scatter(batch, 0);
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
    for (int r = 0; r < reps; r++) want += 1 + (t + r) % 3;
  CHECK(calls == (int64_t)nthreads * reps);
  CHECK(exec_queries.load() == want);
  CHECK(batches >= 1 && batches <= calls);
  printf("coalescer: %lld calls in %lld batches\n", (long long)calls, (long long)batches);
}

int main() {
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
