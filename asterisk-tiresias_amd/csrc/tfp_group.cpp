// tfp_group.cpp — several engines (one per GPU of the node) behind one index and one search
// (include/tiresias_fp.h, "device groups").
//
// The reference's fp_search_fingerprint_info is one SQL pipeline over the whole audio_fingerprint
// table (fp_handler.c:287-374). Here the enrolled clips are sharded over the engines — a clip is
// never split, because the per-frame GROUP BY audio_uuid (:353) is not additive over a split clip —
// and every search runs on all shards in parallel, one worker thread per engine. Each shard's
// per-query winner is the key (count << 32 | global uuid rank): the engines carry the group-wide
// uuid ranks as their tie-break keys (tfp_index_set_tiebreak), so the greatest key over the shards
// is the reference's winner (count(*) DESC, ties to the greatest audio_uuid, :367-374) and the
// combine is an integer max on the host (the results leave the GPUs for the caller anyway).
//
// Batches of host PCM large enough to be throughput-bound are query-sharded: shard s fingerprints
// queries [s·nq/N, (s+1)·nq/N) on its GPU, the frame values are exchanged device to device
// (hipMemcpyPeerAsync over xGMI; a plain device copy when a device repeats), and every shard
// searches the whole batch against its clips (tfp_search_q_device). Smaller batches (batch-1
// latency) are fingerprinted by every shard itself: no exchange on the latency path. Stream
// channels are split over the shards (channel c on shard c mod N): each shard keeps its channels'
// rings and fingerprints their full windows, the windows' frame values are exchanged as for a
// query-sharded batch, and every shard matches all of them against its clips. (TFP_GROUP_STREAM=
// replicate: every shard runs every channel, no exchange; the round-3 form.)
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/tiresias_fp.h"
#include "tfp_coalesce.hpp"
#include "tfp_internal.hpp"
#include "tfp_kernels.hpp"
#include "tfp_shardpool.hpp"

namespace {

struct Member {
  std::string uuid;
  int32_t shard;
  int32_t id;        // the engine's clip id
  int32_t key = -1;  // its tie-break key (ordered like the uuids, sparse; -1 until assigned)
};

// Device buffers of the query-sharded batch path, one set per shard.
struct ShardBufs {
  void* pcm = nullptr;      // this shard's queries (int16)
  void* micro = nullptr;    // their stored values (unused by the search, written by the kernel)
  void* q = nullptr;        // the whole batch's frame values (2 doubles per frame)
  void* keys = nullptr;     // per-query keys
  void* sfp = nullptr;      // split streams: this shard's channels' window values of the tick
  size_t b_pcm = 0, b_micro = 0, b_q = 0, b_keys = 0, b_sfp = 0;
  hipStream_t stream = nullptr;
  hipEvent_t fp_done = nullptr;
  tfp_plan* plan = nullptr;  // this shard's share of the last batch shape (k queries of qn samples)
  int64_t plan_k = -1, plan_qn = -1;
  int32_t plan_sr = 0;
};

hipError_t grow(void** p, size_t* have, size_t want) {
  if (want <= *have) return hipSuccess;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *have = 0;
  hipError_t e = hipMalloc(p, want);
  if (e == hipSuccess) *have = want;
  return e;
}

}  // namespace

struct tfp_group {
  std::vector<tfp_engine*> eng;
  std::vector<int32_t> dev;
  tfp::ShardPool* pool = nullptr;
  std::recursive_mutex mu;
  tfp::ErrorSlot err;  // last-error messages (tfp_internal.hpp)
  std::unordered_map<std::string, int32_t> where;     // uuid -> index in members
  std::vector<Member> members;                         // every clip ever added (uuid "" once removed)
  std::vector<std::vector<int32_t>> id2member;         // [shard][engine clip id] -> member index (-1 removed)
  std::vector<int64_t> rows;                           // live rows per shard (placement)
  std::vector<int32_t> by_uuid;                        // live members in uuid order (global ranks)
  // Tie-break keys (round 6): every live member's key orders like its uuid with gaps between
  // neighbours, so a new clip takes the middle of its neighbours' gap and no other key changes; the
  // shards then get the new clips' keys only (tfp_index_update_tiebreak), an enrolment stays
  // O(new clips). A gap of 1 (or a large batch) respaces every key evenly over [0, 2^31) instead.
  std::unordered_map<int32_t, int32_t> key2member;     // key -> member
  std::vector<size_t> pushed;                          // per shard: engine clip ids whose keys it has
  bool keys_full = true;                               // respace every key and send every shard all its keys
  bool ranks_dirty = true;                             // some shard lacks keys (keys_full or new clip ids)
  int64_t n_respaces = 0, n_partial_pushes = 0;        // full key refreshes / new-clip-only pushes
  std::vector<ShardBufs> bufs;
  tfp::Coalescer coal;   // concurrent channel searches share one batch per shard (tfp_coalesce.hpp)
  bool coalesce = true;  // TFP_COALESCE=0: every call alone
  // ordered pairs of distinct devices; of them, peer-accessible; of those, peer access enabled
  // (tfp_group_peer_stats: the 8-GPU bench line reports them)
  int32_t peer_pairs = 0, peer_can = 0, peer_enabled = 0;
  ~tfp_group() {
    delete pool;
    for (size_t s = 0; s < bufs.size(); s++) {
      (void)hipSetDevice(dev[s]);
      for (void* p : {bufs[s].pcm, bufs[s].micro, bufs[s].q, bufs[s].keys, bufs[s].sfp})
        if (p) (void)hipFree(p);
      if (bufs[s].fp_done) (void)hipEventDestroy(bufs[s].fp_done);
      tfp_plan_destroy(bufs[s].plan);
      if (bufs[s].stream) (void)hipStreamDestroy(bufs[s].stream);
    }
    for (auto* e : eng) tfp_engine_destroy(e);
  }
};

struct tfp_group_stream {
  tfp_group* g = nullptr;
  std::vector<tfp_stream*> st;  // one per shard: every channel (replicated) or its own (split; null if none)
  int32_t nch = 0;
  int64_t W = 0;
  bool split = false;
  std::vector<std::vector<int32_t>> chans;  // split: shard -> its channels (c mod N == s), ascending
  std::vector<std::vector<int16_t>> tick;   // split: the shard's rows of the tick
  std::vector<std::vector<int32_t>> act;    // split: the shard's windows of the tick (local channel indices)
  std::vector<int32_t> nact;
  std::vector<std::vector<unsigned long long>> keys;
  std::vector<std::vector<tfp_result>> res;
};

namespace {

int gfail(tfp_group* g, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int gfail(tfp_group* g, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (g) g->err.note(g, buf);
  return code;
}

// The error of shard s's failed call made on this thread, into the group's message.
int shard_fail(tfp_group* g, int rc, int s) {
  return gfail(g, rc, "shard %d (device %d): %s", s, g->dev[s], tfp_engine_last_error(g->eng[s]));
}

// f(s) on every shard in parallel; a failure becomes the group's error with the failing shard's
// message, read on the thread that ran that shard's call (the engine's per-thread slot).
int run_all(tfp_group* g, const std::function<int(int)>& f) {
  const int n = (int)g->eng.size();
  std::vector<std::string> why(n);
  int bad = 0;
  const int rc = g->pool->run(
      [&](int s) {
        tfp_internal_engine_clear_error(g->eng[s]);
        g->err.clear_own();  // (this pool thread's: f may note a group-level failure, a peer copy's)
        const int r = f(s);
        if (r) {  // the message this call recorded on this thread: the shard engine's, else the group's
          const char* m = tfp_internal_engine_own_error(g->eng[s]);
          if (!m) m = g->err.own();
          why[s] = m ? m : r == TFP_E_NOMEM ? "out of memory" : "device call failed";
        }
        return r;
      },
      &bad);
  return rc ? gfail(g, rc, "shard %d (device %d): %s", bad, g->dev[bad], why[bad].c_str()) : TFP_OK;
}

constexpr int64_t kKeySpan = int64_t(1) << 31;  // tie-break keys lie in [0, 2^31)

// Every shard's tie-break keys (before any search after a change): after a respace, all of each
// shard's clips' keys; otherwise only the clip ids enrolled since (tfp_index_update_tiebreak).
int refresh_ranks(tfp_group* g) {
  if (!g->ranks_dirty) return TFP_OK;
  const int n = (int)g->eng.size();
  const bool full = g->keys_full;
  if (full) {  // even spacing over [0, 2^31) in uuid order
    const int64_t N = (int64_t)g->by_uuid.size(), step = kKeySpan / (N + 1);
    g->key2member.clear();
    g->key2member.reserve(N);
    for (int64_t r = 0; r < N; r++) {
      Member& m = g->members[g->by_uuid[r]];
      m.key = (int32_t)((r + 1) * step);
      g->key2member[m.key] = g->by_uuid[r];
    }
  }
  g->pushed.resize(n, 0);
  auto key_of_id = [&](int s, size_t id) {
    const int32_t mi = g->id2member[s][id];
    return mi < 0 ? -1 : g->members[mi].key;
  };
  const int rc = run_all(g, [&](int s) -> int {
    const size_t have = g->id2member[s].size(), from = full ? 0 : std::min(g->pushed[s], have);
    if (!full && from == have) return TFP_OK;
    std::vector<int32_t> keys(std::max<size_t>(have - from, 1));
    for (size_t id = from; id < have; id++) keys[id - from] = key_of_id(s, id);
    const int r = full ? tfp_index_set_tiebreak(g->eng[s], keys.data(), (int32_t)have)
                       : tfp_index_update_tiebreak(g->eng[s], (int32_t)from, keys.data(), (int32_t)(have - from));
    if (!r) g->pushed[s] = have;
    return r;
  });
  if (rc) {
    g->keys_full = true;  // (the next refresh sends everything again)
    return rc;
  }
  (full ? g->n_respaces : g->n_partial_pushes)++;
  g->keys_full = false;
  g->ranks_dirty = false;
  return TFP_OK;
}

bool uuid_less(const tfp_group* g, int32_t a, int32_t b) { return g->members[a].uuid < g->members[b].uuid; }

// A member into the uuid order; its key: the middle of its neighbours' gap (keys_full: the next
// refresh respaces every key instead).
void insert_live(tfp_group* g, int32_t mi) {
  auto it = std::lower_bound(g->by_uuid.begin(), g->by_uuid.end(), mi,
                             [&](int32_t a, int32_t b) { return uuid_less(g, a, b); });
  const size_t pos = (size_t)(it - g->by_uuid.begin());
  g->by_uuid.insert(it, mi);
  g->ranks_dirty = true;
  if (g->keys_full) return;
  const int64_t lo = pos > 0 ? g->members[g->by_uuid[pos - 1]].key : -1;
  const int64_t hi = pos + 1 < g->by_uuid.size() ? g->members[g->by_uuid[pos + 1]].key : kKeySpan;
  if (hi - lo < 2) {
    g->keys_full = true;
    return;
  }
  Member& m = g->members[mi];
  m.key = (int32_t)(lo + (hi - lo) / 2);
  g->key2member[m.key] = mi;
}

void erase_live(tfp_group* g, int32_t mi) {
  auto it = std::lower_bound(g->by_uuid.begin(), g->by_uuid.end(), mi,
                             [&](int32_t a, int32_t b) { return uuid_less(g, a, b); });
  if (it != g->by_uuid.end() && *it == mi) g->by_uuid.erase(it);
  Member& m = g->members[mi];
  if (m.key >= 0) {
    auto k = g->key2member.find(m.key);
    if (k != g->key2member.end() && k->second == mi) g->key2member.erase(k);
    m.key = -1;
  }
  // (no other key changes: the shards' keys stay valid, the removed clip's is never read again)
}

int32_t lightest(const tfp_group* g) {
  return (int32_t)(std::min_element(g->rows.begin(), g->rows.end()) - g->rows.begin());
}

// A shard's result -> its key (count << 32 | global rank); 0 = no hit.
unsigned long long key_of(const tfp_group* g, int s, const tfp_result& r) {
  if (!r.found || r.clip_id < 0 || (size_t)r.clip_id >= g->id2member[s].size()) return 0ull;
  const int32_t mi = g->id2member[s][r.clip_id];
  if (mi < 0 || g->members[mi].key < 0) return 0ull;
  return ((unsigned long long)(uint32_t)r.match_count << 32) | (uint32_t)g->members[mi].key;
}

// Per query, the greatest key over the shards' results -> the group's result.
void combine(tfp_group* g, const std::vector<std::vector<tfp_result>>& res, int32_t nq, tfp_result* out) {
  for (int32_t i = 0; i < nq; i++) {
    int best_s = -1;
    unsigned long long best = 0ull;
    for (size_t s = 0; s < res.size(); s++) {
      const unsigned long long k = key_of(g, (int)s, res[s][i]);
      if (k > best) best = k, best_s = (int)s;
    }
    out[i] = best_s >= 0 ? res[best_s][i] : res[0][i];
    if (best_s >= 0) out[i].clip_id = best_s;  // the shard holding the winner
    else out[i].found = 0, out[i].match_count = 0, out[i].clip_id = -1, out[i].uuid[0] = 0;
  }
}

// Global key -> result (uuid, count) for the query-sharded path.
void fill_from_key(const tfp_group* g, unsigned long long k, int32_t frame_count, tfp_result* r) {
  memset(r, 0, sizeof *r);
  r->frame_count = frame_count;
  r->clip_id = -1;
  if (!k) return;
  const auto it = g->key2member.find((int32_t)(uint32_t)(k & 0xffffffffu));
  if (it == g->key2member.end()) return;
  const Member& m = g->members[it->second];
  r->found = 1;
  r->match_count = (int32_t)(k >> 32);
  r->clip_id = m.shard;
  snprintf(r->uuid, sizeof r->uuid, "%s", m.uuid.c_str());
}

bool valid_params(const tfp_search_params* P) { return P && P->coefs >= 1 && P->coefs <= 2; }

int add_members(tfp_group* g, int32_t s, int32_t n, const char* const* uuids) {
  // (a large batch: one even respace at the next refresh instead of many halved gaps)
  if (n > 64) g->keys_full = true;
  // the engine assigns clip ids in order of addition (tfp_index_add / _add_batch)
  for (int32_t c = 0; c < n; c++) {
    const int32_t mi = (int32_t)g->members.size();
    g->members.push_back(Member{uuids[c], s, (int32_t)g->id2member[s].size()});
    g->id2member[s].push_back(mi);
    g->where[uuids[c]] = mi;
    insert_live(g, mi);
  }
  return TFP_OK;
}

// Query-sharded batch over host int16 PCM of equal-length queries: shard s fingerprints its share,
// the frame values are exchanged, every shard searches the whole batch.
int search_sharded(tfp_group* g, const int16_t* pcm, const int64_t* offsets, int32_t nq, int32_t sr,
                   const tfp_search_params* P, tfp_result* out) {
  const int n = (int)g->eng.size();
  const int64_t qn = offsets[1] - offsets[0];
  const int64_t nfq = tfp_frame_count(qn), nf = nfq * nq;
  std::vector<int32_t> share(n + 1);
  for (int s = 0; s <= n; s++) share[s] = (int32_t)(((int64_t)nq * s) / n);
  std::vector<int64_t> qoff(nq + 1);
  for (int32_t i = 0; i <= nq; i++) qoff[i] = nfq * i;
  std::vector<std::vector<unsigned long long>> keys(n, std::vector<unsigned long long>(nq));
  // 1: each shard fingerprints its queries into its part of its own q buffer
  int rc = run_all(g, [&](int s) -> int {
    ShardBufs& b = g->bufs[s];
    if (hipSetDevice(g->dev[s]) != hipSuccess) return TFP_E_HIP;
    if (!b.stream && hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking) != hipSuccess) return TFP_E_HIP;
    if (!b.fp_done && hipEventCreateWithFlags(&b.fp_done, hipEventDisableTiming) != hipSuccess) return TFP_E_HIP;
    const int32_t k = share[s + 1] - share[s];
    if (grow(&b.pcm, &b.b_pcm, sizeof(int16_t) * (size_t)(k * qn + 1)) != hipSuccess ||
        grow(&b.micro, &b.b_micro, sizeof(int32_t) * 2 * (size_t)(k * nfq + 1)) != hipSuccess ||
        grow(&b.q, &b.b_q, sizeof(double) * 2 * (size_t)(nf + 1)) != hipSuccess ||
        grow(&b.keys, &b.b_keys, sizeof(unsigned long long) * (size_t)(nq + 1)) != hipSuccess)
      return TFP_E_NOMEM;
    if (!k) return hipEventRecord(b.fp_done, b.stream) == hipSuccess ? TFP_OK : TFP_E_HIP;
    if (hipMemcpyAsync(b.pcm, pcm + offsets[share[s]] - offsets[0], sizeof(int16_t) * (size_t)(k * qn),
                       hipMemcpyHostToDevice, b.stream) != hipSuccess)
      return TFP_E_HIP;
    if (!b.plan || b.plan_k != k || b.plan_qn != qn || b.plan_sr != sr) {
      std::vector<int64_t> off(k + 1);
      for (int32_t i = 0; i <= k; i++) off[i] = qn * i;
      tfp_plan_destroy(b.plan);
      b.plan = nullptr;
      const int r = tfp_plan_create(g->eng[s], off.data(), k, sr, &b.plan);
      if (r) return r;
      b.plan_k = k, b.plan_qn = qn, b.plan_sr = sr;
    }
    const int r = tfp_fingerprint_device(g->eng[s], b.plan, (const int16_t*)b.pcm, (int32_t*)b.micro,
                                         (double*)b.q + 2 * nfq * share[s], b.stream);
    if (r) return r;
    if (hipEventRecord(b.fp_done, b.stream) != hipSuccess || hipStreamSynchronize(b.stream) != hipSuccess)
      return TFP_E_HIP;
    return TFP_OK;
  });
  if (rc) return rc;
  // 2: every shard pulls the other shards' frame values, searches the batch, keys to the host
  rc = run_all(g, [&](int s) -> int {
    ShardBufs& b = g->bufs[s];
    if (hipSetDevice(g->dev[s]) != hipSuccess) return TFP_E_HIP;
    for (int o = 0; o < n; o++) {
      const int32_t k = share[o + 1] - share[o];
      if (o == s || !k) continue;
      const size_t off = sizeof(double) * 2 * (size_t)(nfq * share[o]), bytes = sizeof(double) * 2 * (size_t)(nfq * k);
      if (const hipError_t pe = hipMemcpyPeerAsync((char*)b.q + off, g->dev[s], (const char*)g->bufs[o].q + off, g->dev[o],
                                                   bytes, b.stream);
          pe != hipSuccess)
        return gfail(g, TFP_E_HIP, "frame values of shard %d (device %d) to shard %d (device %d): hipMemcpyPeerAsync: %s", o,
                     g->dev[o], s, g->dev[s], hipGetErrorString(pe));
    }
    int r = tfp_search_q_device(g->eng[s], (const double*)b.q, qoff.data(), nq, P, (uint64_t*)b.keys, b.stream);
    if (r) return r;
    if (hipMemcpyAsync(keys[s].data(), b.keys, sizeof(unsigned long long) * nq, hipMemcpyDeviceToHost, b.stream) !=
            hipSuccess ||
        hipStreamSynchronize(b.stream) != hipSuccess)
      return TFP_E_HIP;
    return TFP_OK;
  });
  if (rc) return rc;
  for (int32_t i = 0; i < nq; i++) {
    unsigned long long k = 0ull;
    for (int s = 0; s < n; s++) k = std::max(k, keys[s][i]);
    fill_from_key(g, k, (int32_t)nfq, &out[i]);
  }
  return TFP_OK;
}

}  // namespace

extern "C" {

int tfp_group_create(const int32_t* devices, int32_t n, tfp_group** out) {
  if (!devices || n <= 0 || !out) return TFP_E_ARG;
  *out = nullptr;
  tfp_group* g = new tfp_group();
  for (int32_t s = 0; s < n; s++) {
    tfp_engine* e = nullptr;
    const int rc = tfp_engine_create(devices[s], &e);
    if (rc) {
      delete g;
      return rc;
    }
    g->eng.push_back(e);
    g->dev.push_back(devices[s]);
  }
  // peer access between the distinct devices (xGMI), for the query-sharded batches and split
  // streams. Counted per ordered pair (tfp_group_peer_stats); a pair without it still copies
  // (hipMemcpyPeerAsync stages through the host), and a failed copy fails the call loudly.
  for (int32_t a = 0; a < n; a++)
    for (int32_t b = 0; b < n; b++) {
      if (devices[a] == devices[b]) continue;
      bool seen = false;  // (a repeated pair of devices counts once)
      for (int32_t a2 = 0; a2 < n && !seen; a2++)
        for (int32_t b2 = 0; b2 < n && !seen; b2++)
          seen = (a2 < a || (a2 == a && b2 < b)) && devices[a2] == devices[a] && devices[b2] == devices[b];
      if (seen) continue;
      g->peer_pairs++;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devices[a], devices[b]) == hipSuccess && can && hipSetDevice(devices[a]) == hipSuccess) {
        g->peer_can++;
        const hipError_t e = hipDeviceEnablePeerAccess(devices[b], 0);
        if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) g->peer_enabled++;
        if (e != hipSuccess) (void)hipGetLastError();
      }
    }
  g->id2member.assign(n, {});
  g->rows.assign(n, 0);
  g->bufs.resize(n);
  g->pool = new tfp::ShardPool(n);
  if (const char* v = tfp::op_env("TFP_COALESCE")) g->coalesce = atoi(v) != 0;
  *out = g;
  return TFP_OK;
}

void tfp_group_destroy(tfp_group* g) { delete g; }

int tfp_group_peer_stats(const tfp_group* g, int32_t* pairs, int32_t* can_access, int32_t* enabled) {
  if (!g) return TFP_E_ARG;
  if (pairs) *pairs = g->peer_pairs;
  if (can_access) *can_access = g->peer_can;
  if (enabled) *enabled = g->peer_enabled;
  return TFP_OK;
}

int tfp_group_tiebreak_stats(tfp_group* g, int64_t* respaces, int64_t* partial_pushes, int64_t* shard_full_key_updates) {
  if (!g) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  if (respaces) *respaces = g->n_respaces;
  if (partial_pushes) *partial_pushes = g->n_partial_pushes;
  if (shard_full_key_updates) {
    int64_t t = 0;
    for (tfp_engine* e : g->eng) t += tfp_internal_delta_main_keys(e);
    *shard_full_key_updates = t;
  }
  return TFP_OK;
}

int32_t tfp_group_size(const tfp_group* g) { return g ? (int32_t)g->eng.size() : 0; }

const char* tfp_group_last_error(const tfp_group* g) { return g ? const_cast<tfp_group*>(g)->err.read(g) : ""; }

tfp_engine* tfp_group_engine(tfp_group* g, int32_t shard) {
  return g && shard >= 0 && shard < (int32_t)g->eng.size() ? g->eng[shard] : nullptr;
}

namespace {
int group_fingerprint(tfp_group* g, const void* x, bool f32, const int64_t* offsets, int32_t nclips, int32_t sr,
                      tfp_frame* out, int64_t cap, int64_t* nframes) {
  if (!g || !offsets || nclips < 0 || !nframes) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  const int n = (int)g->eng.size();
  std::vector<int64_t> foff(nclips + 1, 0);
  for (int32_t c = 0; c < nclips; c++) {
    if (offsets[c + 1] < offsets[c]) return gfail(g, TFP_E_ARG, "offsets not monotone");
    foff[c + 1] = foff[c] + tfp_frame_count(offsets[c + 1] - offsets[c]);
  }
  *nframes = foff[nclips];
  if (foff[nclips] > 0 && (!out || cap < foff[nclips])) return gfail(g, TFP_E_CAPACITY, "need %lld frames", (long long)foff[nclips]);
  if (!foff[nclips]) return TFP_OK;
  // contiguous clip ranges with about equal frames per shard
  std::vector<int32_t> cut(n + 1, nclips);
  cut[0] = 0;
  for (int s = 1; s < n; s++)
    cut[s] = (int32_t)(std::lower_bound(foff.begin(), foff.end(), foff[nclips] * s / n) - foff.begin());
  for (int s = 1; s <= n; s++) cut[s] = std::max(cut[s], cut[s - 1]);
  return run_all(g, [&](int s) -> int {
    const int32_t a = cut[s], b = cut[s + 1];
    if (a >= b) return TFP_OK;
    int64_t got = 0;
    return f32 ? tfp_fingerprint_f32_batch(g->eng[s], (const float*)x, offsets + a, b - a, sr, out + foff[a],
                                           foff[b] - foff[a], &got)
               : tfp_fingerprint_batch(g->eng[s], (const int16_t*)x, offsets + a, b - a, sr, out + foff[a],
                                       foff[b] - foff[a], &got);
  });
}
}  // namespace

int tfp_group_fingerprint_batch(tfp_group* g, const int16_t* pcm, const int64_t* offsets, int32_t nclips, int32_t sr,
                                tfp_frame* out, int64_t cap, int64_t* nframes) {
  return group_fingerprint(g, pcm, false, offsets, nclips, sr, out, cap, nframes);
}

int tfp_group_fingerprint_f32_batch(tfp_group* g, const float* x, const int64_t* offsets, int32_t nclips, int32_t sr,
                                    tfp_frame* out, int64_t cap, int64_t* nframes) {
  return group_fingerprint(g, x, true, offsets, nclips, sr, out, cap, nframes);
}

int tfp_group_index_add(tfp_group* g, const char* uuid, const int32_t* m1, const int32_t* m2, int32_t nframes) {
  if (!g) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  if (!uuid || g->where.count(uuid)) return gfail(g, uuid ? TFP_E_EXISTS : TFP_E_ARG, "uuid %s already indexed", uuid ? uuid : "(null)");
  const int32_t s = lightest(g);
  int32_t id = -1;
  const int rc = tfp_index_add(g->eng[s], uuid, m1, m2, nframes, &id);
  if (rc) return shard_fail(g, rc, s);
  if (id != (int32_t)g->id2member[s].size()) {  // (never expected) undo the engine's add: no clip without a member
    (void)tfp_index_remove(g->eng[s], uuid);
    return gfail(g, TFP_E_HIP, "shard %d clip id %d out of step", s, id);
  }
  g->rows[s] += nframes;
  return add_members(g, s, 1, &uuid);
}

int tfp_group_index_add_batch(tfp_group* g, int32_t nclips, const char* const* uuids, const int64_t* foff,
                              const int32_t* m1, const int32_t* m2) {
  if (!g || nclips < 0 || !uuids || !foff) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  const int n = (int)g->eng.size();
  std::unordered_map<std::string, int> seen;
  for (int32_t c = 0; c < nclips; c++) {
    if (!uuids[c] || !*uuids[c] || strlen(uuids[c]) >= 64) return gfail(g, TFP_E_ARG, "bad uuid %d", c);
    if (foff[c + 1] < foff[c]) return gfail(g, TFP_E_ARG, "frame_offsets not monotone at %d", c);
    if (g->where.count(uuids[c]) || !seen.emplace(uuids[c], c).second)
      return gfail(g, TFP_E_EXISTS, "uuid %s already indexed", uuids[c]);
  }
  // each clip to the shard with the fewest rows so far; per shard one tfp_index_add_batch
  std::vector<std::vector<int32_t>> pick(n);
  std::vector<int64_t> rows = g->rows;
  for (int32_t c = 0; c < nclips; c++) {
    const int32_t s = (int32_t)(std::min_element(rows.begin(), rows.end()) - rows.begin());
    pick[s].push_back(c);
    rows[s] += foff[c + 1] - foff[c];
  }
  std::vector<std::vector<const char*>> uu(n);
  std::vector<std::vector<int64_t>> fo(n);
  std::vector<std::vector<int32_t>> a1(n), a2(n);
  for (int s = 0; s < n; s++) {
    fo[s].push_back(0);
    for (int32_t c : pick[s]) {
      uu[s].push_back(uuids[c]);
      a1[s].insert(a1[s].end(), m1 + foff[c], m1 + foff[c + 1]);
      a2[s].insert(a2[s].end(), m2 + foff[c], m2 + foff[c + 1]);
      fo[s].push_back((int64_t)a1[s].size());
    }
  }
  std::vector<int> rcs(n, TFP_OK);
  const int rc = run_all(g, [&](int s) -> int {
    if (uu[s].empty()) return TFP_OK;
    return rcs[s] = tfp_index_add_batch(g->eng[s], (int32_t)uu[s].size(), uu[s].data(), fo[s].data(), a1[s].data(),
                                        a2[s].data());
  });
  // All-or-nothing over the group, as each engine's add_batch is per call: when a shard failed (a
  // device error: the arguments were checked above), the shards that succeeded drop the batch's
  // clips again, so no clip stays on a GPU without a member (or a catalog row: the shim deletes
  // the batch's rows on failure).
  if (rc) {
    for (int s = 0; s < n; s++)
      if (!uu[s].empty() && rcs[s] == TFP_OK) {
        for (const char* u : uu[s]) (void)tfp_index_remove(g->eng[s], u);
        // the engine's clip ids of the dropped clips stay used: keep the group's id map in step
        g->id2member[s].insert(g->id2member[s].end(), uu[s].size(), -1);
        g->ranks_dirty = true;
      }
    return rc;
  }
  for (int s = 0; s < n; s++)
    if (!uu[s].empty()) {
      add_members(g, s, (int32_t)uu[s].size(), uu[s].data());
      g->rows[s] += fo[s].back();
    }
  return TFP_OK;
}

int tfp_group_index_remove(tfp_group* g, const char* uuid) {
  if (!g || !uuid) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  auto it = g->where.find(uuid);
  if (it == g->where.end()) return gfail(g, TFP_E_NOENT, "uuid %s not indexed", uuid);
  const int32_t mi = it->second;
  Member& m = g->members[mi];
  int64_t nr = 0;
  (void)tfp_index_rows(g->eng[m.shard], uuid, nullptr, nullptr, 0, &nr);
  const int rc = tfp_index_remove(g->eng[m.shard], uuid);
  if (rc) return shard_fail(g, rc, m.shard);
  erase_live(g, mi);
  g->rows[m.shard] -= nr;
  g->id2member[m.shard][m.id] = -1;
  g->where.erase(it);
  m.uuid.clear();
  return TFP_OK;
}

int tfp_group_index_clear(tfp_group* g) {
  if (!g) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  const int n = (int)g->eng.size();
  std::vector<int> rcs(n, TFP_OK);
  const int rc = run_all(g, [&](int s) { return rcs[s] = tfp_index_clear(g->eng[s]); });
  g->ranks_dirty = true;
  g->keys_full = true;
  if (rc == TFP_OK) {
    g->where.clear();
    g->members.clear();
    g->by_uuid.clear();
    for (auto& v : g->id2member) v.clear();
    std::fill(g->rows.begin(), g->rows.end(), 0);
    return TFP_OK;
  }
  // a shard whose clear failed keeps its clips, and the group keeps them as its members
  for (int s = 0; s < n; s++) {
    if (rcs[s] != TFP_OK) continue;
    for (int32_t mi : g->id2member[s]) {
      if (mi < 0) continue;
      Member& m = g->members[mi];
      erase_live(g, mi);
      g->where.erase(m.uuid);
      m.uuid.clear();
    }
    g->id2member[s].clear();
    g->rows[s] = 0;
  }
  return rc;
}

int tfp_group_index_rows(tfp_group* g, const char* uuid, int32_t* m1, int32_t* m2, int64_t cap, int64_t* nframes) {
  if (!g || !uuid) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  auto it = g->where.find(uuid);
  if (it == g->where.end()) return gfail(g, TFP_E_NOENT, "uuid %s not indexed", uuid);
  const int s = g->members[it->second].shard;
  const int rc = tfp_index_rows(g->eng[s], uuid, m1, m2, cap, nframes);
  return rc ? shard_fail(g, rc, s) : TFP_OK;
}

int tfp_group_index_stats(tfp_group* g, int64_t* nrows, int32_t* nclips) {
  if (!g) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  int64_t r = 0;
  int32_t c = 0;
  for (auto* e : g->eng) {
    int64_t a = 0;
    int32_t b = 0;
    const int rc = tfp_index_stats(e, &a, &b);
    if (rc) return rc;
    r += a;
    c += b;
  }
  if (nrows) *nrows = r;
  if (nclips) *nclips = c;
  return TFP_OK;
}

int tfp_group_index_commit(tfp_group* g) {
  if (!g) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  int rc = refresh_ranks(g);
  if (rc) return rc;
  return run_all(g, [&](int s) { return tfp_index_commit(g->eng[s]); });
}

int tfp_group_search_batch(tfp_group* g, const tfp_frame* frames, const int64_t* qoff, int32_t nq,
                           const tfp_search_params* P, tfp_result* out) {
  if (!g || !qoff || nq < 0 || !out) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  int rc = refresh_ranks(g);
  if (rc) return rc;
  const int n = (int)g->eng.size();
  std::vector<std::vector<tfp_result>> res(n, std::vector<tfp_result>(std::max(nq, 1)));
  rc = run_all(g, [&](int s) { return tfp_search_batch(g->eng[s], frames, qoff, nq, P, res[s].data()); });
  if (rc) return rc;
  combine(g, res, nq, out);
  return TFP_OK;
}

namespace {
// One search over host samples on every shard (each fingerprints the whole batch: no exchange on
// the latency path), combined by the integer max of the keys.
int group_search_direct(tfp_group* g, const void* const* ptrs, const int64_t* lens, int32_t nq, bool f32, int32_t sr,
                        const tfp_search_params* P, tfp_result* out) {
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  int rc = refresh_ranks(g);
  if (rc) return rc;
  const int n = (int)g->eng.size();
  std::vector<std::vector<tfp_result>> res(n, std::vector<tfp_result>(std::max(nq, 1)));
  rc = run_all(g, [&](int s) { return tfp_internal_search_gather(g->eng[s], ptrs, lens, nq, f32, sr, P, res[s].data()); });
  if (rc) return rc;
  combine(g, res, nq, out);
  return TFP_OK;
}

int group_search_gather(tfp_group* g, const void* const* ptrs, const int64_t* lens, int32_t nq, bool f32, int32_t sr,
                        const tfp_search_params* P, tfp_result* out) {
  if (!g || nq < 0 || !out || (nq && (!ptrs || !lens))) return TFP_E_ARG;
  for (int32_t i = 0; i < nq; i++)
    if (lens[i] < 0 || (lens[i] && !ptrs[i])) return gfail(g, TFP_E_ARG, "bad query %d", i);
  if (!g->coalesce || nq == 0 || nq > tfp::Coalescer::kMaxCallQueries)
    return group_search_direct(g, ptrs, lens, nq, f32, sr, P, out);
  tfp::SearchReq r;
  r.ptrs.assign(ptrs, ptrs + nq);
  r.lens.assign(lens, lens + nq);
  r.f32 = f32;
  r.sr = sr;
  if (P) r.P = *P;
  else r.P.coefs = 0;  // (invalid: NULL results, fp_handler.c:247-250)
  r.out = out;
  const int rc = g->coal.submit(&r, [g](std::vector<tfp::SearchReq*>& batch) {
    tfp::exec_batch(
        batch,
        [g](const void* const* p, const int64_t* l, int32_t n, bool f, int32_t rate, const tfp_search_params* q,
            tfp_result* o) { return group_search_direct(g, p, l, n, f, rate, q, o); },
        [g] { return std::string(tfp_group_last_error(g)); });
  });
  if (rc) g->err.note(g, r.err.c_str());  // (the leader ran it: the message into this caller's slot)
  return rc;
}

int group_search_samples(tfp_group* g, const void* x, bool f32, const int64_t* offsets, int32_t nq, int32_t sr,
                         const tfp_search_params* P, tfp_result* out) {
  if (!g || !offsets || nq < 0 || !out) return TFP_E_ARG;
  for (int32_t i = 0; i < nq; i++)
    if (offsets[i + 1] < offsets[i]) return gfail(g, TFP_E_ARG, "offsets not monotone");
  if (!x && nq && offsets[nq] > offsets[0]) return gfail(g, TFP_E_ARG, "samples are NULL");
  const int n = (int)g->eng.size();
  // throughput batches of equal-length int16 queries: query-sharded (fingerprint once, exchange)
  bool equal = nq > 0;
  for (int32_t i = 0; i < nq && equal; i++) equal = offsets[i + 1] - offsets[i] == offsets[1] - offsets[0];
  if (!f32 && n > 1 && equal && nq >= 64 * n && offsets[1] > offsets[0] && valid_params(P)) {
    std::lock_guard<std::recursive_mutex> lk(g->mu);
    const int rc = refresh_ranks(g);
    return rc ? rc : search_sharded(g, (const int16_t*)x, offsets, nq, sr, P, out);
  }
  const size_t ss = f32 ? sizeof(float) : sizeof(int16_t);
  std::vector<const void*> ptrs(nq);
  std::vector<int64_t> lens(nq);
  for (int32_t i = 0; i < nq; i++) {
    ptrs[i] = static_cast<const char*>(x) + ss * offsets[i];
    lens[i] = offsets[i + 1] - offsets[i];
  }
  return group_search_gather(g, ptrs.data(), lens.data(), nq, f32, sr, P, out);
}
}  // namespace

int tfp_group_search_pcm_batch(tfp_group* g, const int16_t* pcm, const int64_t* offsets, int32_t nq, int32_t sr,
                               const tfp_search_params* P, tfp_result* out) {
  return group_search_samples(g, pcm, false, offsets, nq, sr, P, out);
}

int tfp_group_search_f32_batch(tfp_group* g, const float* x, const int64_t* offsets, int32_t nq, int32_t sr,
                               const tfp_search_params* P, tfp_result* out) {
  return group_search_samples(g, x, true, offsets, nq, sr, P, out);
}

int tfp_group_search_pcm_gather(tfp_group* g, const int16_t* const* pcms, const int64_t* nsamples, int32_t nq,
                                int32_t sr, const tfp_search_params* P, tfp_result* out) {
  return group_search_gather(g, reinterpret_cast<const void* const*>(pcms), nsamples, nq, false, sr, P, out);
}

int tfp_group_search_coalesce_stats(tfp_group* g, int64_t* calls, int64_t* batches) {
  if (!g) return TFP_E_ARG;
  g->coal.stats(calls, batches);
  return TFP_OK;
}

int tfp_group_stream_create(tfp_group* g, int32_t nch, int32_t sr, int64_t W, tfp_group_stream** out) {
  if (!g || nch <= 0 || W <= 0 || !out) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  *out = nullptr;
  tfp_group_stream* st = new tfp_group_stream();
  const int n = (int)g->eng.size();
  st->g = g;
  st->nch = nch;
  st->W = W;
  const char* mode = tfp::op_env("TFP_GROUP_STREAM");  // operational switch
  st->split = n > 1 && !(mode && !strcmp(mode, "replicate"));
  st->st.assign(n, nullptr);
  if (st->split) {
    st->chans.assign(n, {});
    for (int32_t c = 0; c < nch; c++) st->chans[c % n].push_back(c);
    st->tick.assign(n, {});
    st->act.assign(n, {});
    st->nact.assign(n, 0);
    st->keys.assign(n, {});
    for (int s = 0; s < n; s++) st->act[s].assign(st->chans[s].size(), 0);
  }
  const int rc = run_all(g, [&](int s) {
    if (!st->split) return tfp_stream_create(g->eng[s], nch, sr, W, &st->st[s]);
    return st->chans[s].empty() ? TFP_OK : tfp_stream_create(g->eng[s], (int32_t)st->chans[s].size(), sr, W, &st->st[s]);
  });
  if (rc) {
    for (auto* p : st->st) tfp_stream_destroy(p);
    delete st;
    return rc;
  }
  st->res.assign(g->eng.size(), std::vector<tfp_result>(nch));
  *out = st;
  return TFP_OK;
}

void tfp_group_stream_destroy(tfp_group_stream* st) {
  if (!st) return;
  for (auto* p : st->st) tfp_stream_destroy(p);
  delete st;
}

int tfp_group_stream_reset(tfp_group_stream* st, int32_t ch) {
  if (!st || ch >= st->nch) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(st->g->mu);
  if (st->split) {
    const int n = (int)st->g->eng.size();
    if (ch >= 0) return tfp_stream_reset(st->st[ch % n], ch / n);  // channel c is local channel c / N of shard c mod N
    return run_all(st->g, [&](int s) { return st->st[s] ? tfp_stream_reset(st->st[s], -1) : TFP_OK; });
  }
  return run_all(st->g, [&](int s) { return tfp_stream_reset(st->st[s], ch); });
}

namespace {

// A tick of a split-channel stream: (1) every shard pushes its channels' rows and fingerprints its
// full windows into its sfp buffer; (2) every shard gathers all shards' window values in shard
// order (hipMemcpyPeerAsync; a device copy when a device repeats) and matches them against its
// clips; (3) per window, the greatest key over the shards.
int split_stream_push(tfp_group_stream* st, const int16_t* pcm, int32_t T, const tfp_search_params* P, tfp_result* out) {
  tfp_group* g = st->g;
  const int n = (int)g->eng.size();
  for (int s = 0; s < n; s++) {
    const auto& ch = st->chans[s];
    st->tick[s].resize(ch.size() * (size_t)T);
    for (size_t j = 0; j < ch.size(); j++)
      memcpy(st->tick[s].data() + j * T, pcm + (size_t)ch[j] * T, sizeof(int16_t) * (size_t)T);
  }
  const bool match = valid_params(P);
  const int64_t F = tfp_frame_count(st->W);
  int rc = run_all(g, [&](int s) -> int {
    st->nact[s] = 0;
    if (!st->st[s]) return TFP_OK;
    ShardBufs& b = g->bufs[s];
    if (hipSetDevice(g->dev[s]) != hipSuccess) return TFP_E_HIP;
    const int64_t cap = (int64_t)st->chans[s].size() * F;
    if (match && grow(&b.sfp, &b.b_sfp, sizeof(double) * 2 * (size_t)(cap + 1)) != hipSuccess) return TFP_E_NOMEM;
    int64_t fw = 0;
    return tfp_internal_stream_fp(st->st[s], st->tick[s].data(), T, match ? P : nullptr, (double*)b.sfp, cap,
                                  st->act[s].data(), &st->nact[s], &fw);
  });
  if (rc || !P) return rc;
  for (int32_t c = 0; c < st->nch; c++) {
    memset(&out[c], 0, sizeof out[c]);
    out[c].clip_id = -1;
  }
  std::vector<int32_t> base(n + 1, 0);
  for (int s = 0; s < n; s++) base[s + 1] = base[s] + st->nact[s];
  const int32_t na = base[n];
  if (!match || !na) return TFP_OK;
  std::vector<int64_t> qoff(na + 1);
  for (int32_t i = 0; i <= na; i++) qoff[i] = F * i;
  rc = run_all(g, [&](int s) -> int {
    ShardBufs& b = g->bufs[s];
    if (hipSetDevice(g->dev[s]) != hipSuccess) return TFP_E_HIP;
    if (!b.stream && hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking) != hipSuccess) return TFP_E_HIP;
    if (grow(&b.q, &b.b_q, sizeof(double) * 2 * (size_t)(na * F + 1)) != hipSuccess ||
        grow(&b.keys, &b.b_keys, sizeof(unsigned long long) * (size_t)(na + 1)) != hipSuccess)
      return TFP_E_NOMEM;
    for (int o = 0; o < n; o++) {
      if (!st->nact[o]) continue;
      const size_t off = sizeof(double) * 2 * (size_t)(F * base[o]), bytes = sizeof(double) * 2 * (size_t)(F * st->nact[o]);
      if (const hipError_t pe = hipMemcpyPeerAsync((char*)b.q + off, g->dev[s], g->bufs[o].sfp, g->dev[o], bytes, b.stream);
          pe != hipSuccess)
        return gfail(g, TFP_E_HIP, "stream windows of shard %d (device %d) to shard %d (device %d): hipMemcpyPeerAsync: %s", o,
                     g->dev[o], s, g->dev[s], hipGetErrorString(pe));
    }
    st->keys[s].resize(na);
    int r = tfp_search_q_device(g->eng[s], (const double*)b.q, qoff.data(), na, P, (uint64_t*)b.keys, b.stream);
    if (r) return r;
    if (hipMemcpyAsync(st->keys[s].data(), b.keys, sizeof(unsigned long long) * na, hipMemcpyDeviceToHost, b.stream) !=
            hipSuccess ||
        hipStreamSynchronize(b.stream) != hipSuccess)
      return TFP_E_HIP;
    return TFP_OK;
  });
  if (rc) return rc;
  for (int o = 0; o < n; o++)
    for (int32_t j = 0; j < st->nact[o]; j++) {
      const int32_t i = base[o] + j;
      unsigned long long k = 0ull;
      for (int s = 0; s < n; s++) k = std::max(k, st->keys[s][i]);
      fill_from_key(g, k, (int32_t)F, &out[st->chans[o][st->act[o][j]]]);
    }
  return TFP_OK;
}

}  // namespace

int tfp_group_stream_push(tfp_group_stream* st, const int16_t* pcm, int32_t tick, const tfp_search_params* P,
                          tfp_result* out) {
  if (!st || !pcm || tick <= 0 || (P && !out)) return TFP_E_ARG;
  tfp_group* g = st->g;
  std::lock_guard<std::recursive_mutex> lk(g->mu);
  int rc = P ? refresh_ranks(g) : TFP_OK;
  if (rc) return rc;
  if (st->split) return split_stream_push(st, pcm, tick, P, out);
  rc = run_all(g, [&](int s) { return tfp_stream_push(st->st[s], pcm, tick, P, P ? st->res[s].data() : nullptr); });
  if (rc || !P) return rc;
  combine(g, st->res, st->nch, out);
  return TFP_OK;
}

}  // extern "C"
