// tfp_engine.cpp — C-ABI implementation (include/tiresias_fp.h) on top of the gfx950 kernels.
//
// Owns one HIP device + stream per engine, the per-sample-rate DSP tables, the enrolled
// index (staging rows + the m1-sorted device index rebuilt lazily after changes) and the
// search scratch. Every entry point takes the engine mutex, so concurrent channel threads
// (the reference runs one tiresias_exec per channel, application_handler.c:66) are safe.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <chrono>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/tiresias_fp.h"
#include "tfp_coalesce.hpp"
#include "tfp_index.hpp"
#include "tfp_internal.hpp"
#include "tfp_kernels.hpp"
#include "tfp_math.hpp"
#include "tfp_synth.hpp"
#include "tfp_tables.hpp"

using namespace tfp;

namespace {

// Grow-only device buffer.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevBuf() { if (p) (void)hipFree(p); }
  hipError_t reserve(size_t n) {
    if (n <= bytes) return hipSuccess;
    if (p) { (void)hipFree(p); p = nullptr; bytes = 0; }
    size_t want = n < 256 ? 256 : n;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) bytes = want;
    return e;
  }
  // for buffers that grow a little per call (the merged index): 1/8 headroom, so a run of
  // enrolments does not free and reallocate hundreds of MB each time
  hipError_t reserve_grow(size_t n) { return n <= bytes ? hipSuccess : reserve(n + n / 8); }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
  void swap_with(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(bytes, o.bytes);
  }
};

// A tolerance's key row ranges and key bitsets kept beside the active ones (tfp_engine::tol_lru):
// the dialplan passes the tolerance per call (application_handler.c:114-122), so extensions at
// different tolerances alternate on one engine. Valid while the index is at `version`.
struct TolSlot {
  double tol = 0.0;
  DevBuf rng_all, key_bits;
  bool rng_valid = false, bits_valid = false;
  int32_t bits_cols = -1;
  uint64_t version = 0, used = 0;
};

// A tolerance's clip-set cache kept beside the active one (tfp_engine::cell_lru, round 6): callers
// alternating coefs = 2 tolerances do not rebuild it per call. Valid while the index is at `version`.
struct CellSlot {
  CellCache c;
  double tol = 0.0;
  bool has = false;
  uint64_t version = 0, used = 0;
};

// Pinned host staging (one H2D copy per small call instead of one per array).
struct HostBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~HostBuf() { if (p) (void)hipHostFree(p); }
  hipError_t reserve(size_t n, unsigned flags = hipHostMallocDefault) {
    if (n <= bytes) return hipSuccess;
    if (p) { (void)hipHostFree(p); p = nullptr; bytes = 0; }
    size_t want = n < 65536 ? 65536 : n;
    hipError_t e = hipHostMalloc(&p, want, flags);
    if (e == hipSuccess) bytes = want;
    return e;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

struct Clip {
  std::string uuid;
  bool alive = true;
  int64_t nrows = 0;
  int64_t off = 0;  // first staging row (a clip's rows are contiguous, in frame order)
};

// tfp_host_alloc's buffers: host address -> (bytes, generation), so a call whose samples lie
// inside one hands the GPU the samples in place. The device address is resolved per engine
// (hipHostGetDevicePointer on the engine's own device, cached by base and generation), not taken
// from whichever device was current at allocation.
struct HostAllocs {
  std::mutex mu;
  std::map<uintptr_t, std::pair<size_t, uint64_t>> m;
  uint64_t next_gen = 1;
  // the buffer holding [p, p + n): its base and generation, or false
  bool find(const void* p, size_t n, uintptr_t* base, uint64_t* gen) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lk(mu);
    auto it = m.upper_bound(a);
    if (it == m.begin()) return false;
    --it;
    if (a + n > it->first + it->second.first) return false;
    *base = it->first;
    *gen = it->second.second;
    return true;
  }
};
HostAllocs& host_allocs() {
  static HostAllocs h;
  return h;
}

}  // namespace

struct tfp_plan {
  int32_t nclips = 0, ntiles = 0, sample_rate = 0, tile_frames = 0;
  bool long_clip = false;  // a clip of >= kDirectMaxSamples: the generic kernel
  int64_t nsamples = 0, nframes = 0;
  std::vector<int64_t> soff, foff;
  std::vector<int32_t> toff, tclip;
  DevBuf d_soff, d_foff, d_toff, d_tclip;
  std::vector<int64_t> qoff;  // == foff (frames per clip as queries)
  DevBuf d_qoff;
  tfp_engine* eng = nullptr;
};

struct tfp_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  std::recursive_mutex mu;
  tfp::ErrorSlot err;  // last-error messages (tfp_internal.hpp)
  std::map<int, DevBuf> tables;  // sample rate -> device DspTables
  std::map<int, bool> tables_fixed8k;  // sample rate -> DspTables_fixed8k (kernel variant)

  // staging (append-only) rows of every clip ever added
  std::vector<Clip> clips;
  std::unordered_map<std::string, int32_t> by_uuid;
  DevBuf st_m1, st_m2, st_clip;
  int64_t n_staged = 0, cap_staged = 0;
  bool dirty = true;

  // sorted index
  DevBuf m1s, m2s, cols, rank_of_clip, tiekey;
  // incremental maintenance (merge_index): the last build's clips and staged rows, the merge's
  // output buffers (swapped with m1s/m2s/cols) and scratch
  bool built = false;        // m1s/m2s/cols/col_clip describe clips [0, built_clips) as of the last build
  bool force_full = false;   // TFP_INDEX_FULL: every update is a full build (A/B, tests)
  size_t built_clips = 0;
  int64_t built_staged = 0;
  bool removed_built = false;  // a clip of the last build was removed since (else an update only adds)
  int64_t live_rows = 0;       // staged rows of live clips (kept per add / remove, not counted per build)
  int64_t n_merges = 0, n_full_builds = 0;
  DevBuf m1s_b, m2s_b, cols_b, remap;
  MergeScratch merge;
  int64_t nrows = 0;       // rows that can match (live clip, non-NULL max1)
  int32_t ncols = 0;       // live clips
  std::vector<int32_t> col_clip;                 // column (uuid rank) -> clip id
  std::unordered_map<int32_t, int32_t> key_col;  // tie-break key -> main column (with an override)
  std::unordered_map<int32_t, int32_t> key_col_delta;  // ... -> the index delta's columns
  bool key_identity = true;                      // no override: key == column
  std::vector<int32_t> tiebreak_override;        // clip id -> key (empty = uuid rank)
  // with an override: key_col / the device tie keys of the main columns no longer match it (a full
  // tfp_index_set_tiebreak, or new keys for clips of the last build); tfp_index_update_tiebreak of
  // clips added since leaves them standing, so a delta update costs the delta's clips only
  bool ovr_main_stale = true;
  int64_t n_delta_main_keys = 0;  // delta updates that re-sent every main column's key (tests)

  // scratch
  DevBuf sort_tmp, keys_a, keys_b, vals_a, vals_b, cnt;
  DevBuf pcm, q, qoff, boxes, vote_part, mask, maxc, A, Bt, best, stamp, score, micro, db;
  DevBuf soff, foff, toff, tclip, specs;
  // small host calls: packed upload + the small-batch search workspace
  HostBuf hstage;
  DevBuf dstage;
  HostBuf zstage;                   // mapped + coherent: small 8 kHz calls are read by the kernel in place
  void* zstage_host = nullptr;      // the allocation zstage_dev was taken for
  char* zstage_dev = nullptr;
  DevBuf zlayout;                   // device copy of the last zero-copy call's tile layout
  std::vector<char> zlayout_host;   // ... and its bytes (re-uploaded when they change)
  bool stage_pending = false;  // hstage / zstage may still be read by a copy or kernel on e->stream
  std::unordered_map<uintptr_t, std::pair<uint64_t, char*>> host_dev;  // tfp_host_alloc base -> (generation, device address)
  HostBuf qoff_pin;                   // pinned source of the qoff copy
  std::vector<int64_t> qoff_host;     // what e->qoff holds (copied on stream qoff_stream)
  hipStream_t qoff_stream = nullptr;
  hipEvent_t qoff_ev = nullptr;
  bool qoff_pending = false;
  DevBuf key_bits;           // key-presence bitsets at tolerance rng_tol (launch_key_bits; small path)
  DevBuf key_bits_b;         // the other buffer of an update carried across a merge (merge_index)
  int64_t tiekey_ident = -1; // tiekey on the device holds the identity over this many columns (-1: not known)
  bool key_bits_valid = false;
  HostBuf vres_pin;         // pinned (VoteMeta, best[]) of the vote path
  HostBuf spec_pin;         // pinned copy of the speculative sweep's counts (WideScratch::info), host-mapped
  void* spec_pin_host = nullptr;   // the allocation spec_pin_dev was taken for
  int32_t* spec_pin_dev = nullptr; // its device address (the sweep's last kernel writes it)
  HostBuf small_res;        // host-mapped SmallResult, written by small_vote_kernel (no copy back)
  SmallResult* small_res_dev = nullptr;
  void* small_res_host = nullptr;  // the allocation small_res_dev was taken for
  DevBuf rng_all;            // row ranges of all keys' boxes at tolerance rng_tol (valid for this index)
  double rng_tol = 0.0;
  bool rng_valid = false;
  // other tolerances' ranges and bitsets (least recently used first out), valid at index_version;
  // index_version changes with every index update (rebuild, delta update), which carries only the
  // active tolerance's
  static constexpr int kTolSlots = 3;
  TolSlot tol_lru[kTolSlots];
  uint64_t index_version = 1, tol_clock = 0;
  // the main index's own version (builds and merges; a delta update leaves it): the clip-set caches
  // hold main-index rows only, so they stay valid across delta updates
  uint64_t main_version = 1;
  // general path: clip-set cache at tolerance cell_tol (tfp_scan.hip), built on first use per
  // index version and tolerance
  CellCache cells;
  WideScratch wide;         // the general path's sweep by groups
  double wide_min_tol = 0;  // TFP_WIDE_MIN_TOL: general-path batches below it take the clip-set cells (tests)
  double cell_tol = 0.0;
  bool cell_fresh = false;  // cells holds the cache of cell_tol at index version cell_version
  uint64_t cell_version = 0;
  // other tolerances' clip-set caches (round 6), least recently used out, valid at their version
  static constexpr int kCellSlots = 3;
  CellSlot cell_lru[kCellSlots];
  int64_t n_cell_builds = 0, n_cell_hits = 0, n_cell_from_order = 0;
  // the coefs = 2 sweep's sort path per batch (tfp_sweep_stats): the bin sort's speculative pass
  // stood, the library sort ran, a speculative pass was redone; crowd bins the bin sort copied
  int64_t n_sweep_bins = 0, n_sweep_lib = 0, n_sweep_redo = 0, n_sweep_crowd = 0;
  // coefs = 2 with an index delta (round 6): the delta's own clip-set cache (its staged rows in clip
  // order, columns numbered from 0 in uuid order), swept after the main cache into the same maxima,
  // so an enrolment followed by a coefs = 2 search does not merge the index (fp_handler.c:559-571:
  // the reference's INSERT makes a clip searchable for the cost of its own rows)
  CellCache dcells;
  double dcell_tol = 0.0;
  uint64_t dcell_version = 0, dl_version = 0;  // index versions of dcells and of the delta rows' order
  bool dcell_fresh = false;
  DevBuf dl_key, dl_m1, dl_key_b, dl_m1_b;
  CacheBuf dl_sort_tmp;
  bool delta_wide = true;  // TFP_DELTA_WIDE=0: coefs = 2 searches merge the delta first (A/B, tests)
  int64_t n_delta_cell_builds = 0, n_delta_sweeps = 0;
  // the index rows in clip order (tfp_kernels.hpp), the source of the caches at tolerances up to
  // kOrderMaxTol: built on the first search that needs it, then carried through every merge
  DevBuf o_key, o_m1, o_key_b, o_m1_b, o_newcol;
  int64_t o_rows = 0;
  bool o_valid = false;
  int64_t n_order_builds = 0, n_order_merges = 0;
  CacheBuf o_sort_tmp;
  OrderScratch o_merge;
  // scan scratch: stamp / score / touched nq x ncols int32 each, tcnt nq int32; kept all-zero
  // by the scan kernels themselves
  DevBuf touched, tcnt;
  size_t scan_zeroed = 0;  // bytes of stamp / score / touched known to be zero
  // launch configuration and test/A-B knobs, read once at engine creation
  FpLaunchCfg fpcfg;
  int32_t class_ku_max = 10;  // TFP_VOTE_CLASS_MAX: pattern-class vote up to this many used keys (-1: always the GEMM)
  bool dbg_vote = false;      // TFP_DEBUG_VOTE: log the vote path's shape per batch
  bool dbg_index = false;     // TFP_DEBUG_INDEX: log each index update's phases (host ms)
  int32_t fail_compact = 0;   // TFP_TEST_FAIL_COMPACT=n: the next n staging compactions fail (tests)
  int64_t fail_query_len = -1;  // TFP_TEST_FAIL_QUERY_SAMPLES=n: a search with a query of n samples fails (tests)
  int32_t kb_win = 0;           // TFP_KEYBITS_WIN: LDS words per column window of launch_key_bits (tests; 0 = default)
  int64_t kb_direct = -1;       // TFP_KEYBITS_DIRECT: pieces below this many rows use global atomics (tests; -1 = default)
  DevBuf logfix_key, logfix_val, logfix_bits;  // device copy of the glibc log correction table (LogFix)
  LogFix logfix{nullptr, nullptr, 0};
  // index delta (round 4, tfp_index.hpp): the live clips added since the last build, searched by the
  // coefs = 1 vote paths beside the main index instead of merged into it per enrolment
  static constexpr int32_t kDeltaMaxClips = 512;        // columns reserved for them
  static constexpr int64_t kDeltaMaxRows = 1ll << 20;  // beyond either limit the next update merges
  bool use_delta = true;          // TFP_INDEX_DELTA=0: every update merges (A/B, tests)
  // The delta pads the main columns to a multiple of 1024 and reserves kDeltaMaxClips columns
  // after them, which a small DB's vote passes would pay for on every search (300 clips -> 1,536
  // columns); below this many main columns an update merges instead (cheap at that size).
  // TFP_INDEX_DELTA=1 (tests) takes the delta at any size.
  int64_t delta_min_cols = 4096;
  bool force_merge = false;       // consolidate(): the next rebuild merges the delta
  std::vector<int32_t> delta_clip;  // delta column delta_col0 + j -> clip id (uuid order)
  std::vector<int32_t> delta_at;    // delta j's insertion point among the main columns' uuids
  int32_t delta_col0 = 0;           // first delta column (a multiple of 1024)
  int64_t delta_rows = 0;           // staged rows of the delta's clips
  int64_t n_delta_updates = 0;
  DevBuf d_delta, d_delta_at, kbox;
  double kbox_tol = 0.0;
  bool kbox_valid = false;
  int32_t key_bits_cols = -1;       // the column count key_bits was laid out for (its row width)
  Coalescer coal;          // concurrent small host-sample searches share one batch (tfp_coalesce.hpp)
  bool coalesce = true;    // TFP_COALESCE=0: every call runs alone (A/B)
  hipEvent_t null_in = nullptr, null_out = nullptr;  // (NullStreamOrder)
  ~tfp_engine() {
    if (qoff_ev) (void)hipEventDestroy(qoff_ev);
    if (null_in) (void)hipEventDestroy(null_in);
    if (null_out) (void)hipEventDestroy(null_out);
  }
};

namespace {

int fail(tfp_engine* e, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(tfp_engine* e, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (e) e->err.note(e, buf);
  return code;
}

#define HIPCHK(e, expr)                                                                          \
  do {                                                                                           \
    hipError_t _st = (expr);                                                                     \
    if (_st != hipSuccess)                                                                       \
      return fail((e), _st == hipErrorOutOfMemory ? TFP_E_NOMEM : TFP_E_HIP, "%s: %s", #expr,   \
                  hipGetErrorString(_st));                                                       \
  } while (0)

// A device-form call given no stream (NULL) runs on the engine's own stream, ordered after the work
// queued on the HIP null stream before the call and before the null stream's later work: the
// null stream is the default stream of torch and of CUDA-style callers, and the engine's stream
// is non-blocking, so without this a caller's default-stream producers and consumers (a torch
// copy, a gloo all_gather of the frame values) could race the engine's kernels. Two event
// records and two stream waits, no host wait.
class NullStreamOrder {
 public:
  NullStreamOrder(tfp_engine* e, void* stream) : e_(e), on_(stream == nullptr) {
    if (!on_) return;
    if (!e_->null_in && hipEventCreateWithFlags(&e_->null_in, hipEventDisableTiming) != hipSuccess) e_->null_in = nullptr;
    if (!e_->null_out && hipEventCreateWithFlags(&e_->null_out, hipEventDisableTiming) != hipSuccess) e_->null_out = nullptr;
    ok_ = e_->null_in && e_->null_out && hipEventRecord(e_->null_in, nullptr) == hipSuccess &&
          hipStreamWaitEvent(e_->stream, e_->null_in, 0) == hipSuccess;
  }
  bool ok() const { return !on_ || ok_; }
  ~NullStreamOrder() {
    if (on_ && ok_ && hipEventRecord(e_->null_out, e_->stream) == hipSuccess) (void)hipStreamWaitEvent(nullptr, e_->null_out, 0);
  }

 private:
  tfp_engine* e_;
  bool on_, ok_ = false;
};

// The device copy of the glibc log correction table (frame values == glibc's 10*log10|c|).
int ensure_logfix(tfp_engine* e) {
  if (e->logfix.n) return TFP_OK;
  const uint32_t* k;
  const double* v;
  int32_t n;
  log_fix_hash(&k, &v, &n);  // (the hashed form: one or two key loads per lookup on the device)
  if (n <= 0) return TFP_OK;
  const size_t slots = (size_t)1 << kLogFixHashBits;
  HIPCHK(e, e->logfix_key.reserve(sizeof(uint32_t) * slots));
  HIPCHK(e, e->logfix_val.reserve(sizeof(double) * slots));
  HIPCHK(e, hipMemcpyAsync(e->logfix_key.p, k, sizeof(uint32_t) * slots, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(e->logfix_val.p, v, sizeof(double) * slots, hipMemcpyHostToDevice, e->stream));
  // the keys present as a bitmap over the 2^24 reduced arguments (2 MiB)
  std::vector<uint32_t> bits(1u << 19, 0u);
  for (size_t j = 0; j < slots; j++)
    if (k[j] != kLogFixEmpty) bits[k[j] >> 5] |= 1u << (k[j] & 31);
  HIPCHK(e, e->logfix_bits.reserve(sizeof(uint32_t) * bits.size()));
  HIPCHK(e, hipMemcpyAsync(e->logfix_bits.p, bits.data(), sizeof(uint32_t) * bits.size(), hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  e->logfix = LogFix{e->logfix_key.as<uint32_t>(), e->logfix_val.as<double>(), n, 1, e->logfix_bits.as<uint32_t>()};
  return TFP_OK;
}

int ensure_tables(tfp_engine* e, int sr, const DspTables** out, bool* fixed8k = nullptr) {
  int rc0 = ensure_logfix(e);
  if (rc0) return rc0;
  auto it = e->tables.find(sr);
  if (it == e->tables.end()) {
    DspTables host;
    if (!build_tables(sr, &host)) return fail(e, TFP_E_ARG, "bad sample rate %d", sr);
    e->tables_fixed8k[sr] = DspTables_fixed8k(host);
    DevBuf& d = e->tables[sr];
    HIPCHK(e, d.reserve(sizeof(DspTables)));
    HIPCHK(e, hipMemcpyAsync(d.p, &host, sizeof host, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    it = e->tables.find(sr);
  }
  *out = it->second.as<DspTables>();
  if (fixed8k) *fixed8k = e->tables_fixed8k[sr];
  return TFP_OK;
}

// Clip layout: sample, frame and 16-frame-tile offsets.
void layout(const int64_t* offsets, int32_t nclips, std::vector<int64_t>& soff, std::vector<int64_t>& foff,
            std::vector<int32_t>& toff, std::vector<int32_t>* tclip = nullptr, int tile_frames = kFramesPerBlock) {
  soff.assign(offsets, offsets + nclips + 1);
  const int64_t base = soff[0];
  for (auto& v : soff) v -= base;
  foff.assign(nclips + 1, 0);
  toff.assign(nclips + 1, 0);
  for (int32_t c = 0; c < nclips; c++) {
    const int64_t nf = tfp_frame_count(soff[c + 1] - soff[c]);
    foff[c + 1] = foff[c] + nf;
    toff[c + 1] = toff[c] + (int32_t)((nf + tile_frames - 1) / tile_frames);
  }
  if (tclip) {
    tclip->assign(std::max<int32_t>(toff[nclips], 1), 0);
    for (int32_t c = 0; c < nclips; c++)
      for (int32_t t = toff[c]; t < toff[c + 1]; t++) (*tclip)[t] = c;
  }
}

int upload(tfp_engine* e, DevBuf& d, const void* h, size_t bytes, hipStream_t s = nullptr) {
  HIPCHK(e, d.reserve(bytes));
  if (bytes) HIPCHK(e, hipMemcpyAsync(d.p, h, bytes, hipMemcpyHostToDevice, s ? s : e->stream));
  return TFP_OK;
}

// The engine's device address of [p, p + n) if it lies inside one tfp_host_alloc buffer, else
// nullptr. Resolved on the engine's device (current here) once per buffer and cached.
const char* engine_host_ptr(tfp_engine* e, const void* p, size_t n) {
  uintptr_t base;
  uint64_t gen;
  if (!host_allocs().find(p, n, &base, &gen)) return nullptr;
  auto& slot = e->host_dev[base];
  if (slot.first != gen) {
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, reinterpret_cast<void*>(base), 0) != hipSuccess) {
      (void)hipGetLastError();
      e->host_dev.erase(base);
      return nullptr;  // (the call copies the samples instead)
    }
    slot = {gen, static_cast<char*>(d)};
  }
  return slot.second + (reinterpret_cast<uintptr_t>(p) - base);
}

// Fingerprint host samples (int16 PCM, or with f32 the fp32 values aubio_source produced):
// clip c is the lens[c] samples at ptrs[c] (the clips may lie anywhere: a coalesced batch gathers
// the queries of several callers); leaves micro/db on the device in e->micro / e->db.
// exact_q: the frame values (e->db) equal glibc's 10*log10|c| bit for bit (LogFix lookups); a
// coefs = 1 search needs only their truncation, which is exact either way.
int fingerprint_host(tfp_engine* e, const void* const* ptrs, const int64_t* lens, bool f32, int32_t nclips, int32_t sr,
                     int64_t* nframes_out, std::vector<int64_t>* foff_out, bool exact_q = true) {
  const size_t ss = f32 ? sizeof(float) : sizeof(int16_t);
  const DspTables* T;
  bool fx = false;
  int rc = ensure_tables(e, sr, &T, &fx);
  if (rc) return rc;
  std::vector<int64_t> foff(nclips + 1, 0);
  std::vector<int32_t> toff(nclips + 1, 0), tclip;
  // small batches at 8 kHz: 4-frame wave tiles (more waves, fewer passes per wave)
  bool small = false;
  for (int32_t c = 0; c < nclips; c++)
    if (lens[c] >= kDirectMaxSamples) fx = false;  // (the 8 kHz kernel's 32-bit buffer offsets)
  if (fx && !f32) {
    int64_t nf16 = 0;
    for (int32_t c = 0; c < nclips; c++) nf16 += (tfp_frame_count(lens[c]) + 15) / 16;
    small = nf16 <= 256;
  }
  const int tile_frames = fp_tile_frames(e->fpcfg, fx, f32, small);
  for (int32_t c = 0; c < nclips; c++) {
    const int64_t nfc = tfp_frame_count(lens[c]);
    foff[c + 1] = foff[c] + nfc;
    toff[c + 1] = toff[c] + (int32_t)((nfc + tile_frames - 1) / tile_frames);
  }
  tclip.assign(std::max<int32_t>(toff[nclips], 1), 0);
  for (int32_t c = 0; c < nclips; c++)
    for (int32_t t = toff[c]; t < toff[c + 1]; t++) tclip[t] = c;
  const int64_t nf = foff[nclips];
  HIPCHK(e, e->micro.reserve(sizeof(int32_t) * 2 * (nf + 1)));
  HIPCHK(e, e->db.reserve(sizeof(double) * 2 * (nf + 1)));
  // Where the samples come from:
  //  - in place: every clip lies in a tfp_host_alloc buffer (the shim's WAV reads): the kernel reads
  //    them through their device mapping, clip c at sample offset sbeg[c] from the lowest address;
  //  - else packed (sbeg = prefix sums): into the pinned staging (small calls) or the device buffer.
  // Throughput batches that are one contiguous buffer keep the DMA copy into HBM.
  bool contiguous = true;
  int64_t ns = 0;
  for (int32_t c = 0; c < nclips; c++) {
    ns += lens[c];
    if (c + 1 < nclips && static_cast<const char*>(ptrs[c]) + ss * lens[c] != ptrs[c + 1]) contiguous = false;
  }
  std::vector<int64_t> sbeg(nclips + 1, 0), send(nclips + 1, 0);
  const char* base_dev = nullptr;
  bool in_place = ns > 0 && (small || !contiguous);
  if (in_place) {
    std::vector<const char*> dv(nclips, nullptr);
    for (int32_t c = 0; c < nclips && in_place; c++) {
      if (!lens[c]) continue;
      dv[c] = engine_host_ptr(e, ptrs[c], ss * lens[c]);
      in_place = dv[c] != nullptr;
      if (in_place && (!base_dev || dv[c] < base_dev)) base_dev = dv[c];
    }
    for (int32_t c = 0; c < nclips && in_place; c++) {
      const int64_t d = lens[c] ? (int64_t)(dv[c] - base_dev) : 0;
      in_place = d % (int64_t)ss == 0;
      sbeg[c] = d / (int64_t)ss;
      send[c] = sbeg[c] + lens[c];
    }
  }
  if (!in_place) {
    for (int32_t c = 0; c < nclips; c++) {
      sbeg[c + 1] = sbeg[c] + lens[c];
      send[c] = sbeg[c + 1];
    }
  }
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t b_pcm = in_place ? 0 : al(ss * ns), b_sb = al(sizeof(int64_t) * nclips),
               b_fo = al(sizeof(int64_t) * foff.size()), b_to = al(sizeof(int32_t) * toff.size()),
               b_tc = al(sizeof(int32_t) * tclip.size());
  const size_t lay = 2 * b_sb + b_fo + b_to + b_tc, total = b_pcm + lay;
  auto pack_layout = [&](char* h) {
    memcpy(h, sbeg.data(), sizeof(int64_t) * nclips);
    memcpy(h + b_sb, send.data(), sizeof(int64_t) * nclips);
    memcpy(h + 2 * b_sb, foff.data(), sizeof(int64_t) * foff.size());
    memcpy(h + 2 * b_sb + b_fo, toff.data(), sizeof(int32_t) * toff.size());
    memcpy(h + 2 * b_sb + b_fo + b_to, tclip.data(), sizeof(int32_t) * tclip.size());
  };
  auto pack_samples = [&](char* h) {
    if (contiguous) {
      if (ns) memcpy(h, ptrs[0], ss * ns);
      return;
    }
    for (int32_t c = 0; c < nclips; c++)
      if (lens[c]) memcpy(h + ss * sbeg[c], ptrs[c], ss * lens[c]);
  };
  const void* d_pcm;
  const char* lay_d;
  if (total <= ((size_t)8 << 20)) {
    // small call: pack every array into pinned staging, one H2D copy. The 4-frame-tile calls
    // (a query, batch-1 latency) skip the copy: the kernel reads the mapped, coherent staging in
    // place (a copy plus its hand-off to the kernel cost ~16 us before the first kernel started).
    // Every caller waits for e->stream before it returns and then clears stage_pending, so the
    // staging buffer is free here; after an error return the stream is drained first.
    if (e->stage_pending) HIPCHK(e, hipStreamSynchronize(e->stream));
    const bool zero_copy = small || in_place;
    char* h;
    if (zero_copy) {
      HIPCHK(e, e->zstage.reserve(total, hipHostMallocMapped | hipHostMallocCoherent));
      if (e->zstage.p != e->zstage_host) {
        HIPCHK(e, hipHostGetDevicePointer(reinterpret_cast<void**>(&e->zstage_dev), e->zstage.p, 0));
        e->zstage_host = e->zstage.p;
      }
      h = e->zstage.as<char>();
    } else {
      HIPCHK(e, e->hstage.reserve(total));
      HIPCHK(e, e->dstage.reserve(total));
      h = e->hstage.as<char>();
    }
    if (!in_place) pack_samples(h);
    pack_layout(h + b_pcm);
    if (!zero_copy) HIPCHK(e, hipMemcpyAsync(e->dstage.p, h, total, hipMemcpyHostToDevice, e->stream));
    e->stage_pending = true;
    char* d = zero_copy ? e->zstage_dev : e->dstage.as<char>();
    d_pcm = in_place ? base_dev : d;
    lay_d = d + b_pcm;  // the layout arrays' device address
    if (zero_copy) {
      // The tile layout is read first and in a dependent chain (tile -> clip -> its bounds -> the
      // PCM address): keep it in device memory. It depends only on the query lengths (and, in
      // place, the buffers' relative positions), so it is uploaded only when it changes (from the
      // pinned staging; the PCM stays in place).
      if (e->zlayout_host.size() != lay || memcmp(e->zlayout_host.data(), h + b_pcm, lay) != 0) {
        HIPCHK(e, e->zlayout.reserve(lay));
        HIPCHK(e, hipMemcpyAsync(e->zlayout.p, h + b_pcm, lay, hipMemcpyHostToDevice, e->stream));
        e->zlayout_host.assign(h + b_pcm, h + total);
      }
      lay_d = e->zlayout.as<char>();
    }
  } else {
    std::vector<char> hl(lay);
    pack_layout(hl.data());
    if ((rc = upload(e, e->soff, hl.data(), lay))) return rc;
    if (in_place) {
      d_pcm = base_dev;
    } else {
      HIPCHK(e, e->pcm.reserve(ss * ns));
      if (contiguous) {
        if ((rc = upload(e, e->pcm, ptrs[0], ss * ns))) return rc;
      } else {
        for (int32_t c = 0; c < nclips; c++)
          if (lens[c])
            HIPCHK(e, hipMemcpyAsync(e->pcm.as<char>() + ss * sbeg[c], ptrs[c], ss * lens[c], hipMemcpyHostToDevice,
                                     e->stream));
      }
      d_pcm = e->pcm.p;
    }
    lay_d = e->soff.as<char>();
    HIPCHK(e, hipStreamSynchronize(e->stream));  // (hl is released on return)
  }
  const int64_t* d_sbeg = reinterpret_cast<const int64_t*>(lay_d);
  const int64_t* d_send = reinterpret_cast<const int64_t*>(lay_d + b_sb);
  const int64_t* d_foff = reinterpret_cast<const int64_t*>(lay_d + 2 * b_sb);
  const int32_t* d_toff = reinterpret_cast<const int32_t*>(lay_d + 2 * b_sb + b_fo);
  const int32_t* d_tclip = reinterpret_cast<const int32_t*>(lay_d + 2 * b_sb + b_fo + b_to);
  if (f32)
    HIPCHK(e, launch_fingerprint_f32(e->fpcfg, T, static_cast<const float*>(d_pcm), d_sbeg, d_send, d_foff, d_toff, d_tclip,
                                     toff[nclips], e->micro.as<int32_t>(), e->db.as<double>(), e->stream,
                                     exact_q ? e->logfix : LogFix{}));
  else
    HIPCHK(e, launch_fingerprint(e->fpcfg, T, fx, tile_frames, static_cast<const int16_t*>(d_pcm), d_sbeg, d_send, d_foff,
                                 d_toff, d_tclip, toff[nclips], nf, e->micro.as<int32_t>(), e->db.as<double>(),
                                 e->stream, exact_q ? e->logfix : LogFix{}, nclips == 1 && sbeg[0] == 0 ? send[0] : -1));
  *nframes_out = nf;
  if (foff_out) *foff_out = foff;
  return TFP_OK;
}

// The clips of one buffer at sample offsets offsets[0..nclips] as (pointer, length) lists.
void split_offsets(const void* pcm, size_t ss, const int64_t* offsets, int32_t nclips, std::vector<const void*>* ptrs,
                   std::vector<int64_t>* lens) {
  ptrs->resize(nclips);
  lens->resize(nclips);
  for (int32_t c = 0; c < nclips; c++) {
    (*ptrs)[c] = static_cast<const char*>(pcm) + ss * offsets[c];
    (*lens)[c] = offsets[c + 1] - offsets[c];
  }
}

int copy_frames_out(tfp_engine* e, int64_t nf, const std::vector<int64_t>& foff, tfp_frame* out) {
  std::vector<int32_t> m(2 * nf);
  std::vector<double> d(2 * nf);
  if (nf) {
    HIPCHK(e, hipMemcpyAsync(m.data(), e->micro.p, sizeof(int32_t) * 2 * nf, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(d.data(), e->db.p, sizeof(double) * 2 * nf, hipMemcpyDeviceToHost, e->stream));
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  e->stage_pending = false;
  size_t c = 0;
  for (int64_t g = 0; g < nf; g++) {
    while (c + 1 < foff.size() && foff[c + 1] <= g) c++;
    out[g].frame_idx = (int32_t)(g - foff[c]);
    out[g].m1 = m[2 * g];
    out[g].m2 = m[2 * g + 1];
    out[g].reserved = 0;
    out[g].q1 = d[2 * g];
    out[g].q2 = d[2 * g + 1];
  }
  return TFP_OK;
}

// ---- index -------------------------------------------------------------------------------

int stage_reserve(tfp_engine* e, int64_t extra) {
  const int64_t need = e->n_staged + extra;
  if (need <= e->cap_staged) return TFP_OK;
  int64_t cap = std::max<int64_t>(need, std::max<int64_t>(1 << 16, e->cap_staged * 2));
  DevBuf n1, n2, nc;
  HIPCHK(e, n1.reserve(sizeof(int32_t) * cap));
  HIPCHK(e, n2.reserve(sizeof(int32_t) * cap));
  HIPCHK(e, nc.reserve(sizeof(int32_t) * cap));
  if (e->n_staged) {
    HIPCHK(e, hipMemcpyAsync(n1.p, e->st_m1.p, sizeof(int32_t) * e->n_staged, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(n2.p, e->st_m2.p, sizeof(int32_t) * e->n_staged, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(nc.p, e->st_clip.p, sizeof(int32_t) * e->n_staged, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  std::swap(e->st_m1.p, n1.p); std::swap(e->st_m1.bytes, n1.bytes);
  std::swap(e->st_m2.p, n2.p); std::swap(e->st_m2.bytes, n2.bytes);
  std::swap(e->st_clip.p, nc.p); std::swap(e->st_clip.bytes, nc.bytes);
  e->cap_staged = cap;
  return TFP_OK;
}

int new_clip(tfp_engine* e, const char* uuid, int64_t nrows, int64_t off, int32_t* id) {
  if (!uuid || !*uuid || strlen(uuid) >= 64) return fail(e, TFP_E_ARG, "bad uuid");
  if (e->by_uuid.count(uuid)) return fail(e, TFP_E_EXISTS, "uuid %s already indexed", uuid);
  Clip c;
  c.uuid = uuid;
  c.nrows = nrows;
  c.off = off;
  *id = (int32_t)e->clips.size();
  e->clips.push_back(c);
  e->by_uuid[uuid] = *id;
  e->live_rows += nrows;
  e->dirty = true;
  return TFP_OK;
}

// Staging rows of live clips, moved down over the rows of removed clips (clip ids and row order
// kept): one block per run of rows.
__global__ void compact_rows_kernel(const int64_t* __restrict__ runs /*[n][3]: src, dst, len*/, const int32_t* m1,
                                    const int32_t* m2, const int32_t* cl, int32_t* o1, int32_t* o2, int32_t* oc) {
  const int64_t src = runs[3 * blockIdx.x], dst = runs[3 * blockIdx.x + 1], len = runs[3 * blockIdx.x + 2];
  for (int64_t i = threadIdx.x; i < len; i += blockDim.x) {
    o1[dst + i] = m1[src + i];
    o2[dst + i] = m2[src + i];
    oc[dst + i] = cl[src + i];
  }
}

// Drops the staging rows of removed clips once they outnumber a quarter of the live rows (else
// delete/re-enrol cycles grow the staging area, and every rebuild sorts the dead rows too).
int compact_staging(tfp_engine* e) {
  int64_t live = 0;
  for (const auto& c : e->clips)
    if (c.alive) live += c.nrows;
  const int64_t dead = e->n_staged - live;
  if (dead <= std::max<int64_t>(1 << 16, live / 4)) return TFP_OK;
  // The new layout is built aside and written into e->clips only once the copy has succeeded: a
  // failure below (allocation, launch) leaves the staging rows and every clip's offset as they were.
  std::vector<int64_t> runs, new_off(e->clips.size(), 0);
  int64_t dst = 0;
  for (size_t i = 0; i < e->clips.size(); i++) {
    const Clip& c = e->clips[i];
    if (!c.alive || !c.nrows) continue;
    const size_t nr = runs.size();
    if (nr && runs[nr - 3] + runs[nr - 1] == c.off && runs[nr - 2] + runs[nr - 1] == dst) runs[nr - 1] += c.nrows;
    else runs.insert(runs.end(), {c.off, dst, c.nrows});
    new_off[i] = dst;
    dst += c.nrows;
  }
  DevBuf n1, n2, nc, d_runs;
  const int64_t cap = std::max<int64_t>(live, 1 << 16);
  HIPCHK(e, n1.reserve(sizeof(int32_t) * cap));
  HIPCHK(e, n2.reserve(sizeof(int32_t) * cap));
  HIPCHK(e, nc.reserve(sizeof(int32_t) * cap));
  const int32_t nruns = (int32_t)(runs.size() / 3);
  if (e->fail_compact > 0) {  // TFP_TEST_FAIL_COMPACT: an allocation failure here, for the tests
    e->fail_compact--;
    return fail(e, TFP_E_NOMEM, "compact_staging: injected allocation failure");
  }
  if (nruns) {
    int rc = upload(e, d_runs, runs.data(), sizeof(int64_t) * runs.size());
    if (rc) return rc;
    hipLaunchKernelGGL(compact_rows_kernel, dim3(nruns), dim3(256), 0, e->stream, d_runs.as<int64_t>(),
                       e->st_m1.as<int32_t>(), e->st_m2.as<int32_t>(), e->st_clip.as<int32_t>(), n1.as<int32_t>(),
                       n2.as<int32_t>(), nc.as<int32_t>());
    HIPCHK(e, hipGetLastError());
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  std::swap(e->st_m1.p, n1.p); std::swap(e->st_m1.bytes, n1.bytes);
  std::swap(e->st_m2.p, n2.p); std::swap(e->st_m2.bytes, n2.bytes);
  std::swap(e->st_clip.p, nc.p); std::swap(e->st_clip.bytes, nc.bytes);
  for (size_t i = 0; i < e->clips.size(); i++) {
    Clip& c = e->clips[i];
    if (c.alive) c.off = new_off[i];
    else c.nrows = 0, c.off = 0;
  }
  e->n_staged = live;
  e->cap_staged = cap;
  return TFP_OK;
}

// Live clips in uuid order (the columns: the tie-break order of SQLite's result sort) and each
// clip's rank (-1 when dead). Incremental: the previous build's order with the clips added since
// merged in (no re-sort of every uuid).
// Returns true for an update that only adds (no clip of the last build removed) with at most
// kMergeBreaks new uuids placed before an old one: the old columns are then col_clip as it stands
// (no alive filter), *brk is the merge's column map (old col c -> c + breakpoints <= c) and rank
// holds the new clips' ranks only (the merge and the device rank table read no other; skipping
// the scatter over every clip is most of an enrolment's host time at 100k clips).
bool live_order(const tfp_engine* e, bool incremental, std::vector<int32_t>* live, std::vector<int32_t>* rank,
                MergeBreaks* brk) {
  auto by_uuid = [&](int32_t a, int32_t b) { return e->clips[a].uuid < e->clips[b].uuid; };
  live->clear();
  brk->n = -1;
  if (incremental) {
    const bool add_only = !e->removed_built;
    std::vector<int32_t> kept, add;
    if (!add_only) {
      kept.reserve(e->col_clip.size());
      for (int32_t c : e->col_clip)
        if (e->clips[c].alive) kept.push_back(c);
    }
    const std::vector<int32_t>& old = add_only ? e->col_clip : kept;
    for (int32_t i = (int32_t)e->built_clips; i < (int32_t)e->clips.size(); i++)
      if (e->clips[i].alive) add.push_back(i);
    std::sort(add.begin(), add.end(), by_uuid);
    // each new uuid's place by binary search, the old runs between them copied whole: log C
    // string compares per new clip instead of a linear merge (each compare is two uuid strings
    // on the heap, a cache miss apiece: ~10 ms at 100k clips)
    live->reserve(old.size() + add.size());
    std::vector<int32_t> at_col(add.size());
    int32_t before_old = 0;  // new uuids placed before some old one
    auto from = old.begin();
    for (size_t j = 0; j < add.size(); j++) {
      const auto at = std::lower_bound(from, old.end(), add[j], by_uuid);
      live->insert(live->end(), from, at);
      live->push_back(add[j]);
      from = at;
      at_col[j] = (int32_t)(at - old.begin());
      before_old += at != old.end();
    }
    live->insert(live->end(), from, old.end());
    if (add_only && before_old <= kMergeBreaks) {
      brk->n = 0;
      for (int32_t p : at_col)
        if ((size_t)p < old.size()) brk->p[brk->n++] = p;
      rank->assign(std::max<size_t>(e->clips.size(), 1), -1);
      for (size_t j = 0; j < add.size(); j++) (*rank)[add[j]] = at_col[j] + (int32_t)j;
      return true;
    }
  } else {
    for (int32_t i = 0; i < (int32_t)e->clips.size(); i++)
      if (e->clips[i].alive) live->push_back(i);
    std::sort(live->begin(), live->end(), by_uuid);
  }
  rank->assign(std::max<size_t>(e->clips.size(), 1), -1);
  for (size_t r = 0; r < live->size(); r++) (*rank)[(*live)[r]] = (int32_t)r;
  return false;
}

// Staging rows [b, b + n) sorted by m1 with the rows that cannot match (dead clip or NULL max1,
// key INT32_MAX) last: m1 in keys_b, m2 in vals_a, col in keys_a; the count of the others (the
// first ones) in e->cnt. Asynchronous: the merge runs over all n rows (those with key INT32_MAX
// land after every index row, past the new row count) and the count is read with its result,
// one host wait per update instead of two.
int sort_staged_rows(tfp_engine* e, int64_t b, int64_t n) {
  HIPCHK(e, e->keys_a.reserve(sizeof(int32_t) * (n + 1)));
  HIPCHK(e, e->keys_b.reserve(sizeof(int32_t) * (n + 1)));
  HIPCHK(e, e->vals_a.reserve(sizeof(int32_t) * (n + 1)));
  HIPCHK(e, e->vals_b.reserve(sizeof(int32_t) * (n + 1)));
  HIPCHK(e, launch_index_keys(e->st_m1.as<int32_t>() + b, e->st_clip.as<int32_t>() + b, e->rank_of_clip.as<int32_t>(), n,
                              e->keys_a.as<int32_t>(), e->vals_a.as<int32_t>(), e->stream));
  size_t tb = 0;
  HIPCHK(e, radix_sort_pairs(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, n, e->stream));
  HIPCHK(e, e->sort_tmp.reserve(tb));
  HIPCHK(e, radix_sort_pairs(e->sort_tmp.p, &tb, e->keys_a.as<int32_t>(), e->keys_b.as<int32_t>(),
                             e->vals_a.as<int32_t>(), e->vals_b.as<int32_t>(), n, e->stream));
  HIPCHK(e, e->cnt.reserve(sizeof(int64_t)));
  HIPCHK(e, launch_count_below(e->keys_b.as<int32_t>(), n, INT32_MAX, e->cnt.as<int64_t>(), e->stream));
  HIPCHK(e, launch_index_gather(e->vals_b.as<int32_t>(), e->st_m2.as<int32_t>() + b, e->st_clip.as<int32_t>() + b,
                                e->rank_of_clip.as<int32_t>(), n, e->vals_a.as<int32_t>(), e->keys_a.as<int32_t>(), e->stream));
  return TFP_OK;
}

// e->cnt (sort_staged_rows' row count) after the work queued on e->stream. Synchronous.
int read_sorted_count(tfp_engine* e, int64_t* valid) {
  HIPCHK(e, hipMemcpyAsync(valid, e->cnt.p, sizeof *valid, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return TFP_OK;
}

// Index update without a full re-sort (tfp_index.hip): the rows staged since the last build are
// sorted alone and merged into (m1s, m2s, cols) in one pass that also drops removed clips' rows
// and renumbers the columns around the inserted / removed uuids. Commits nothing on failure.
// fast_brk: live_order's column map of an update that only adds (rank then holds the new clips'
// ranks only), else nullptr (the map from rank over every old column).
int merge_index(tfp_engine* e, const std::vector<int32_t>& rank, const MergeBreaks* fast_brk, int32_t new_cols,
                bool* carried) {
  *carried = false;
  const int64_t b = e->built_staged, n = e->n_staged - e->built_staged;
  bool removed = false;
  MergeBreaks brk;
  int rc = TFP_OK;
  if (fast_brk) {
    brk = *fast_brk;
  } else {
    // old column -> new column (-1: the clip was removed)
    std::vector<int32_t> remap(std::max<size_t>(e->col_clip.size(), 1), -1);
    for (size_t c = 0; c < e->col_clip.size(); c++) {
      remap[c] = rank[e->col_clip[c]];
      removed |= remap[c] < 0;
    }
    // without removals remap[c] - c only steps up (uuid order is kept): its breakpoints, when few
    brk.n = removed ? -1 : 0;
    for (size_t c = 0, shift = 0; brk.n >= 0 && c < e->col_clip.size(); c++)
      while ((size_t)remap[c] - c > shift) {
        if (brk.n == kMergeBreaks) {
          brk.n = -1;
          break;
        }
        brk.p[brk.n++] = (int32_t)c;
        shift++;
      }
    if (brk.n < 0 && (rc = upload(e, e->remap, remap.data(), sizeof(int32_t) * remap.size())))  // (only when gathered)
      return rc;
  }
  // (e.g. new tie-break keys only: the rows and their columns are unchanged; a clip without rows
  // placed before an old one still renumbers the columns)
  if (n == 0 && !removed && brk.n == 0) return TFP_OK;
  if (n > 0 && (rc = sort_staged_rows(e, b, n))) return rc;
  const int64_t R = e->nrows;
  HIPCHK(e, e->m1s_b.reserve_grow(sizeof(int32_t) * (R + n + 1)));
  HIPCHK(e, e->m2s_b.reserve_grow(sizeof(int32_t) * (R + n + 1)));
  HIPCHK(e, e->cols_b.reserve_grow(sizeof(int32_t) * (R + n + 1)));
  int64_t kept = R;
  HIPCHK(e, launch_merge_update(e->m1s.as<int32_t>(), e->m2s.as<int32_t>(), e->cols.as<int32_t>(), R, e->remap.as<int32_t>(),
                                removed, brk, e->keys_b.as<int32_t>(), e->vals_a.as<int32_t>(), e->keys_a.as<int32_t>(), n,
                                &e->merge, e->m1s_b.as<int32_t>(), e->m2s_b.as<int32_t>(), e->cols_b.as<int32_t>(), &kept,
                                e->stream));
  int64_t valid = 0;
  if (n > 0 && (rc = read_sorted_count(e, &valid))) return rc;
  HIPCHK(e, hipStreamSynchronize(e->stream));
  std::swap(e->m1s.p, e->m1s_b.p); std::swap(e->m1s.bytes, e->m1s_b.bytes);
  std::swap(e->m2s.p, e->m2s_b.p); std::swap(e->m2s.bytes, e->m2s_b.bytes);
  std::swap(e->cols.p, e->cols_b.p); std::swap(e->cols.bytes, e->cols_b.bytes);
  e->nrows = kept + valid;
  // The clip order (when built) through the same update: its old rows renumbered, the new rows
  // inserted (tfp_index.hpp). Best effort: on failure it is rebuilt when next needed.
  if (e->o_valid) {
    e->o_valid = false;
    auto by_uuid = [&](int32_t a, int32_t c) { return e->clips[a].uuid < e->clips[c].uuid; };
    std::vector<int32_t> add;
    for (int32_t i = (int32_t)e->built_clips; i < (int32_t)e->clips.size(); i++)
      if (e->clips[i].alive) add.push_back(i);
    std::sort(add.begin(), add.end(), by_uuid);
    const int32_t D = (int32_t)add.size();
    std::vector<int32_t> nca(2 * (size_t)std::max(D, 1));  // new columns, then their insertion points among the old columns
    for (int32_t j = 0; j < D; j++) {
      nca[j] = rank[add[j]];
      nca[D + j] = fast_brk ? rank[add[j]] - j
                            : (int32_t)(std::lower_bound(e->col_clip.begin(), e->col_clip.end(), add[j], by_uuid) - e->col_clip.begin());
    }
    int64_t orows = 0;
    const size_t on = (size_t)std::max<int64_t>(e->o_rows + valid, 1);
    if ((!D || upload(e, e->o_newcol, nca.data(), sizeof(int32_t) * nca.size()) == TFP_OK) &&
        e->o_key_b.reserve_grow(sizeof(unsigned long long) * on) == hipSuccess &&
        e->o_m1_b.reserve_grow(sizeof(int32_t) * on) == hipSuccess &&
        launch_order_merge(e->o_key.as<unsigned long long>(), e->o_m1.as<int32_t>(), e->o_rows, e->remap.as<int32_t>(), removed,
                           brk, e->keys_b.as<int32_t>(), e->vals_a.as<int32_t>(), e->keys_a.as<int32_t>(), valid,
                           e->o_newcol.as<int32_t>(), e->o_newcol.as<int32_t>() + D, D, &e->merge, &e->o_merge,
                           e->o_key_b.as<unsigned long long>(), e->o_m1_b.as<int32_t>(), &orows, e->stream) == hipSuccess &&
        hipStreamSynchronize(e->stream) == hipSuccess && orows == e->nrows) {  // (nca is read by then)
      e->o_key.swap_with(e->o_key_b);
      e->o_m1.swap_with(e->o_m1_b);
      e->o_rows = orows;
      e->o_valid = true;
      e->n_order_merges++;
    } else {
      (void)hipGetLastError();
    }
  }
  // The small path's key ranges and bitsets, carried to the merged index at their tolerance
  // instead of rebuilt from every box row (tfp_index.hpp): the ranges are searched again, every
  // surviving column's bits move to its new column (removed clips' and an index delta's columns
  // dropped: the delta's clips are among the new rows), then the new rows' bits are set. Best
  // effort: on any failure the bitsets are rebuilt when next needed.
  const int32_t W = key_bits_words(new_cols);
  const int32_t Cm = (int32_t)e->col_clip.size();
  if (e->rng_valid && e->key_bits_valid && e->key_bits_cols >= Cm &&
      e->key_bits.bytes >= sizeof(uint32_t) * (size_t)kKeyRange * key_bits_words(e->key_bits_cols)) {
    hipStream_t s = e->stream;
    bool ok = launch_key_ranges_all(e->m1s.as<int32_t>(), e->nrows, e->rng_tol, e->rng_all.as<int64_t>(), s) == hipSuccess &&
              e->key_bits_b.reserve(sizeof(uint32_t) * (size_t)kKeyRange * W) == hipSuccess &&
              launch_key_bits_remap(e->key_bits.as<uint32_t>(), key_bits_words(e->key_bits_cols), Cm,
                                    brk.n >= 0 ? nullptr : e->remap.as<int32_t>(), brk, e->key_bits_b.as<uint32_t>(), W,
                                    s) == hipSuccess;
    if (ok) {
      std::swap(e->key_bits.p, e->key_bits_b.p);
      std::swap(e->key_bits.bytes, e->key_bits_b.bytes);
    }
    if (ok && valid > 0)
      ok = launch_key_bits_add(e->rng_all.as<int64_t>(), e->m1s.as<int32_t>(), e->keys_b.as<int32_t>(), e->keys_a.as<int32_t>(),
                               valid, W, e->key_bits.as<uint32_t>(), s) == hipSuccess;
    if (!ok) (void)hipGetLastError();
    *carried = ok;
  }
  return TFP_OK;
}

int full_index(tfp_engine* e);

int delta_update(tfp_engine* e);
bool delta_eligible(const tfp_engine* e);

int rebuild(tfp_engine* e) {
  if (!e->dirty) return TFP_OK;
  if (delta_eligible(e)) return delta_update(e);
  int rc;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  // Incremental (merge) when there is an index to merge into, the new rows are few next to it, and
  // the staging area needs no compaction (the staged rows since the last build are then exactly
  // rows [built_staged, n_staged)); otherwise the full build.
  const int64_t live_rows = e->live_rows;
  const int64_t dead = e->n_staged - live_rows, fresh = e->n_staged - e->built_staged;
  const bool incremental = e->built && !e->force_full && fresh <= std::max<int64_t>(e->nrows / 2, 0) &&
                           dead <= std::max<int64_t>(1 << 16, live_rows / 4) && e->n_staged < INT32_MAX;
  if (!incremental) {
    e->built = false;  // a failure below leaves the next attempt a full build as well
    if ((rc = compact_staging(e))) return rc;
    // the sort and the index rows use 32-bit row numbers
    if (e->n_staged >= INT32_MAX)
      return fail(e, TFP_E_CAPACITY, "%lld staged rows (limit 2^31 - 1)", (long long)e->n_staged);
  }
  std::vector<int32_t> live, rank;
  MergeBreaks brk;
  const bool add_only = live_order(e, incremental, &live, &rank, &brk);
  const double t_order = ms_since(t0);
  const size_t nkeys = std::max<size_t>(live.size(), 1);
  std::vector<int32_t> tiekey;  // column -> tie-break key: with an override every column, else the identity's new tail
  // key -> column: the identity without an override (the key is the uuid rank), so no map is built
  // (a 100k-entry hash map was most of an enrolment's host time); with one, a map that also
  // rejects a key given twice
  std::unordered_map<int32_t, int32_t> key_col;
  const bool ovr = !e->tiebreak_override.empty();
  if (ovr) {
    key_col.reserve(live.size());
    tiekey.assign(nkeys, 0);
  }
  for (size_t r = 0; ovr && r < live.size(); r++) {
    const int32_t clip = live[r];
    // With an override every live clip needs its own key (a clip added after the override would
    // otherwise take its local rank, which can equal another shard's global key).
    if ((size_t)clip >= e->tiebreak_override.size())
      return fail(e, TFP_E_ARG, "clip %s was added after tfp_index_set_tiebreak: set the tie-break keys again",
                  e->clips[clip].uuid.c_str());
    const int32_t k = e->tiebreak_override[clip];
    if (!key_col.emplace(k, (int32_t)r).second) return fail(e, TFP_E_ARG, "tie-break key %d given to two live clips", k);
    tiekey[r] = k;
  }
  // Device copies, only the parts that changed (two 400 KB pageable uploads were a tenth of an
  // enrolment at 100k clips): a merge reads the ranks of the clips added since the last build
  // only (their staged rows), and identity tie keys keep their prefix.
  {
    const size_t rb = incremental ? std::min(e->built_clips, rank.size()) : 0;
    HIPCHK(e, e->rank_of_clip.reserve_grow(sizeof(int32_t) * rank.size()));
    HIPCHK(e, hipMemcpyAsync(e->rank_of_clip.as<int32_t>() + rb, rank.data() + rb, sizeof(int32_t) * (rank.size() - rb),
                             hipMemcpyHostToDevice, e->stream));
    const void* before = e->tiekey.p;
    const int64_t ident = e->tiekey_ident;
    e->tiekey_ident = -1;
    HIPCHK(e, e->tiekey.reserve_grow(sizeof(int32_t) * nkeys));
    const size_t tb = !ovr && e->tiekey.p == before && ident > 0 ? std::min<size_t>((size_t)ident, nkeys) : 0;
    if (!ovr) {
      tiekey.resize(nkeys - tb);
      std::iota(tiekey.begin(), tiekey.end(), (int32_t)tb);
    }
    if (nkeys > tb)
      HIPCHK(e, hipMemcpyAsync(e->tiekey.as<int32_t>() + tb, tiekey.data(), sizeof(int32_t) * (nkeys - tb),
                               hipMemcpyHostToDevice, e->stream));
    if (!ovr) e->tiekey_ident = (int64_t)nkeys;
  }
  const double t_keys = ms_since(t0);
  bool carried = false;
  if (incremental) {
    if ((rc = merge_index(e, rank, add_only ? &brk : nullptr, (int32_t)live.size(), &carried))) return rc;
    e->n_merges++;
  } else {
    e->nrows = 0;
    e->o_valid = false;  // (the clip order is rebuilt from the new index when next needed)
    if ((rc = full_index(e))) return rc;
    e->n_full_builds++;
  }
  e->ncols = (int32_t)live.size();
  e->col_clip = std::move(live);
  e->delta_clip.clear();  // (every clip is in the main index now)
  e->delta_at.clear();
  e->delta_col0 = e->ncols;
  e->delta_rows = 0;
  e->key_col = std::move(key_col);
  e->key_col_delta.clear();
  e->ovr_main_stale = !ovr;  // (with an override: its keys for these columns are on the device now)
  e->key_identity = !ovr;
  e->built = true;
  e->built_clips = e->clips.size();
  e->built_staged = e->n_staged;
  e->removed_built = false;
  e->dirty = false;
  e->index_version++;  // (other tolerances' cached ranges and bitsets are for the previous index)
  e->main_version++;
  e->rng_valid = carried;  // the key-range and clip-set caches follow the index (merge_index may carry the ranges and bitsets)
  e->key_bits_valid = carried && e->key_bits_valid;
  if (e->key_bits_valid) e->key_bits_cols = e->ncols;
  e->cell_fresh = false;
  if (e->dbg_index)
    fprintf(stderr, "[tfp] index %s: %lld rows, %d clips; order %.3f keys %.3f total %.3f ms\n",
            incremental ? "merge" : "full build", (long long)e->nrows, e->ncols, t_order, t_keys, ms_since(t0));
  return TFP_OK;
}

// The full build: every staged row of a live clip, radix-sorted by m1 (the sorted arrays become
// the index buffers).
int full_index(tfp_engine* e) {
  const int64_t n = e->n_staged;
  int64_t valid = 0;
  if (n > 0) {
    int rc = sort_staged_rows(e, 0, n);
    if (!rc) rc = read_sorted_count(e, &valid);
    if (rc) return rc;
    std::swap(e->m1s.p, e->keys_b.p); std::swap(e->m1s.bytes, e->keys_b.bytes);
    std::swap(e->m2s.p, e->vals_a.p); std::swap(e->m2s.bytes, e->vals_a.bytes);
    std::swap(e->cols.p, e->keys_a.p); std::swap(e->cols.bytes, e->keys_a.bytes);
  } else {
    HIPCHK(e, e->m1s.reserve(4));
    HIPCHK(e, e->m2s.reserve(4));
    HIPCHK(e, e->cols.reserve(4));
  }
  e->nrows = valid;
  return TFP_OK;
}

// The active tolerance's ranges and bitsets exchanged with slot t's.
void swap_active(tfp_engine* e, TolSlot& t) {
  e->rng_all.swap_with(t.rng_all);
  e->key_bits.swap_with(t.key_bits);
  std::swap(e->rng_tol, t.tol);
  std::swap(e->rng_valid, t.rng_valid);
  std::swap(e->key_bits_valid, t.bits_valid);
  std::swap(e->key_bits_cols, t.bits_cols);
}

// Row ranges of every key's box at tolerance tole, cached per index version and tolerance: the
// active tolerance's, and up to kTolSlots others (a search at another tolerance moves the active
// ones into the least recently used slot, and takes its tolerance's from a slot when it is there).
int ensure_ranges(tfp_engine* e, double tole, hipStream_t s) {
  if (e->rng_valid && memcmp(&e->rng_tol, &tole, sizeof tole) == 0) return TFP_OK;
  TolSlot* hit = nullptr;
  TolSlot* victim = &e->tol_lru[0];
  for (TolSlot& t : e->tol_lru) {
    if (t.version != e->index_version) t.rng_valid = t.bits_valid = false;
    if (t.rng_valid && memcmp(&t.tol, &tole, sizeof tole) == 0) hit = &t;
    // the victim: a slot holding nothing valid, else the least recently used
    if (t.rng_valid != victim->rng_valid ? !t.rng_valid : t.used < victim->used) victim = &t;
  }
  if (hit) {
    swap_active(e, *hit);  // (the previous active ones, valid or not, into the slot)
    hit->version = e->index_version;
    hit->used = ++e->tol_clock;
    return TFP_OK;
  }
  if (e->rng_valid) {
    swap_active(e, *victim);  // the active ones kept; their buffers' old contents reused below
    victim->version = e->index_version;
    victim->used = ++e->tol_clock;
  }
  HIPCHK(e, e->rng_all.reserve(sizeof(int64_t) * 2 * kKeyRange));
  HIPCHK(e, launch_key_ranges_all(e->m1s.as<int32_t>(), e->nrows, tole, e->rng_all.as<int64_t>(), s));
  e->rng_tol = tole;
  e->rng_valid = true;
  e->key_bits_valid = false;
  return TFP_OK;
}

// The small path's key-presence bitsets, from the cached row ranges (after ensure_ranges).
int delta_bits(tfp_engine* e, hipStream_t s);

int ensure_key_bits(tfp_engine* e, hipStream_t s) {
  if (e->key_bits_valid) return TFP_OK;
  HIPCHK(e, e->key_bits.reserve(sizeof(uint32_t) * (size_t)kKeyRange * key_bits_words(e->ncols)));
  // the boxes' rows in all: a row is in the boxes of the keys within tol of its m1
  const double tl = e->rng_tol;
  const int64_t per_row = std::isfinite(tl) && tl >= 0 && tl < kKeyRange ? 2 * (int64_t)ceil(tl) + 2 : kKeyRange;
  HIPCHK(e, launch_key_bits(e->rng_all.as<int64_t>(), e->cols.as<int32_t>(), e->ncols, e->nrows * std::min<int64_t>(per_row, kKeyRange),
                            e->kb_win, e->kb_direct, e->key_bits.as<uint32_t>(), s));
  int rc = delta_bits(e, s);  // (the delta's columns, from its staged rows)
  if (rc) return rc;
  e->key_bits_valid = true;
  e->key_bits_cols = e->ncols;
  return TFP_OK;
}

// ---- index delta ---------------------------------------------------------------------------

// The delta's key bits at the bitsets' tolerance (rng_tol), into columns that hold no bit.
int delta_bits(tfp_engine* e, hipStream_t s) {
  if (e->delta_clip.empty()) return TFP_OK;
  if (!e->kbox_valid || memcmp(&e->kbox_tol, &e->rng_tol, sizeof e->rng_tol) != 0) {
    HIPCHK(e, e->kbox.reserve(sizeof(int64_t) * 2 * kKeyRange));
    HIPCHK(e, launch_key_boxes(e->rng_tol, e->kbox.as<int64_t>(), s));
    e->kbox_tol = e->rng_tol;
    e->kbox_valid = true;
  }
  const int32_t kspan = (int32_t)ceil(e->rng_tol) + 1;  // (delta_tol_ok: tol <= 8)
  HIPCHK(e, launch_delta_bits(e->d_delta.as<DeltaClip>(), (int32_t)e->delta_clip.size(), e->st_m1.as<int32_t>(),
                              e->kbox.as<int64_t>(), kspan, key_bits_words(e->ncols), e->key_bits.as<uint32_t>(), s));
  return TFP_OK;
}

// Tolerances the delta's bits are set for: finite, 0 <= tol <= 8 (a row is in at most 2 ceil(tol) + 3
// keys' boxes); other searches merge the delta first.
bool delta_tol_ok(double tol) { return std::isfinite(tol) && tol >= 0.0 && tol <= 8.0; }

bool delta_eligible(const tfp_engine* e) {
  if (!e->use_delta || !e->built || e->force_full || e->force_merge || e->removed_built || e->n_staged >= INT32_MAX ||
      (int64_t)e->col_clip.size() < e->delta_min_cols)
    return false;
  int64_t n = 0, rows = 0;
  for (size_t i = e->built_clips; i < e->clips.size(); i++)
    if (e->clips[i].alive) {
      n++;
      rows += e->clips[i].nrows;
    }
  return n <= tfp_engine::kDeltaMaxClips && rows <= tfp_engine::kDeltaMaxRows;
}

// An update that only adds (or removes clips added since the last build): the new clips become the
// delta, in uuid order after the main columns; the tie keys are re-derived (global uuid ranks, or
// the override's keys), and the key bits get the delta's columns. The main index, its row ranges
// and its columns' bits stay as they are: the cost is the new clips' rows, not a pass over the DB.
int delta_update(tfp_engine* e) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  hipStream_t s = e->stream;
  auto by_uuid = [&](int32_t a, int32_t b) { return e->clips[a].uuid < e->clips[b].uuid; };
  std::vector<int32_t> add;
  int64_t rows = 0;
  for (int32_t i = (int32_t)e->built_clips; i < (int32_t)e->clips.size(); i++)
    if (e->clips[i].alive) {
      add.push_back(i);
      rows += e->clips[i].nrows;
    }
  std::sort(add.begin(), add.end(), by_uuid);
  const int32_t Cm = (int32_t)e->col_clip.size(), D = (int32_t)add.size();
  std::vector<int32_t> at(std::max(D, 1));
  for (int32_t j = 0; j < D; j++)
    at[j] = (int32_t)(std::lower_bound(e->col_clip.begin(), e->col_clip.end(), add[j], by_uuid) - e->col_clip.begin());
  const int32_t col0 = D ? (Cm + 1023) / 1024 * 1024 : Cm;
  const int32_t ncols = D ? col0 + tfp_engine::kDeltaMaxClips : Cm;
  // tie keys (and the key -> column maps with an override)
  const bool ovr = !e->tiebreak_override.empty();
  const void* tk_before = e->tiekey.p;
  HIPCHK(e, e->tiekey.reserve_grow(sizeof(int32_t) * std::max(ncols, 1)));
  std::unordered_map<int32_t, int32_t> key_col_delta;
  std::vector<int32_t> tk;  // host staging of the keys uploaded (kept until the sync below)
  if (ovr) {
    auto key_of_clip = [&](int32_t clip, int32_t* k) -> int {
      if ((size_t)clip >= e->tiebreak_override.size())
        return fail(e, TFP_E_ARG, "clip %s was added after tfp_index_set_tiebreak: set the tie-break keys again",
                    e->clips[clip].uuid.c_str());
      *k = e->tiebreak_override[clip];
      return TFP_OK;
    };
    // the main columns' keys: only when the override changed for them (or their device copy was
    // lost to a larger buffer); otherwise the delta's clips alone (O(new clips), round 6)
    const bool main_up = e->ovr_main_stale || e->tiekey.p != tk_before;
    e->n_delta_main_keys += main_up;
    if (e->ovr_main_stale) {
      std::unordered_map<int32_t, int32_t> key_col;
      key_col.reserve(Cm);
      for (int32_t c = 0; c < Cm; c++) {
        int32_t k;
        if (int rc = key_of_clip(e->col_clip[c], &k)) return rc;
        if (!key_col.emplace(k, c).second) return fail(e, TFP_E_ARG, "tie-break key %d given to two live clips", k);
      }
      e->key_col = std::move(key_col);
    }
    tk.assign(main_up ? std::max(ncols, 1) : std::max(D, 1), 0);
    key_col_delta.reserve(D);
    for (int32_t j = 0; j < D; j++) {
      int32_t k;
      if (int rc = key_of_clip(add[j], &k)) return rc;
      if (e->key_col.count(k) || !key_col_delta.emplace(k, col0 + j).second)
        return fail(e, TFP_E_ARG, "tie-break key %d given to two live clips", k);
      tk[main_up ? col0 + j : j] = k;
    }
    if (main_up) {
      for (int32_t c = 0; c < Cm; c++) tk[c] = e->tiebreak_override[e->col_clip[c]];
      HIPCHK(e, hipMemcpyAsync(e->tiekey.p, tk.data(), sizeof(int32_t) * ncols, hipMemcpyHostToDevice, s));
    } else if (D) {
      HIPCHK(e, hipMemcpyAsync(e->tiekey.as<int32_t>() + col0, tk.data(), sizeof(int32_t) * D, hipMemcpyHostToDevice, s));
    }
    e->ovr_main_stale = false;
    e->tiekey_ident = -1;
  } else {
    HIPCHK(e, e->d_delta_at.reserve(sizeof(int32_t) * std::max(D, 1)));
    if (D) HIPCHK(e, hipMemcpyAsync(e->d_delta_at.p, at.data(), sizeof(int32_t) * D, hipMemcpyHostToDevice, s));
    HIPCHK(e, launch_delta_tiekey(e->d_delta_at.as<int32_t>(), D, Cm, col0, ncols, e->tiekey.as<int32_t>(), s));
    e->tiekey_ident = D ? -1 : Cm;
  }
  // the delta's clips for the bits kernel
  std::vector<DeltaClip> dc(std::max(D, 1));
  for (int32_t j = 0; j < D; j++) {
    const Clip& c = e->clips[add[j]];
    dc[j] = DeltaClip{c.off, (int32_t)c.nrows, col0 + j};
  }
  HIPCHK(e, e->d_delta.reserve(sizeof(DeltaClip) * std::max(D, 1)));
  if (D) HIPCHK(e, hipMemcpyAsync(e->d_delta.p, dc.data(), sizeof(DeltaClip) * D, hipMemcpyHostToDevice, s));
  e->delta_clip = std::move(add);
  e->delta_at.assign(at.begin(), at.begin() + D);
  e->delta_col0 = col0;
  e->delta_rows = rows;
  e->ncols = ncols;
  e->key_col_delta = std::move(key_col_delta);
  e->key_identity = !ovr;
  // key bits: the first delta after a build widens the rows (the delta's columns start at a
  // multiple of 1024): the main columns' words move to the wider rows in one 2-D device copy
  // (~13 MB at 100k clips) instead of a rebuild from the index rows (46 ms at 100k clips)
  if (e->key_bits_valid && D > 0 && e->key_bits_cols != ncols && e->key_bits_cols <= col0) {
    const int32_t Wo = key_bits_words(e->key_bits_cols), Wn = key_bits_words(ncols);
    if (Wn > Wo) {
      const size_t nb = sizeof(uint32_t) * (size_t)kKeyRange * Wn;
      HIPCHK(e, e->key_bits_b.reserve(nb));
      HIPCHK(e, hipMemsetAsync(e->key_bits_b.p, 0, nb, s));
      HIPCHK(e, hipMemcpy2DAsync(e->key_bits_b.p, sizeof(uint32_t) * Wn, e->key_bits.p, sizeof(uint32_t) * Wo,
                                 sizeof(uint32_t) * Wo, kKeyRange, hipMemcpyDeviceToDevice, s));
      std::swap(e->key_bits.p, e->key_bits_b.p);
      std::swap(e->key_bits.bytes, e->key_bits_b.bytes);
    }
    e->key_bits_cols = ncols;
  }
  // the delta columns cleared and set again when the layout stands, else rebuilt later
  if (e->key_bits_valid && e->key_bits_cols == ncols && D > 0) {
    const int32_t W = key_bits_words(ncols);
    HIPCHK(e, hipMemset2DAsync(e->key_bits.as<uint32_t>() + col0 / 32, sizeof(uint32_t) * W, 0,
                               sizeof(uint32_t) * (tfp_engine::kDeltaMaxClips / 32), kKeyRange, s));
    int rc = delta_bits(e, s);
    if (rc) return rc;
  } else {
    e->key_bits_valid = false;
  }
  HIPCHK(e, hipStreamSynchronize(s));  // (dc and at are released on return)
  e->dirty = false;
  e->index_version++;  // (other tolerances' cached ranges and bitsets are for the previous index)
  e->n_delta_updates++;
  if (e->dbg_index)
    fprintf(stderr, "[tfp] index delta: %d clips (%lld rows) beside %d main columns; %.3f ms\n", D, (long long)rows, Cm,
            std::chrono::duration<double, std::milli>(clk::now() - t0).count());
  return TFP_OK;
}

// The delta merged into the main index now (coefs = 2, a fallback to the row scan, a tolerance the
// delta's bits do not cover).
int consolidate(tfp_engine* e) {
  if (e->delta_clip.empty() && !e->dirty) return TFP_OK;
  e->force_merge = true;
  e->dirty = true;
  const int rc = rebuild(e);
  e->force_merge = false;
  return rc;
}

// The clip order of the current index (tfp_kernels.hpp), built when first needed: the index rows'
// keys (nearest-integer key, column, m2) radix-sorted once; merge_index carries it afterwards.
int ensure_order(tfp_engine* e, hipStream_t s) {
  if (e->o_valid) return TFP_OK;
  const int64_t R = e->nrows;
  if (R >= INT32_MAX) return fail(e, TFP_E_CAPACITY, "clip order: %lld rows", (long long)R);
  const size_t n = (size_t)std::max<int64_t>(R, 1);
  HIPCHK(e, e->o_key.reserve_grow(sizeof(unsigned long long) * n));
  HIPCHK(e, e->o_m1.reserve_grow(sizeof(int32_t) * n));
  HIPCHK(e, e->o_key_b.reserve_grow(sizeof(unsigned long long) * n));
  HIPCHK(e, e->o_m1_b.reserve_grow(sizeof(int32_t) * n));
  HIPCHK(e, launch_order_fill(e->m1s.as<int32_t>(), e->m2s.as<int32_t>(), e->cols.as<int32_t>(), R,
                              e->o_key_b.as<unsigned long long>(), e->o_m1_b.as<int32_t>(), s));
  HIPCHK(e, order_sort(e->o_key_b.as<unsigned long long>(), e->o_key.as<unsigned long long>(), e->o_m1_b.as<int32_t>(),
                       e->o_m1.as<int32_t>(), R, &e->o_sort_tmp, s));
  e->o_rows = R;
  e->o_valid = true;
  e->n_order_builds++;
  return TFP_OK;
}

// The keys' "%f" boxes at tolerance tole (launch_key_boxes), for the caches built from a clip order.
int ensure_kbox(tfp_engine* e, double tole, hipStream_t s) {
  if (e->kbox_valid && memcmp(&e->kbox_tol, &tole, sizeof tole) == 0) return TFP_OK;
  HIPCHK(e, e->kbox.reserve(sizeof(int64_t) * 2 * kKeyRange));
  HIPCHK(e, launch_key_boxes(tole, e->kbox.as<int64_t>(), s));
  e->kbox_tol = tole;
  e->kbox_valid = true;
  return TFP_OK;
}

// The general path's clip-set cache at tolerance tole (after ensure_ranges at tole): the active one,
// or one of kCellSlots others (least recently used out), per index version. Built from the clip
// order for tolerances up to kOrderMaxTol (no sort), else from the boxes' rows.
int ensure_cells(tfp_engine* e, double tole, hipStream_t s) {
  if (e->cell_fresh && e->cell_version == e->main_version && memcmp(&e->cell_tol, &tole, sizeof tole) == 0) return TFP_OK;
  CellSlot* hit = nullptr;
  CellSlot* victim = &e->cell_lru[0];
  for (CellSlot& t : e->cell_lru) {
    if (t.version != e->main_version) t.has = false;
    if (t.has && memcmp(&t.tol, &tole, sizeof tole) == 0) hit = &t;
    if (t.has != victim->has ? !t.has : t.used < victim->used) victim = &t;
  }
  const bool active = e->cell_fresh && e->cell_version == e->main_version;
  CellSlot* into = hit ? hit : victim;
  // the active cache (when current) goes into the slot the wanted one comes from (or the victim's,
  // whose buffers the build below then reuses)
  e->cells.swap(into->c);
  std::swap(e->cell_tol, into->tol);
  into->has = active;
  into->version = e->main_version;
  into->used = ++e->tol_clock;
  if (hit) {
    e->cell_tol = tole;
    e->cell_fresh = true;
    e->cell_version = e->main_version;
    e->n_cell_hits++;
    return TFP_OK;
  }
  e->n_cell_builds++;
  // The cache is optional: if building it fails (an allocation or a library call), the batch takes
  // the row scan, which needs none of it (tfp_scan.hip).
  hipError_t st = hipSuccess;
  if (tole >= 0.0 && tole <= kOrderMaxTol && e->nrows > 0 && e->nrows < INT32_MAX) {
    int rc = ensure_order(e, s);
    if (rc) return rc;
    if ((rc = ensure_kbox(e, tole, s))) return rc;
    st = e->cells.build_from_order(e->o_key.as<unsigned long long>(), e->o_m1.as<int32_t>(), e->o_rows, e->kbox.as<int64_t>(),
                                   (int32_t)e->col_clip.size(), tole, s);
    if (st == hipSuccess && e->cells.valid) e->n_cell_from_order++;
  } else {
    std::vector<int64_t> rng(2 * kKeyRange), off(kKeyRange + 1, 0);
    HIPCHK(e, hipMemcpyAsync(rng.data(), e->rng_all.p, sizeof(int64_t) * rng.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(e, hipStreamSynchronize(s));
    for (int k = 0; k < kKeyRange; k++) off[k + 1] = off[k] + std::max<int64_t>(0, rng[2 * k + 1] - rng[2 * k]);
    st = e->cells.build(e->rng_all.as<int64_t>(), off.data(), e->m2s.as<int32_t>(), e->cols.as<int32_t>(),
                        (int32_t)e->col_clip.size(), e->nrows, tole, s);
  }
  if (st != hipSuccess) {
    (void)hipGetLastError();
    if (e->dbg_vote) fprintf(stderr, "[tfp] clip-set cache not built (%s): row scan\n", hipGetErrorString(st));
    e->cells.invalidate();
    HIPCHK(e, hipStreamSynchronize(s));
  }
  e->cell_tol = tole;
  e->cell_fresh = true;
  e->cell_version = e->main_version;
  return TFP_OK;
}

// The index delta's clip-set cache at tolerance tole (<= kOrderMaxTol): the delta's staged rows in
// clip order (sorted once per delta version, for any tolerance), then the main cache's filter.
// Valid (or known empty: no delta row in a box) at the current index version.
int ensure_delta_cells(tfp_engine* e, double tole, hipStream_t s) {
  if (e->dcell_fresh && e->dcell_version == e->index_version && memcmp(&e->dcell_tol, &tole, sizeof tole) == 0) return TFP_OK;
  e->dcell_fresh = false;
  e->dcells.invalidate();
  const int32_t D = (int32_t)e->delta_clip.size();
  const int64_t n = e->delta_rows;
  if (D > 0 && n > 0) {
    if (e->dl_version != e->index_version) {
      HIPCHK(e, e->dl_key.reserve_grow(sizeof(unsigned long long) * n));
      HIPCHK(e, e->dl_m1.reserve_grow(sizeof(int32_t) * n));
      HIPCHK(e, e->dl_key_b.reserve_grow(sizeof(unsigned long long) * n));
      HIPCHK(e, e->dl_m1_b.reserve_grow(sizeof(int32_t) * n));
      HIPCHK(e, launch_delta_order_fill(e->d_delta.as<DeltaClip>(), D, e->st_m1.as<int32_t>(), e->st_m2.as<int32_t>(),
                                        e->dl_key_b.as<unsigned long long>(), e->dl_m1_b.as<int32_t>(), s));
      HIPCHK(e, order_sort(e->dl_key_b.as<unsigned long long>(), e->dl_key.as<unsigned long long>(), e->dl_m1_b.as<int32_t>(),
                           e->dl_m1.as<int32_t>(), n, &e->dl_sort_tmp, s));
      e->dl_version = e->index_version;
    }
    int rc = ensure_kbox(e, tole, s);
    if (rc) return rc;
    HIPCHK(e, e->dcells.build_from_order(e->dl_key.as<unsigned long long>(), e->dl_m1.as<int32_t>(), n, e->kbox.as<int64_t>(),
                                         D, tole, s));
    e->n_delta_cell_builds++;
  }
  e->dcell_tol = tole;
  e->dcell_version = e->index_version;
  e->dcell_fresh = true;
  return TFP_OK;
}

// Can the sweep serve a search at tolerance tole with the index delta beside the main index?
bool delta_wide_ok(const tfp_engine* e, double tole) {
  return e->delta_wide && tole >= 0.0 && tole <= kOrderMaxTol && tole >= e->wide_min_tol;
}

// ---- search core: frames' q values already on device (e->q, 2 doubles per frame) -----------

int search_core(tfp_engine* e, const int64_t* h_qoff, int32_t nq, const double* d_q, const tfp_search_params* P,
                std::vector<unsigned long long>& keys, unsigned long long* d_keys_out, hipStream_t s) {
  int rc = rebuild(e);  // synchronous on e->stream
  if (rc) return rc;
  keys.assign(nq, 0ull);
  const int64_t nf = h_qoff[nq] - h_qoff[0];
  SearchConsts sc;
  memset(&sc, 0, sizeof sc);
  sc.coefs = P->coefs;
  sc.tole = P->tolerance < 0 ? TFP_DEFAULT_TOLERANCE : P->tolerance;  // fp_handler.c:252-256
  sc.has_low = P->freq_ignore_low > 0;
  sc.has_high = P->freq_ignore_high > 0;
  if (sc.has_low) sc.thr_low = 10 * log10((double)P->freq_ignore_low);
  if (sc.has_high) sc.thr_high = 10 * log10((double)P->freq_ignore_high);
  // the index delta serves the coefs = 1 vote paths at the tolerances its bits cover, and the sweep
  // (its own clip-set cache beside the main one) at tolerances up to kOrderMaxTol; any other search
  // reads the sorted rows, so the delta is merged into them first
  if (!e->delta_clip.empty() && ((sc.coefs == 1 && !delta_tol_ok(sc.tole)) || (sc.coefs != 1 && !delta_wide_ok(e, sc.tole))) &&
      (rc = consolidate(e)))
    return rc;
  const bool has_delta = !e->delta_clip.empty();
  const int64_t R_all = e->nrows + e->delta_rows;  // rows that may match (main index + delta)

  std::vector<int64_t> qo(h_qoff, h_qoff + nq + 1);
  for (auto& v : qo) v -= h_qoff[0];
  if (!d_keys_out && sc.coefs == 1 && nq >= 1 && nq <= kSmallQ && e->ncols > 0 && R_all > 0) {
    // small batch (batch-1 latency): one vote launch over the cached key bitsets, results into
    // host-mapped memory
    bool fits = true;
    for (int32_t i = 0; i < nq; i++) fits &= qo[i + 1] - qo[i] <= 2048;  // counts bounded like the fp16 path
    if (fits) {
      SmallQueries sq;
      memset(&sq, 0, sizeof sq);
      sq.nq = nq;
      for (int32_t i = 0; i <= nq; i++) sq.qoff[i] = qo[i];
      const int32_t C = e->ncols;
      HIPCHK(e, e->small_res.reserve(small_result_bytes(C), hipHostMallocMapped | hipHostMallocCoherent));
      if (e->small_res.p != e->small_res_host) {
        HIPCHK(e, hipHostGetDevicePointer(reinterpret_cast<void**>(&e->small_res_dev), e->small_res.p, 0));
        e->small_res_host = e->small_res.p;
      }
      if ((rc = ensure_ranges(e, sc.tole, s)) || (rc = ensure_key_bits(e, s))) return rc;
      HIPCHK(e, launch_search_small(d_q, sq, sc, e->key_bits.as<uint32_t>(), C, e->tiekey.as<int32_t>(), e->small_res_dev,
                                    s));
      HIPCHK(e, hipStreamSynchronize(s));
      // the vote ran after the fingerprint kernel, which read the staged upload: it is free again
      e->stage_pending = false;
      // the vote's blocks wrote their per-query maxima into host memory: the max over the blocks
      SmallResult* h = e->small_res.as<SmallResult>();
      if (!h->bad) {
        if (h->ku > 0) {
          const unsigned long long* part = small_result_parts(h);
          const int32_t nb = small_vote_blocks(C);
          for (int32_t i = 0; i < nq; i++) {
            unsigned long long k = 0ull;
            for (int32_t b = 0; b < nb; b++) k = std::max(k, part[(size_t)b * kSmallQ + i]);
            keys[i] = k;
          }
        }
        return TFP_OK;
      }
      // a key outside the vote range: redo the batch on the general path below (the index's rows:
      // the delta merged first)
      if (has_delta) {
        if ((rc = consolidate(e))) return rc;
        return search_core(e, h_qoff, nq, d_q, P, keys, d_keys_out, s);
      }
    }
  }
  // Query offsets are the same on every call of one plan or stream: copy them only when they
  // change, from pinned memory so the copy is asynchronous (a pageable copy would make the host
  // wait for the queries' fingerprint kernels before it could launch the search).
  if (qo != e->qoff_host || s != e->qoff_stream) {
    const size_t bytes = sizeof(int64_t) * qo.size();
    if (e->qoff_pending) HIPCHK(e, hipEventSynchronize(e->qoff_ev));  // previous copy done reading
    HIPCHK(e, e->qoff.reserve(bytes));
    HIPCHK(e, e->qoff_pin.reserve(bytes));
    memcpy(e->qoff_pin.p, qo.data(), bytes);
    HIPCHK(e, hipMemcpyAsync(e->qoff.p, e->qoff_pin.p, bytes, hipMemcpyHostToDevice, s));
    if (!e->qoff_ev) HIPCHK(e, hipEventCreateWithFlags(&e->qoff_ev, hipEventDisableTiming));
    HIPCHK(e, hipEventRecord(e->qoff_ev, s));
    e->qoff_pending = true;
    e->qoff_host = qo;
    e->qoff_stream = s;
  }
  HIPCHK(e, e->boxes.reserve(sizeof(FrameBox) * (nf + 1)));
  const int32_t Qp = ((nq + 127) / 128) * 128;
  // one buffer: the vote path's key mask (32 words), max count (1), pad (1), VoteMeta (4), then
  // best[Qp] (u64); zeroed by prep_boxes. VoteMeta directly before best[]: one copy brings both back.
  constexpr int kMaskWords = kKeyRange / 32, kMetaWord = kMaskWords + 2, kMiscWords = kMetaWord + 4;
  static_assert(sizeof(VoteMeta) == 16 && kMiscWords % 2 == 0, "meta + 8-byte aligned best[]");
  const int32_t nzero = kMiscWords + 2 * Qp;
  HIPCHK(e, e->best.reserve(sizeof(uint32_t) * nzero));
  uint32_t* d_mask = e->best.as<uint32_t>();
  int32_t* d_max = reinterpret_cast<int32_t*>(d_mask + kMaskWords);
  unsigned long long* d_best = reinterpret_cast<unsigned long long*>(d_mask + kMiscWords);
  const int32_t C = e->ncols;
  const int64_t R = e->nrows;
  int64_t max_frames = 0;
  for (int32_t i = 0; i < nq; i++) max_frames = std::max<int64_t>(max_frames, qo[i + 1] - qo[i]);
  const bool vote = sc.coefs == 1 && C > 0 && R_all > 0 && max_frames < 16384;  // packed scores exact below 16384 frames
  if (!vote && has_delta && !delta_wide_ok(e, sc.tole)) {  // (the cells form and the row scan read the sorted rows)
    if ((rc = consolidate(e))) return rc;
    return search_core(e, h_qoff, nq, d_q, P, keys, d_keys_out, s);
  }
  // the vote path needs only the zeroing; the scan path the frames' boxes too
  HIPCHK(e, launch_prep_boxes(d_q, vote ? 0 : nf, sc, e->boxes.as<FrameBox>(), d_mask, nzero, s));

  bool done = false;
  if (vote) {
    // vote-matrix path, no host round trip: key mask -> used-key compaction -> A (per-query
    // counts) and Bt -> GEMM
    const int32_t Cp = ((C + 31) / 32) * 32;
    HIPCHK(e, e->A.reserve(sizeof(_Float16) * (size_t)Qp * kVoteKpMax));
    HIPCHK(e, e->Bt.reserve(sizeof(_Float16) * (size_t)Cp * kVoteKpMax));
    VoteMeta* d_meta = reinterpret_cast<VoteMeta*>(d_mask + kMetaWord);
    if ((rc = ensure_ranges(e, sc.tole, s)) || (rc = ensure_key_bits(e, s))) return rc;
    HIPCHK(e, launch_key_mask(d_q, sc, nf, d_mask, d_max, d_meta, s));
    HIPCHK(e, launch_build_A(d_q, sc, e->qoff.as<int64_t>(), nq, Qp, d_mask, d_max, d_meta, e->class_ku_max,
                             e->A.as<_Float16>(), e->Bt.as<_Float16>(), Cp, s));
    HIPCHK(e, launch_build_B(d_mask, e->key_bits.as<uint32_t>(), C, d_meta, Cp, e->Bt.as<_Float16>(), s));
    HIPCHK(e, e->vote_part.reserve(sizeof(unsigned long long) * (size_t)vote_chunks(Cp) * Qp));
    HIPCHK(e, launch_vote_gemm(e->A.as<_Float16>(), e->Bt.as<_Float16>(), Qp, Cp, d_meta, e->tiekey.as<int32_t>(),
                               e->vote_part.as<unsigned long long>(), d_best, d_mask, e->key_bits.as<uint32_t>(), C, s));
    // the results go out before the ok flag is known (one host wait); a redo overwrites them.
    // Host results: (VoteMeta, best[nq]) in one copy into pinned memory.
    const size_t back = sizeof(VoteMeta) + (d_keys_out ? 0 : sizeof(unsigned long long) * nq);
    HIPCHK(e, e->vres_pin.reserve(back));
    if (d_keys_out)
      HIPCHK(e, hipMemcpyAsync(d_keys_out, d_best, sizeof(unsigned long long) * nq, hipMemcpyDeviceToDevice, s));
    HIPCHK(e, hipMemcpyAsync(e->vres_pin.p, d_meta, back, hipMemcpyDeviceToHost, s));
    HIPCHK(e, hipStreamSynchronize(s));
    VoteMeta hm;
    memcpy(&hm, e->vres_pin.p, sizeof hm);
    if (!d_keys_out && nq)
      memcpy(keys.data(), e->vres_pin.as<char>() + sizeof(VoteMeta), sizeof(unsigned long long) * nq);
    if (e->dbg_vote) fprintf(stderr, "[tfp] vote: nq %d Qp %d C %d ku %d kp %d ok %d\n", nq, Qp, C, hm.ku, hm.kp, hm.ok);
    if (hm.ok) return TFP_OK;
    // a count above fp16's exact range or a key outside the vote range: the scan path below (over
    // the sorted rows: the delta merged into them first)
    if (has_delta) {
      if ((rc = consolidate(e))) return rc;
      return search_core(e, h_qoff, nq, d_q, P, keys, d_keys_out, s);
    }
    HIPCHK(e, launch_prep_boxes(d_q, nf, sc, e->boxes.as<FrameBox>(), d_mask, nzero, s));
  }
  for (int pass = 0;; pass++) {
    bool spec = false;  // the sweep ran without the host reading its sort's counts (checked below)
    bool spec_mapped = false;  // its counts were written to spec_pin by its last kernel
    bool out_written = false;  // the sweep wrote its keys straight into d_keys_out
    bool swept = false;        // the sweep by groups ran (not the cells form / row scan)
    bool bins_used = false;
    if (!done && C > 0 && R > 0 && (sc.coefs == 1 || sc.coefs == 2) && sc.tole >= e->wide_min_tol) {
      // general path: the sweep by groups (tfp_scan.hip), unless a frame needs the row scan
      if ((rc = ensure_ranges(e, sc.tole, s)) || (rc = ensure_cells(e, sc.tole, s))) return rc;
      if (e->dbg_vote && !e->cells.valid) fprintf(stderr, "[tfp] general path: no clip-set cache (row scan)\n");
      // with a delta: its cache too (a failure to build it merges the delta, below)
      bool dsweep = has_delta && e->cells.valid;
      if (dsweep && ensure_delta_cells(e, sc.tole, s) != TFP_OK) {
        (void)hipGetLastError();
        e->err.clear_own();  // (recovered: the merge below serves the batch)
        dsweep = false;
      }
      if (e->cells.valid && (dsweep || !has_delta)) {
        HIPCHK(e, e->wide.reserve(nf, nq, s));
        bool ok = false;
        // (a device caller's output buffer takes the sweep's keys directly: zeroed by the prepare)
        unsigned long long* wbest = d_keys_out ? reinterpret_cast<unsigned long long*>(d_keys_out) : d_best;
        HIPCHK(e, launch_scan_wide_prepare(e->boxes.as<FrameBox>(), e->qoff.as<int64_t>(), nq, nf, max_frames, sc.tole,
                                           &e->wide, &ok, s, pass == 0, d_keys_out ? wbest : nullptr));
        bins_used = e->wide.ukeys_ready;  // (the bin sort ran on this pass)
        if (ok) {
          // a speculative sweep's counts come back through host-mapped memory, written by its last kernel
          int32_t* d_info = nullptr;
          if (e->wide.spec) {
            HIPCHK(e, e->spec_pin.reserve(4 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent));
            if (e->spec_pin.p != e->spec_pin_host) {
              HIPCHK(e, hipHostGetDevicePointer(reinterpret_cast<void**>(&e->spec_pin_dev), e->spec_pin.p, 0));
              e->spec_pin_host = e->spec_pin.p;
            }
            d_info = e->spec_pin_dev;
          }
          HIPCHK(e, launch_scan_wide(nq, nf, &e->cells, e->tiekey.as<int32_t>(), C, &e->wide, wbest, s, d_info, &spec_mapped));
          if (dsweep && e->dcells.valid) {  // the delta's clips into the same maxima
            HIPCHK(e, launch_scan_wide(nq, nf, &e->dcells, e->tiekey.as<int32_t>(), C, &e->wide, wbest, s, d_info, &spec_mapped,
                                       e->delta_col0));
            e->n_delta_sweeps++;
          }
          done = true;
          swept = true;
          out_written = d_keys_out != nullptr;
          spec = e->wide.spec;
        }
        if (e->dbg_vote) fprintf(stderr, "[tfp] general path: nq %d nf %lld C %d tol %g -> %s%s\n", nq, (long long)nf, C,
                                 sc.tole, ok ? "sweep by groups" : "cells / row scan", spec ? " (speculative)" : "");
      }
    }
    if (!done && has_delta) {  // the cells form and the row scan read the sorted rows: the delta merged first
      if ((rc = consolidate(e))) return rc;
      return search_core(e, h_qoff, nq, d_q, P, keys, d_keys_out, s);
    }
    if (!done && C > 0 && R > 0 && (sc.coefs == 1 || sc.coefs == 2)) {
      // general path (tfp_scan.hip): queries in chunks of <= 256 MB of scratch per array
      if ((rc = ensure_ranges(e, sc.tole, s)) || (rc = ensure_cells(e, sc.tole, s))) return rc;
      int64_t chunk = (int64_t)(256ll << 20) / (4ll * C);
      chunk = std::max<int64_t>(1, std::min<int64_t>(chunk, nq));
      const size_t bytes = sizeof(int32_t) * chunk * C;
      if (bytes > e->scan_zeroed || bytes > e->stamp.bytes || bytes > e->score.bytes || bytes > e->touched.bytes ||
          sizeof(int32_t) * chunk > e->tcnt.bytes) {
        HIPCHK(e, e->stamp.reserve(bytes));
        HIPCHK(e, e->score.reserve(bytes));
        HIPCHK(e, e->touched.reserve(bytes));
        HIPCHK(e, e->tcnt.reserve(sizeof(int32_t) * chunk));
        const size_t z = std::min(std::min(e->stamp.bytes, e->score.bytes), e->touched.bytes);
        HIPCHK(e, hipMemsetAsync(e->stamp.p, 0, z, s));
        HIPCHK(e, hipMemsetAsync(e->score.p, 0, z, s));
        HIPCHK(e, hipMemsetAsync(e->tcnt.p, 0, e->tcnt.bytes, s));
        e->scan_zeroed = z;  // (touched is written before it is read)
      }
      if (e->cells.valid && e->cells.ensure_entries(s) != hipSuccess) {  // (the cells form's candidates)
        (void)hipGetLastError();
        e->cells.invalidate();  // every frame takes the row scan
      }
      for (int64_t q0 = 0; q0 < nq; q0 += chunk) {
        const int32_t n = (int32_t)std::min<int64_t>(chunk, nq - q0);
        HIPCHK(e, launch_scan(e->boxes.as<FrameBox>(), e->qoff.as<int64_t>(), qo.data(), (int32_t)q0, n,
                              e->m1s.as<int32_t>(), e->m2s.as<int32_t>(), e->cols.as<int32_t>(), R, &e->cells,
                              e->tiekey.as<int32_t>(), C, e->stamp.as<int32_t>(), e->score.as<int32_t>(),
                              e->touched.as<int32_t>(), e->tcnt.as<int32_t>(), d_best, s));
      }
    }
    // the speculative sweep's counts come back with the results (one host wait per batch)
    if (spec && !spec_mapped) {
      HIPCHK(e, e->spec_pin.reserve(4 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent));
      HIPCHK(e, hipMemcpyAsync(e->spec_pin.p, e->wide.info, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    }
    if (d_keys_out) {
      if (!out_written)
        HIPCHK(e, hipMemcpyAsync(d_keys_out, d_best, sizeof(unsigned long long) * nq, hipMemcpyDeviceToDevice, s));
    } else if (nq) {
      HIPCHK(e, hipMemcpyAsync(keys.data(), d_best, sizeof(unsigned long long) * nq, hipMemcpyDeviceToHost, s));
    }
    // (the scan kernels read and write engine scratch: the next call, on any stream or thread, may
    // reuse it only once they are done)
    HIPCHK(e, hipStreamSynchronize(s));
    if (spec) {
      const int32_t* info = e->spec_pin.as<int32_t>();
      if (info[1] > 0 || info[2] > 0) {  // a frame for the row scan, or a window the one-sort key cannot order
        if (e->dbg_vote) fprintf(stderr, "[tfp] speculative sweep redone (info %d %d %d)\n", info[0], info[1], info[2]);
        e->n_sweep_redo++;
        done = false;
        HIPCHK(e, hipMemsetAsync(d_best, 0, sizeof(unsigned long long) * nq, s));
        continue;
      }
      if (bins_used) e->n_sweep_crowd += info[3];
    }
    if (swept) (bins_used ? e->n_sweep_bins : e->n_sweep_lib)++;
    return TFP_OK;
  }
}

// The index column of a tie-break key (-1: none). Without an override the key is the clip's rank
// among all live uuids: a main column's, or with a delta (ranks at[j] + j, ascending) either a delta
// column's or main column k - #{delta ranks below k}.
int32_t col_of_key(const tfp_engine* e, int32_t k) {
  if (e->key_identity) {
    const int32_t Cm = (int32_t)e->col_clip.size(), D = (int32_t)e->delta_clip.size();
    if (k < 0 || k >= Cm + D) return -1;
    int32_t lo = 0, hi = D;  // first delta j with rank >= k
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      if (e->delta_at[mid] + mid < k) lo = mid + 1; else hi = mid;
    }
    if (lo < D && e->delta_at[lo] + lo == k) return e->delta_col0 + lo;
    return k - lo;
  }
  auto it = e->key_col.find(k);
  if (it != e->key_col.end()) return it->second;
  auto jt = e->key_col_delta.find(k);
  return jt == e->key_col_delta.end() ? -1 : jt->second;
}

// The clip of an index column (-1: none): a main column or a delta column.
int32_t clip_of_col(const tfp_engine* e, int32_t col) {
  if (col >= 0 && (size_t)col < e->col_clip.size()) return e->col_clip[col];
  const int32_t j = col - e->delta_col0;
  return j >= 0 && (size_t)j < e->delta_clip.size() ? e->delta_clip[j] : -1;
}

void fill_results(tfp_engine* e, const std::vector<unsigned long long>& keys, const int64_t* qoff, int32_t nq,
                  tfp_result* out) {
  for (int32_t i = 0; i < nq; i++) {
    tfp_result& r = out[i];
    memset(&r, 0, sizeof r);
    r.frame_count = (int32_t)(qoff[i + 1] - qoff[i]);
    r.clip_id = -1;
    const unsigned long long k = keys[i];
    if (!k) continue;
    const int32_t clip = clip_of_col(e, col_of_key(e, (int32_t)(uint32_t)(k & 0xffffffffu)));
    if (clip < 0) continue;
    r.found = 1;
    r.match_count = (int32_t)(k >> 32);
    r.clip_id = clip;
    snprintf(r.uuid, sizeof r.uuid, "%s", e->clips[clip].uuid.c_str());
  }
}

bool valid_params(const tfp_search_params* P) { return P && P->coefs >= 1 && P->coefs <= 2; }

}  // namespace

// =========================================================================================
extern "C" {

int tfp_abi_version(void) { return TFP_ABI_VERSION; }

int tfp_device_count(int32_t* count) {
  int n = 0;
  if (!count) return TFP_E_ARG;
  *count = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return TFP_E_NODEV;
  *count = n;
  return TFP_OK;
}

int64_t tfp_frame_count(int64_t n) { return n <= 0 ? 0 : (n + TFP_HOP - 1) / TFP_HOP; }

int tfp_engine_create(int32_t device, tfp_engine** out) {
  if (!out) return TFP_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return TFP_E_NODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return TFP_E_NODEV;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return TFP_E_NODEV;  // code objects are gfx950-only
  if (hipSetDevice(device) != hipSuccess) return TFP_E_HIP;
  tfp_engine* e = new tfp_engine();
  e->device = device;
  if (fp_launch_config(device, &e->fpcfg) != hipSuccess) {
    delete e;
    return TFP_E_HIP;
  }
  // test knobs (tfp::knob: only under TFP_TEST_KNOBS)
  if (const char* v = tfp::knob("TFP_VOTE_CLASS_MAX")) e->class_ku_max = (int32_t)atoi(v);
  e->dbg_vote = tfp::knob("TFP_DEBUG_VOTE") != nullptr;
  e->dbg_index = tfp::knob("TFP_DEBUG_INDEX") != nullptr;
  if (const char* v = tfp::knob("TFP_TEST_FAIL_COMPACT")) e->fail_compact = (int32_t)atoi(v);
  if (const char* v = tfp::knob("TFP_TEST_FAIL_QUERY_SAMPLES")) e->fail_query_len = atoll(v);
  if (const char* v = tfp::knob("TFP_KEYBITS_WIN")) e->kb_win = atoi(v);
  if (const char* v = tfp::knob("TFP_KEYBITS_DIRECT")) e->kb_direct = atoll(v);
  e->force_full = tfp::knob("TFP_INDEX_FULL") != nullptr;
  if (const char* v = tfp::knob("TFP_WIDE_MIN_TOL")) e->wide_min_tol = atof(v);
  e->wide.points_only = tfp::knob("TFP_WIDE_POINTS") != nullptr;
  e->wide.ch128 = tfp::knob("TFP_WIDE_CH128") != nullptr;
  e->wide.unpacked = tfp::knob("TFP_WIDE_UNPACKED") != nullptr;
  e->wide.libsort = tfp::knob("TFP_WIDE_LIBSORT") != nullptr;
  e->wide.debug_bins = tfp::knob("TFP_DEBUG_BINS") != nullptr;
  if (const char* v = tfp::knob("TFP_DELTA_WIDE")) e->delta_wide = atoi(v) != 0;
  // operational switches (documented: tiresias_fp.h), read as plain environment variables
  if (const char* v = tfp::op_env("TFP_COALESCE")) e->coalesce = atoi(v) != 0;
  if (const char* v = tfp::op_env("TFP_INDEX_DELTA")) e->use_delta = atoi(v) != 0;
  // test form: the delta even below delta_min_cols main columns (small test DBs)
  if (const char* v = tfp::knob("TFP_INDEX_DELTA"))
    if (atoi(v) != 0) e->delta_min_cols = 0;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    delete e;
    return TFP_E_HIP;
  }
  *out = e;
  return TFP_OK;
}

void tfp_engine_destroy(tfp_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  (void)hipStreamSynchronize(e->stream);
  hipStream_t s = e->stream;
  delete e;
  (void)hipStreamDestroy(s);
}

__attribute__((visibility("hidden"))) const char* tfp_ingest_last_error();  // tfp_wav.cpp: engine-less errors of this thread
const char* tfp_engine_last_error(const tfp_engine* e) {
  return e ? const_cast<tfp_engine*>(e)->err.read(e) : tfp_ingest_last_error();
}

int tfp_host_alloc(size_t bytes, void** out) {
  if (!bytes || !out) return TFP_E_ARG;
  *out = nullptr;
  void* p = nullptr;
  // portable: pinned for every device; each engine maps it on its own device (engine_host_ptr)
  if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess)
    return TFP_E_NOMEM;
  HostAllocs& h = host_allocs();
  std::lock_guard<std::mutex> lk(h.mu);
  h.m[reinterpret_cast<uintptr_t>(p)] = {bytes, h.next_gen++};
  *out = p;
  return TFP_OK;
}

void tfp_host_free(void* p) {
  if (!p) return;
  HostAllocs& h = host_allocs();
  {
    std::lock_guard<std::mutex> lk(h.mu);
    if (!h.m.erase(reinterpret_cast<uintptr_t>(p))) return;  // not ours
  }
  (void)hipHostFree(p);
}

namespace {
int fingerprint_batch_impl(tfp_engine* e, const void* pcm, bool f32, const int64_t* offsets, int32_t nclips,
                           int32_t sr, tfp_frame* out, int64_t cap, int64_t* nframes) {
  if (!e) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (!offsets || nclips < 0 || !nframes || (!pcm && nclips && offsets[nclips] > offsets[0]))
    return fail(e, TFP_E_ARG, "bad arguments");
  for (int32_t c = 0; c < nclips; c++)
    if (offsets[c + 1] < offsets[c]) return fail(e, TFP_E_ARG, "offsets not monotone");
  int64_t need = 0;
  for (int32_t c = 0; c < nclips; c++) need += tfp_frame_count(offsets[c + 1] - offsets[c]);
  *nframes = need;
  if (need > 0 && (!out || cap < need)) return fail(e, TFP_E_CAPACITY, "need %lld frames", (long long)need);
  if (need == 0) return TFP_OK;
  HIPCHK(e, hipSetDevice(e->device));
  int64_t nf;
  std::vector<int64_t> foff;
  std::vector<const void*> ptrs;
  std::vector<int64_t> lens;
  split_offsets(pcm, f32 ? sizeof(float) : sizeof(int16_t), offsets, nclips, &ptrs, &lens);
  int rc = fingerprint_host(e, ptrs.data(), lens.data(), f32, nclips, sr, &nf, &foff);
  if (rc) return rc;
  return copy_frames_out(e, nf, foff, out);
}
}  // namespace

int tfp_fingerprint_batch(tfp_engine* e, const int16_t* pcm, const int64_t* offsets, int32_t nclips, int32_t sr,
                          tfp_frame* out, int64_t cap, int64_t* nframes) {
  return fingerprint_batch_impl(e, pcm, false, offsets, nclips, sr, out, cap, nframes);
}

int tfp_fingerprint_f32_batch(tfp_engine* e, const float* x, const int64_t* offsets, int32_t nclips, int32_t sr,
                              tfp_frame* out, int64_t cap, int64_t* nframes) {
  return fingerprint_batch_impl(e, x, true, offsets, nclips, sr, out, cap, nframes);
}

int tfp_fingerprint_pcm(tfp_engine* e, const int16_t* pcm, int64_t n, int32_t sr, tfp_frame* out, int64_t cap,
                        int64_t* nframes) {
  if (n < 0) return TFP_E_ARG;
  int64_t off[2] = {0, n};
  return tfp_fingerprint_batch(e, pcm, off, 1, sr, out, cap, nframes);
}

int tfp_plan_create(tfp_engine* e, const int64_t* offsets, int32_t nclips, int32_t sr, tfp_plan** out) {
  if (!e || !offsets || nclips < 0 || !out) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  const DspTables* T;
  bool fx = false;
  int rc = ensure_tables(e, sr, &T, &fx);
  if (rc) return rc;
  tfp_plan* p = new tfp_plan();
  p->eng = e;
  p->nclips = nclips;
  p->sample_rate = sr;
  for (int32_t c = 0; c < nclips; c++)
    if (offsets[c + 1] - offsets[c] >= kDirectMaxSamples) p->long_clip = true;
  p->tile_frames = fp_tile_frames(e->fpcfg, fx && !p->long_clip, false, false);
  layout(offsets, nclips, p->soff, p->foff, p->toff, &p->tclip, p->tile_frames);
  p->nsamples = p->soff[nclips];
  p->nframes = p->foff[nclips];
  p->ntiles = p->toff[nclips];
  if ((rc = upload(e, p->d_soff, p->soff.data(), sizeof(int64_t) * p->soff.size())) ||
      (rc = upload(e, p->d_foff, p->foff.data(), sizeof(int64_t) * p->foff.size())) ||
      (rc = upload(e, p->d_toff, p->toff.data(), sizeof(int32_t) * p->toff.size())) ||
      (rc = upload(e, p->d_tclip, p->tclip.data(), sizeof(int32_t) * p->tclip.size())) ||
      (rc = upload(e, p->d_qoff, p->foff.data(), sizeof(int64_t) * p->foff.size()))) {
    delete p;
    return rc;
  }
  if (hipStreamSynchronize(e->stream) != hipSuccess) { delete p; return fail(e, TFP_E_HIP, "sync"); }
  *out = p;
  return TFP_OK;
}

void tfp_plan_destroy(tfp_plan* p) { delete p; }
int64_t tfp_plan_frames(const tfp_plan* p) { return p ? p->nframes : -1; }

int tfp_fingerprint_device(tfp_engine* e, const tfp_plan* p, const int16_t* d_pcm, int32_t* d_micro, double* d_db,
                           void* stream) {
  if (!e || !p || !d_micro || (!d_pcm && p->nsamples)) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  NullStreamOrder order(e, stream);
  if (!order.ok()) return fail(e, TFP_E_HIP, "ordering after the null stream failed");
  const DspTables* T;
  bool fx = false;
  int rc = ensure_tables(e, p->sample_rate, &T, &fx);
  if (rc) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  HIPCHK(e, launch_fingerprint(e->fpcfg, T, fx && !p->long_clip, p->tile_frames, d_pcm, p->d_soff.as<int64_t>(), p->d_soff.as<int64_t>() + 1,
                               p->d_foff.as<int64_t>(), p->d_toff.as<int32_t>(),
                               p->d_tclip.as<int32_t>(), p->ntiles, p->nframes, d_micro, d_db, s, e->logfix));
  return TFP_OK;
}

int tfp_index_add(tfp_engine* e, const char* uuid, const int32_t* m1, const int32_t* m2, int32_t nframes,
                  int32_t* clip_id) {
  if (!e || nframes < 0 || (nframes && (!m1 || !m2))) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  int32_t id;
  if (!uuid || !*uuid || strlen(uuid) >= 64) return fail(e, TFP_E_ARG, "bad uuid");
  if (e->by_uuid.count(uuid)) return fail(e, TFP_E_EXISTS, "uuid %s already indexed", uuid);
  int rc = stage_reserve(e, nframes);
  if (rc) return rc;
  // the rows go in past the staged ones first; the clip is registered only once they are there
  // (a failed copy leaves the index as it was)
  const int64_t o = e->n_staged;
  if (nframes) {
    std::vector<int32_t> cl(nframes, (int32_t)e->clips.size());
    HIPCHK(e, hipMemcpyAsync(e->st_m1.as<int32_t>() + o, m1, sizeof(int32_t) * nframes, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->st_m2.as<int32_t>() + o, m2, sizeof(int32_t) * nframes, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->st_clip.as<int32_t>() + o, cl.data(), sizeof(int32_t) * nframes, hipMemcpyHostToDevice,
                             e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  if ((rc = new_clip(e, uuid, nframes, o, &id))) return rc;
  e->n_staged += nframes;
  if (clip_id) *clip_id = id;
  return TFP_OK;
}

// de-interleave (m1, m2) pairs + clip ids into staging
__global__ void stage_from_micro_kernel(const int32_t* micro, int64_t nf, const int64_t* foff, int32_t nclips,
                                        int32_t clip0, int32_t* m1, int32_t* m2, int32_t* clip) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nf; g += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = nclips;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (foff[mid] <= g) lo = mid; else hi = mid;
    }
    m1[g] = micro[2 * g];
    m2[g] = micro[2 * g + 1];
    clip[g] = clip0 + lo;
  }
}

int tfp_index_add_device(tfp_engine* e, int32_t nclips, const char* const* uuids, const int64_t* frame_offsets,
                         const int32_t* d_micro, void* stream) {
  if (!e || nclips < 0 || !uuids || !frame_offsets || (!d_micro && frame_offsets[nclips] > frame_offsets[0]))
    return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  NullStreamOrder order(e, stream);
  if (!order.ok()) return fail(e, TFP_E_HIP, "ordering after the null stream failed");
  std::unordered_map<std::string, int> seen;
  for (int32_t c = 0; c < nclips; c++) {
    if (!uuids[c] || !*uuids[c] || strlen(uuids[c]) >= 64) return fail(e, TFP_E_ARG, "bad uuid %d", c);
    if (frame_offsets[c + 1] < frame_offsets[c]) return fail(e, TFP_E_ARG, "frame_offsets not monotone at %d", c);
    if (e->by_uuid.count(uuids[c]) || !seen.emplace(uuids[c], c).second)
      return fail(e, TFP_E_EXISTS, "uuid %s already indexed", uuids[c]);
  }
  const int64_t nf = frame_offsets[nclips] - frame_offsets[0];
  int rc = stage_reserve(e, nf);
  if (rc) return rc;
  const int32_t clip0 = (int32_t)e->clips.size();
  // rows first, clips registered once they are staged (a failure leaves the index as it was)
  if (nf) {
    std::vector<int64_t> fo(frame_offsets, frame_offsets + nclips + 1);
    for (auto& v : fo) v -= frame_offsets[0];
    if ((rc = upload(e, e->foff, fo.data(), sizeof(int64_t) * fo.size()))) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    if (s != e->stream) HIPCHK(e, hipStreamSynchronize(e->stream));
    const int64_t o = e->n_staged;
    hipLaunchKernelGGL(stage_from_micro_kernel, dim3(2048), dim3(256), 0, s, d_micro + 2 * frame_offsets[0], nf,
                       e->foff.as<int64_t>(), nclips, clip0, e->st_m1.as<int32_t>() + o, e->st_m2.as<int32_t>() + o,
                       e->st_clip.as<int32_t>() + o);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipStreamSynchronize(s));
  }
  for (int32_t c = 0; c < nclips; c++) {
    int32_t id;
    if ((rc = new_clip(e, uuids[c], frame_offsets[c + 1] - frame_offsets[c],
                       e->n_staged + frame_offsets[c] - frame_offsets[0], &id)))
      return rc;  // (cannot fail: checked above)
  }
  e->n_staged += nf;
  return TFP_OK;
}

// TFP_TEST_FAIL_ADD_BATCH=n (tests): the n-th tfp_index_add_batch call of the process since the
// variable took its value fails as a device error would, before it changes anything.
static bool injected_add_batch_failure() {
  static std::mutex mu;
  static std::string val;
  static int64_t calls = 0;
  const char* v = tfp::knob("TFP_TEST_FAIL_ADD_BATCH");
  std::lock_guard<std::mutex> lk(mu);
  if (!v) return false;
  if (val != v) {
    val = v;
    calls = 0;
  }
  return ++calls == atoll(v);
}

int tfp_index_add_batch(tfp_engine* e, int32_t nclips, const char* const* uuids, const int64_t* frame_offsets,
                        const int32_t* m1, const int32_t* m2) {
  if (!e || nclips < 0 || !uuids || !frame_offsets) return TFP_E_ARG;
  const int64_t nf = frame_offsets[nclips] - frame_offsets[0];
  if (nf < 0 || (nf && (!m1 || !m2))) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  std::unordered_map<std::string, int> seen;
  for (int32_t c = 0; c < nclips; c++) {
    if (!uuids[c] || !*uuids[c] || strlen(uuids[c]) >= 64) return fail(e, TFP_E_ARG, "bad uuid %d", c);
    if (frame_offsets[c + 1] < frame_offsets[c]) return fail(e, TFP_E_ARG, "frame_offsets not monotone at %d", c);
    if (e->by_uuid.count(uuids[c]) || !seen.emplace(uuids[c], c).second)
      return fail(e, TFP_E_EXISTS, "uuid %s already indexed", uuids[c]);
  }
  if (injected_add_batch_failure()) return fail(e, TFP_E_HIP, "tfp_index_add_batch: injected device failure");
  int rc = stage_reserve(e, nf);
  if (rc) return rc;
  // All-or-nothing: the rows go in past the staged ones, and the clips are registered only once
  // every copy has succeeded.
  const int32_t clip0 = (int32_t)e->clips.size();
  if (nf) {
    std::vector<int32_t> cl(nf);
    for (int32_t c = 0; c < nclips; c++)
      std::fill(cl.begin() + (frame_offsets[c] - frame_offsets[0]), cl.begin() + (frame_offsets[c + 1] - frame_offsets[0]),
                clip0 + c);
    const int64_t o = e->n_staged;
    const int32_t* s1 = m1 + frame_offsets[0];
    const int32_t* s2 = m2 + frame_offsets[0];
    HIPCHK(e, hipMemcpyAsync(e->st_m1.as<int32_t>() + o, s1, sizeof(int32_t) * nf, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->st_m2.as<int32_t>() + o, s2, sizeof(int32_t) * nf, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->st_clip.as<int32_t>() + o, cl.data(), sizeof(int32_t) * nf, hipMemcpyHostToDevice,
                             e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  for (int32_t c = 0; c < nclips; c++) {
    int32_t id;
    const int64_t b = frame_offsets[c] - frame_offsets[0], n = frame_offsets[c + 1] - frame_offsets[c];
    if ((rc = new_clip(e, uuids[c], n, e->n_staged + b, &id))) return rc;  // (cannot fail: checked above)
  }
  e->n_staged += nf;
  return TFP_OK;
}

int tfp_index_rows(tfp_engine* e, const char* uuid, int32_t* m1, int32_t* m2, int64_t cap, int64_t* nframes) {
  if (!e || !uuid || cap < 0 || (cap && (!m1 || !m2))) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  auto it = e->by_uuid.find(uuid);
  if (it == e->by_uuid.end()) return fail(e, TFP_E_NOENT, "uuid %s not indexed", uuid);
  const Clip& c = e->clips[it->second];
  if (nframes) *nframes = c.nrows;
  if (cap < c.nrows) return fail(e, TFP_E_CAPACITY, "need %lld rows", (long long)c.nrows);
  if (c.nrows) {
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipMemcpyAsync(m1, e->st_m1.as<int32_t>() + c.off, sizeof(int32_t) * c.nrows, hipMemcpyDeviceToHost,
                             e->stream));
    HIPCHK(e, hipMemcpyAsync(m2, e->st_m2.as<int32_t>() + c.off, sizeof(int32_t) * c.nrows, hipMemcpyDeviceToHost,
                             e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  return TFP_OK;
}

int tfp_index_remove(tfp_engine* e, const char* uuid) {
  if (!e || !uuid) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  auto it = e->by_uuid.find(uuid);
  if (it == e->by_uuid.end()) return fail(e, TFP_E_NOENT, "uuid %s not indexed", uuid);
  Clip& c = e->clips[it->second];
  c.alive = false;
  e->live_rows -= c.nrows;
  e->removed_built |= (size_t)it->second < e->built_clips;
  e->by_uuid.erase(it);
  e->dirty = true;
  return TFP_OK;
}

int tfp_index_clear(tfp_engine* e) {
  if (!e) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  e->clips.clear();
  e->by_uuid.clear();
  e->tiebreak_override.clear();
  e->n_staged = 0;
  e->built = false;
  e->built_clips = 0;
  e->built_staged = 0;
  e->removed_built = false;
  e->live_rows = 0;
  e->col_clip.clear();
  e->delta_clip.clear();
  e->delta_at.clear();
  e->delta_col0 = 0;
  e->delta_rows = 0;
  e->dirty = true;
  return TFP_OK;
}

int tfp_index_stats(tfp_engine* e, int64_t* nrows, int32_t* nclips) {
  if (!e) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  int64_t r = 0;
  int32_t c = 0;
  for (const auto& cl : e->clips)
    if (cl.alive) { r += cl.nrows; c++; }
  if (nrows) *nrows = r;
  if (nclips) *nclips = c;
  return TFP_OK;
}

int tfp_index_commit(tfp_engine* e) {
  if (!e) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  return rebuild(e);
}

int tfp_index_build_stats(tfp_engine* e, int64_t* full_builds, int64_t* merges) {
  if (!e) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (full_builds) *full_builds = e->n_full_builds;
  if (merges) *merges = e->n_merges;
  return TFP_OK;
}

int tfp_index_delta_stats(tfp_engine* e, int64_t* delta_updates, int32_t* delta_clips) {
  if (!e) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (delta_updates) *delta_updates = e->n_delta_updates;
  if (delta_clips) *delta_clips = (int32_t)e->delta_clip.size();
  return TFP_OK;
}

int tfp_index_set_tiebreak(tfp_engine* e, const int32_t* keys, int32_t n) {
  if (!e || n < 0 || (n && !keys)) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  e->tiebreak_override.assign(keys, keys + n);
  e->ovr_main_stale = true;
  e->dirty = true;
  return TFP_OK;
}

int tfp_index_update_tiebreak(tfp_engine* e, int32_t first_clip_id, const int32_t* keys, int32_t n) {
  if (!e || first_clip_id < 0 || n < 0 || (n && !keys)) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if ((size_t)first_clip_id > e->tiebreak_override.size() || (e->tiebreak_override.empty() && first_clip_id > 0))
    return fail(e, TFP_E_ARG, "tie-break keys from clip id %d: the keys before it were never set", first_clip_id);
  if ((size_t)first_clip_id + (size_t)n > e->tiebreak_override.size()) e->tiebreak_override.resize((size_t)first_clip_id + n);
  std::copy(keys, keys + n, e->tiebreak_override.begin() + first_clip_id);
  // new keys for clips of the last build change the main columns' keys (a full refresh at the next
  // update); keys of clips added since concern the delta or the next merge only
  if ((size_t)first_clip_id < e->built_clips && n > 0) e->ovr_main_stale = true;
  e->dirty = true;
  return TFP_OK;
}

int tfp_index_uuid_of_key(tfp_engine* e, int32_t key, char* uuid, int32_t len) {
  if (!e || !uuid || len <= 0) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  const int32_t clip = clip_of_col(e, col_of_key(e, key));
  if (clip < 0) return fail(e, TFP_E_NOENT, "no clip with key %d", key);
  snprintf(uuid, len, "%s", e->clips[clip].uuid.c_str());
  return TFP_OK;
}

int tfp_search_batch(tfp_engine* e, const tfp_frame* frames, const int64_t* qoff, int32_t nq,
                     const tfp_search_params* P, tfp_result* out) {
  if (!e || !qoff || nq < 0 || !out) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  const int64_t nf = nq ? qoff[nq] - qoff[0] : 0;
  if (nf && !frames) return fail(e, TFP_E_ARG, "frames is NULL");
  std::vector<unsigned long long> keys(nq, 0ull);
  if (valid_params(P) && nq) {  // coefs out of range: NULL for every query (fp_handler.c:247-250)
    HIPCHK(e, hipSetDevice(e->device));
    std::vector<double> q(2 * (nf + 1));
    for (int64_t i = 0; i < nf; i++) {
      q[2 * i] = frames[qoff[0] + i].q1;
      q[2 * i + 1] = frames[qoff[0] + i].q2;
    }
    int rc = upload(e, e->q, q.data(), sizeof(double) * q.size());
    if (rc) return rc;
    if ((rc = search_core(e, qoff, nq, e->q.as<double>(), P, keys, nullptr, e->stream))) return rc;
  }
  fill_results(e, keys, qoff, nq, out);
  return TFP_OK;
}

int tfp_search(tfp_engine* e, const tfp_frame* frames, int32_t nframes, const tfp_search_params* P, tfp_result* out) {
  if (nframes < 0) return TFP_E_ARG;
  int64_t qoff[2] = {0, nframes};
  return tfp_search_batch(e, frames, qoff, 1, P, out);
}

namespace {
// One search over host samples, the queries given as (pointer, samples); no coalescing.
int search_gather_impl(tfp_engine* e, const void* const* ptrs, const int64_t* lens, int32_t nq, bool f32, int32_t sr,
                       const tfp_search_params* P, tfp_result* out) {
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  std::vector<int64_t> foff(nq + 1, 0);
  for (int32_t i = 0; i < nq; i++) foff[i + 1] = foff[i] + tfp_frame_count(lens[i]);
  for (int32_t i = 0; e->fail_query_len >= 0 && i < nq; i++)  // (test knob: a query that fails on the device)
    if (lens[i] == e->fail_query_len)
      return fail(e, TFP_E_NOMEM, "hipMalloc for query %d of %d (%lld samples): out of memory (TFP_TEST_FAIL_QUERY_SAMPLES)", i,
                  nq, (long long)lens[i]);
  std::vector<unsigned long long> keys(nq, 0ull);
  if (valid_params(P) && nq && foff[nq] > 0) {
    int64_t nf;
    int rc = fingerprint_host(e, ptrs, lens, f32, nq, sr, &nf, nullptr, P->coefs == 2);
    if (rc) return rc;
    if ((rc = search_core(e, foff.data(), nq, e->db.as<double>(), P, keys, nullptr, e->stream))) return rc;
    e->stage_pending = false;  // search_core waited for e->stream (keys on the host)
  }
  fill_results(e, keys, foff.data(), nq, out);
  return TFP_OK;
}

// Argument checks, then the call alone (large batches, TFP_COALESCE=0) or through the coalescer.
int search_gather_entry(tfp_engine* e, const void* const* ptrs, const int64_t* lens, int32_t nq, bool f32, int32_t sr,
                        const tfp_search_params* P, tfp_result* out) {
  if (!e || nq < 0 || !out || (nq && (!ptrs || !lens))) return TFP_E_ARG;
  for (int32_t i = 0; i < nq; i++)
    if (lens[i] < 0 || (lens[i] && !ptrs[i])) return fail(e, TFP_E_ARG, "bad query %d", i);
  if (!e->coalesce || nq == 0 || nq > Coalescer::kMaxCallQueries)
    return search_gather_impl(e, ptrs, lens, nq, f32, sr, P, out);
  SearchReq r;
  r.ptrs.assign(ptrs, ptrs + nq);
  r.lens.assign(lens, lens + nq);
  r.f32 = f32;
  r.sr = sr;
  if (P) r.P = *P;
  else r.P.coefs = 0;  // (invalid: NULL results, fp_handler.c:247-250)
  r.out = out;
  const int rc = e->coal.submit(&r, [e](std::vector<SearchReq*>& batch) {
    exec_batch(
        batch,
        [e](const void* const* p, const int64_t* l, int32_t n, bool f, int32_t rate, const tfp_search_params* q,
            tfp_result* o) { return search_gather_impl(e, p, l, n, f, rate, q, o); },
        [e] { return std::string(tfp_engine_last_error(e)); });
  });
  if (rc) e->err.note(e, r.err.c_str());  // (the leader ran it: the message into this caller's slot)
  return rc;
}

int search_samples_impl(tfp_engine* e, const void* pcm, bool f32, const int64_t* offsets, int32_t nq, int32_t sr,
                        const tfp_search_params* P, tfp_result* out) {
  if (!e || !offsets || nq < 0 || !out) return TFP_E_ARG;
  for (int32_t i = 0; i < nq; i++)
    if (offsets[i + 1] < offsets[i]) return fail(e, TFP_E_ARG, "offsets not monotone");
  if (!pcm && nq && offsets[nq] > offsets[0]) return fail(e, TFP_E_ARG, "samples are NULL");
  std::vector<const void*> ptrs;
  std::vector<int64_t> lens;
  split_offsets(pcm, f32 ? sizeof(float) : sizeof(int16_t), offsets, nq, &ptrs, &lens);
  return search_gather_entry(e, ptrs.data(), lens.data(), nq, f32, sr, P, out);
}
}  // namespace

int tfp_search_pcm_batch(tfp_engine* e, const int16_t* pcm, const int64_t* offsets, int32_t nq, int32_t sr,
                         const tfp_search_params* P, tfp_result* out) {
  return search_samples_impl(e, pcm, false, offsets, nq, sr, P, out);
}

int tfp_search_f32_batch(tfp_engine* e, const float* x, const int64_t* offsets, int32_t nq, int32_t sr,
                         const tfp_search_params* P, tfp_result* out) {
  return search_samples_impl(e, x, true, offsets, nq, sr, P, out);
}

int tfp_search_pcm_gather(tfp_engine* e, const int16_t* const* pcms, const int64_t* nsamples, int32_t nq, int32_t sr,
                          const tfp_search_params* P, tfp_result* out) {
  return search_gather_entry(e, reinterpret_cast<const void* const*>(pcms), nsamples, nq, false, sr, P, out);
}

int tfp_sweep_stats(tfp_engine* e, int64_t* bins, int64_t* library, int64_t* redone, int64_t* crowd_bins) {
  if (!e) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (bins) *bins = e->n_sweep_bins;
  if (library) *library = e->n_sweep_lib;
  if (redone) *redone = e->n_sweep_redo;
  if (crowd_bins) *crowd_bins = e->n_sweep_crowd;
  return TFP_OK;
}

int tfp_index_cache_stats(tfp_engine* e, int64_t* cache_builds, int64_t* cache_hits, int64_t* from_order,
                          int64_t* order_builds, int64_t* order_merges, int64_t* delta_cache_builds,
                          int64_t* delta_sweeps) {
  if (!e) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (cache_builds) *cache_builds = e->n_cell_builds;
  if (cache_hits) *cache_hits = e->n_cell_hits;
  if (from_order) *from_order = e->n_cell_from_order;
  if (order_builds) *order_builds = e->n_order_builds;
  if (order_merges) *order_merges = e->n_order_merges;
  if (delta_cache_builds) *delta_cache_builds = e->n_delta_cell_builds;
  if (delta_sweeps) *delta_sweeps = e->n_delta_sweeps;
  return TFP_OK;
}

int64_t tfp_internal_delta_main_keys(tfp_engine* e) { return e ? e->n_delta_main_keys : 0; }
const char* tfp_internal_engine_own_error(tfp_engine* e) { return e ? e->err.own() : nullptr; }
void tfp_internal_engine_clear_error(tfp_engine* e) {
  if (e) e->err.clear_own();
}

int tfp_search_coalesce_stats(tfp_engine* e, int64_t* calls, int64_t* batches) {
  if (!e) return TFP_E_ARG;
  e->coal.stats(calls, batches);
  return TFP_OK;
}

// (internal, tfp_internal.hpp) the device group's per-shard search: already coalesced by the group
int tfp_internal_search_gather(tfp_engine* e, const void* const* ptrs, const int64_t* lens, int32_t nq, bool f32,
                               int32_t sr, const tfp_search_params* P, tfp_result* out) {
  if (!e || nq < 0 || !out || (nq && (!ptrs || !lens))) return TFP_E_ARG;
  return search_gather_impl(e, ptrs, lens, nq, f32, sr, P, out);
}

int tfp_search_device(tfp_engine* e, const tfp_plan* p, const int16_t* d_pcm, const tfp_search_params* P,
                      uint64_t* d_keys, void* stream) {
  if (!e || !p || !d_keys || !valid_params(P)) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  NullStreamOrder order(e, stream);
  if (!order.ok()) return fail(e, TFP_E_HIP, "ordering after the null stream failed");
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  const DspTables* T;
  bool fx = false;
  int rc = ensure_tables(e, p->sample_rate, &T, &fx);
  if (rc) return rc;
  HIPCHK(e, e->micro.reserve(sizeof(int32_t) * 2 * (p->nframes + 1)));
  HIPCHK(e, e->db.reserve(sizeof(double) * 2 * (p->nframes + 1)));
  HIPCHK(e, launch_fingerprint(e->fpcfg, T, fx && !p->long_clip, p->tile_frames, d_pcm, p->d_soff.as<int64_t>(), p->d_soff.as<int64_t>() + 1,
                               p->d_foff.as<int64_t>(), p->d_toff.as<int32_t>(),
                               p->d_tclip.as<int32_t>(), p->ntiles, p->nframes, e->micro.as<int32_t>(),
                               e->db.as<double>(), s, P->coefs == 2 ? e->logfix : LogFix{}));
  std::vector<unsigned long long> keys;
  return search_core(e, p->foff.data(), p->nclips, e->db.as<double>(), P, keys,
                     reinterpret_cast<unsigned long long*>(d_keys), s);
}

int tfp_search_q_device(tfp_engine* e, const double* d_q, const int64_t* qoff, int32_t nq, const tfp_search_params* P,
                        uint64_t* d_keys, void* stream) {
  if (!e || !qoff || nq < 0 || !d_keys || !valid_params(P) || (!d_q && nq && qoff[nq] > qoff[0])) return TFP_E_ARG;
  for (int32_t i = 0; i < nq; i++)
    if (qoff[i + 1] < qoff[i]) return fail(e, TFP_E_ARG, "query offsets not monotone");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  NullStreamOrder order(e, stream);
  if (!order.ok()) return fail(e, TFP_E_HIP, "ordering after the null stream failed");
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  std::vector<unsigned long long> keys;
  return search_core(e, qoff, nq, d_q ? d_q + 2 * qoff[0] : d_q, P, keys, reinterpret_cast<unsigned long long*>(d_keys),
                     s);
}

// ---- streams ------------------------------------------------------------------------------

struct tfp_stream {
  tfp_engine* eng = nullptr;
  int32_t nch = 0, sr = 0;
  int64_t W = 0;                 // window samples
  int64_t wpos = 0;              // ring position of the oldest sample of every window
  std::vector<int64_t> filled;   // samples of history per channel (saturates at W)
  DevBuf ring;
  HostBuf stage_h;               // this tick's samples + window layout: mapped, coherent pinned memory
  void* stage_host = nullptr;    // the allocation stage_dev was taken for
  char* stage_dev = nullptr;     // its device address: the kernels read it in place (no upload)
  bool stage_pending = false;    // stage_h may still be read by the last tick's kernels
};

// ring[c][2W]: every sample is written at p and p + W, so the last W samples of a channel are
// always the contiguous run ring[c][wpos .. wpos + W).
__global__ void stream_scatter_kernel(const int16_t* __restrict__ tick, int32_t T, int64_t W, int64_t wpos,
                                      int32_t nch, int16_t* __restrict__ ring) {
  const int64_t n = (int64_t)nch * T;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i / T, t = i % T;
    int64_t p = wpos + t;
    if (p >= W) p -= W;
    const int16_t v = tick[i];
    ring[c * 2 * W + p] = v;
    ring[c * 2 * W + p + W] = v;
  }
}

int tfp_stream_create(tfp_engine* e, int32_t nch, int32_t sr, int64_t W, tfp_stream** out) {
  if (!e || nch <= 0 || W <= 0 || !out) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  const DspTables* T;
  int rc = ensure_tables(e, sr, &T);
  if (rc) return rc;
  tfp_stream* st = new tfp_stream();
  st->eng = e;
  st->nch = nch;
  st->sr = sr;
  st->W = W;
  st->filled.assign(nch, 0);
  if (st->ring.reserve(sizeof(int16_t) * 2 * W * nch) != hipSuccess) {
    delete st;
    return fail(e, TFP_E_NOMEM, "stream ring of %lld bytes", (long long)(4 * W * nch));
  }
  (void)hipMemsetAsync(st->ring.p, 0, sizeof(int16_t) * 2 * W * nch, e->stream);
  *out = st;
  return TFP_OK;
}

void tfp_stream_destroy(tfp_stream* st) {
  if (!st) return;
  {
    std::lock_guard<std::recursive_mutex> lk(st->eng->mu);
    (void)hipSetDevice(st->eng->device);
    (void)hipStreamSynchronize(st->eng->stream);  // the last tick's kernels may still read stage_h
  }
  delete st;
}

int tfp_stream_reset(tfp_stream* st, int32_t ch) {
  if (!st || ch >= st->nch) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(st->eng->mu);
  if (ch < 0) std::fill(st->filled.begin(), st->filled.end(), 0);
  else st->filled[ch] = 0;
  return TFP_OK;
}

// One tick into a stream: the samples into the ring, then (match) the windows that are full after
// it fingerprinted into d_db (frame values, 2 doubles per frame; nullptr: the engine's buffer) at
// window i's frames [i F, (i + 1) F). act = their channels, in channel order. Caller holds e->mu.
static int stream_tick(tfp_stream* st, const int16_t* pcm, int32_t T, const tfp_search_params* P, double* d_db,
                       int64_t cap_frames, std::vector<int32_t>& act, int64_t* F_out, std::vector<int64_t>& fov) {
  const bool match = P && valid_params(P);
  tfp_engine* e = st->eng;
  HIPCHK(e, hipSetDevice(e->device));
  int rc;
  // Windows to match after this tick: the channels whose history is full once it is in.
  const int64_t wpos = (st->wpos + T) % st->W;
  act.clear();
  if (match)
    for (int32_t c = 0; c < st->nch; c++)
      if (std::min<int64_t>(st->W, st->filled[c] + T) >= st->W) act.push_back(c);
  const int32_t na = (int32_t)act.size();
  const int64_t F = tfp_frame_count(st->W);
  *F_out = F;
  if (d_db && (int64_t)na * F > cap_frames) return fail(e, TFP_E_ARG, "stream tick: %d windows of %lld frames past %lld", na,
                                                        (long long)F, (long long)cap_frames);
  const DspTables* Tb;
  bool fx = false;
  if ((rc = ensure_tables(e, st->sr, &Tb, &fx))) return rc;
  const int32_t tile = fp_tile_frames(e->fpcfg, fx, false, false);
  const int32_t tiles = (int32_t)((F + tile - 1) / tile);
  // One mapped pinned buffer per tick, read in place by the kernels: the tick's samples, then the
  // windows' layout (sbeg, send, foff, toff, tclip). An upload and its hand-off to the first
  // kernel cost ~16 us a tick. The previous tick's kernels must be done reading the buffer.
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t b_pcm = al(sizeof(int16_t) * (size_t)st->nch * T), b_sb = al(sizeof(int64_t) * na),
               b_fo = al(sizeof(int64_t) * (na + 1)), b_to = al(sizeof(int32_t) * (na + 1)),
               b_tc = al(sizeof(int32_t) * (size_t)na * tiles);
  const size_t total = b_pcm + 2 * b_sb + b_fo + b_to + b_tc;
  if (st->stage_pending) HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, st->stage_h.reserve(total, hipHostMallocMapped | hipHostMallocCoherent));
  if (st->stage_h.p != st->stage_host) {
    HIPCHK(e, hipHostGetDevicePointer(reinterpret_cast<void**>(&st->stage_dev), st->stage_h.p, 0));
    st->stage_host = st->stage_h.p;
  }
  char* h = st->stage_h.as<char>();
  memcpy(h, pcm, sizeof(int16_t) * (size_t)st->nch * T);
  int64_t* sb = reinterpret_cast<int64_t*>(h + b_pcm);
  int64_t* se = reinterpret_cast<int64_t*>(h + b_pcm + b_sb);
  int64_t* fo = reinterpret_cast<int64_t*>(h + b_pcm + 2 * b_sb);
  int32_t* to = reinterpret_cast<int32_t*>(h + b_pcm + 2 * b_sb + b_fo);
  int32_t* tc = reinterpret_cast<int32_t*>(h + b_pcm + 2 * b_sb + b_fo + b_to);
  for (int32_t i = 0; i < na; i++) {
    sb[i] = (int64_t)act[i] * 2 * st->W + wpos;
    se[i] = sb[i] + st->W;
    fo[i] = (int64_t)i * F;
    to[i] = i * tiles;
    for (int32_t t = 0; t < tiles; t++) tc[(size_t)i * tiles + t] = i;
  }
  fo[na] = (int64_t)na * F;
  to[na] = na * tiles;
  st->stage_pending = true;
  const char* d = st->stage_dev;
  hipLaunchKernelGGL(stream_scatter_kernel, dim3(1024), dim3(256), 0, e->stream, reinterpret_cast<const int16_t*>(d), T,
                     st->W, st->wpos, st->nch, st->ring.as<int16_t>());
  HIPCHK(e, hipGetLastError());
  st->wpos = wpos;
  for (auto& f : st->filled) f = std::min<int64_t>(st->W, f + T);
  fov.assign(fo, fo + na + 1);  // (the pinned buffer is rewritten next tick)
  if (!na) return TFP_OK;
  HIPCHK(e, e->micro.reserve(sizeof(int32_t) * 2 * (fo[na] + 1)));
  if (!d_db) HIPCHK(e, e->db.reserve(sizeof(double) * 2 * (fo[na] + 1)));
  const int64_t* d_sb = reinterpret_cast<const int64_t*>(d + b_pcm);
  HIPCHK(e, launch_fingerprint(e->fpcfg, Tb, fx, tile, st->ring.as<int16_t>(), d_sb,
                               reinterpret_cast<const int64_t*>(d + b_pcm + b_sb),
                               reinterpret_cast<const int64_t*>(d + b_pcm + 2 * b_sb),
                               reinterpret_cast<const int32_t*>(d + b_pcm + 2 * b_sb + b_fo),
                               reinterpret_cast<const int32_t*>(d + b_pcm + 2 * b_sb + b_fo + b_to), to[na], fo[na],
                               e->micro.as<int32_t>(), d_db ? d_db : e->db.as<double>(), e->stream,
                               P->coefs == 2 ? e->logfix : LogFix{}));
  return TFP_OK;
}

int tfp_stream_push(tfp_stream* st, const int16_t* pcm, int32_t T, const tfp_search_params* P, tfp_result* out) {
  if (!st || !pcm || T <= 0 || T > st->W || (P && !out)) return TFP_E_ARG;
  tfp_engine* e = st->eng;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  const bool match = P && valid_params(P);  // fp_handler.c:247-250: bad params -> NULL results
  std::vector<int32_t> act;
  std::vector<int64_t> fov;
  int64_t F = 0;
  int rc = stream_tick(st, pcm, T, P, nullptr, 0, act, &F, fov);
  if (rc) return rc;
  if (!P) return TFP_OK;
  for (int32_t c = 0; c < st->nch; c++) {
    memset(&out[c], 0, sizeof out[c]);
    out[c].clip_id = -1;
  }
  const int32_t na = (int32_t)act.size();
  if (!match || !na) return TFP_OK;  // full windows only
  std::vector<unsigned long long> keys;
  if ((rc = search_core(e, fov.data(), na, e->db.as<double>(), P, keys, nullptr, e->stream))) return rc;
  st->stage_pending = false;  // search_core waited for e->stream
  std::vector<tfp_result> res(na);
  fill_results(e, keys, fov.data(), na, res.data());
  for (int32_t i = 0; i < na; i++) out[act[i]] = res[i];
  return TFP_OK;
}

int tfp_internal_stream_fp(tfp_stream* st, const int16_t* pcm, int32_t T, const tfp_search_params* P, double* d_db,
                           int64_t cap_frames, int32_t* act, int32_t* nact, int64_t* frames_per_window) {
  const bool match = P && valid_params(P);
  if (!st || !pcm || T <= 0 || T > st->W || !nact || !frames_per_window || (match && (!d_db || !act))) return TFP_E_ARG;
  tfp_engine* e = st->eng;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  std::vector<int32_t> a;
  std::vector<int64_t> fov;
  int rc = stream_tick(st, pcm, T, P, d_db, cap_frames, a, frames_per_window, fov);
  if (rc) return rc;
  HIPCHK(e, hipStreamSynchronize(e->stream));  // the values are read by other devices' streams next
  st->stage_pending = false;
  *nact = (int32_t)a.size();
  if (match) std::copy(a.begin(), a.end(), act);
  return TFP_OK;
}

int tfp_synth_pcm(const tfp_synth_spec* specs, int32_t nclips, int64_t spc, int16_t* out) {
  if (nclips < 0 || spc < 0 || (nclips && (!specs || !out))) return TFP_E_ARG;
  for (int32_t c = 0; c < nclips; c++) {
    const SynthClip p = synth_clip(specs[c].seed, specs[c].clip);
    for (int64_t s = 0; s < spc; s++) out[(int64_t)c * spc + s] = synth_sample(p, specs[c].offset + s);
  }
  return TFP_OK;
}

int tfp_synth_pcm_device(tfp_engine* e, const tfp_synth_spec* specs, int32_t nclips, int64_t spc, int16_t* d_out,
                         void* stream) {
  if (!e || nclips < 0 || spc < 0 || (nclips && (!specs || !d_out))) return TFP_E_ARG;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(e, hipSetDevice(e->device));
  NullStreamOrder order(e, stream);
  if (!order.ok()) return fail(e, TFP_E_HIP, "ordering after the null stream failed");
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  static_assert(sizeof(tfp_synth_spec) == sizeof(SynthSpecDev), "spec layout");
  int rc = upload(e, e->specs, specs, sizeof(tfp_synth_spec) * nclips);
  if (rc) return rc;
  if (s != e->stream) HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, launch_synth(e->specs.as<SynthSpecDev>(), nclips, spc, d_out, s));
  HIPCHK(e, hipStreamSynchronize(s));  // specs buffer is reused by the next call
  return TFP_OK;
}

int tfp_synchronize(tfp_engine* e, void* stream) {
  if (!e) return TFP_E_ARG;
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(stream ? (hipStream_t)stream : e->stream));
  return TFP_OK;
}

}  // extern "C"
