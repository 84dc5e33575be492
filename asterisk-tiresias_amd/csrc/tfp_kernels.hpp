// tfp_kernels.hpp — host-callable launchers for the gfx950 kernels (internal interface).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "tfp_math.hpp"
#include "tfp_tables.hpp"

namespace tfp {

// Test and diagnostic knobs (TFP_GENERIC, TFP_WIDE_POINTS, TFP_INDEX_FULL, ...): each forces a
// form that some input reaches on its own, or injects a failure, so the -m gpu suite can run every
// form against the oracle. They are read only when TFP_TEST_KNOBS is set (tests/conftest.py sets
// it), so the environment of a production process cannot change which kernel a search runs.
inline const char* knob(const char* name) {
  const char* on = getenv("TFP_TEST_KNOBS");
  return on && *on && strcmp(on, "0") != 0 ? getenv(name) : nullptr;
}
// The operational switches the public header and INTEGRATION.md document (TFP_COALESCE=0,
// TFP_INDEX_DELTA=0, TFP_GROUP_STREAM=replicate): plain environment reads, TFP_TEST_KNOBS or not.
// Each picks a form whose results are identical, so none can change what a search returns.
inline const char* op_env(const char* name) {
  const char* v = getenv(name);
  return v && *v ? v : nullptr;
}

constexpr int kFramesPerBlock = 16;   // frames per wave tile of the generic kernel (16 lanes per frame)
// Frames per wave tile of fingerprint8k_kernel's throughput launches. 16: the tile tail (deferred
// logs, DCT) amortised over 4 passes. Measured, not kept: 8-frame tiles with the smaller log
// buffer that lets 3 workgroups (3 waves/SIMD at <= 168 VGPRs) share a CU: 0.565 ms per C2
// launch vs 0.536 (the LDS array is ~50 % busy at 2 waves/SIMD; a third wave adds contention).
constexpr int kTile8k = 16;
// fingerprint8k_kernel's throughput launches read a clip through a buffer resource whose range and
// offsets are 32-bit byte counts: clips of this many samples or more take the generic kernel
// (64-bit sample offsets) instead. (2^30 samples = 37 hours at 8 kHz.)
constexpr int64_t kDirectMaxSamples = (int64_t(1) << 30) - (int64_t(1) << 16);
constexpr int32_t kKeyOffset = 512;   // trunc(dB) key k stored at k + 512 (|k| <= 459)
constexpr int32_t kKeyRange = 1024;

// One query frame's search box (fp_handler.c:287-351 restated). flags: 1 = the frame runs
// its SQL (not ignored, bounds printable), 2 = the max2 condition is present.
struct FrameBox {
  int64_t L1, U1, L2, U2;
  int32_t k;
  int32_t flags;
};

struct SearchConsts {
  int32_t coefs;
  int32_t has_low, has_high;
  int32_t pad;
  double tole, thr_low, thr_high;
};

struct SynthSpecDev {
  uint64_t seed;
  int64_t clip;
  int64_t offset;
};

// Fingerprint clips: clip c = samples [sbeg[c], send[c]) of d_pcm (for concatenated clips pass
// send = soff + 1); frames of clip c are written from foff[c]; toff[nclips+1] are 16-frame tile
// offsets (ntiles = toff[nclips]) and tclip[tile] the clip of each tile.
// Per-engine launch configuration: read once when the engine is created (fp_launch_config),
// grid caps from the engine's own device.
struct FpLaunchCfg {
  int32_t grid_cap_8k = 0;       // resident blocks of fingerprint8k_kernel (kTile8k-frame tiles) on the device
  int32_t grid_cap_8k_small = 0; // ... of its 4-frame-tile form (small batches)
  int32_t grid_cap_generic = 0;  // resident blocks of fingerprint_kernel<int16_t>
  int32_t grid_cap_f32 = 0;      // resident blocks of fingerprint_kernel<float>
  bool force_generic = false;    // TFP_GENERIC=1: the generic kernel at 8 kHz too (tests)
  float rare_thr = 0x1p-98f;     // TFP_RARE_THR_LOG2=n: bins with 0 < |S|^2 < 2^n take the spec-order path (tests)
};
// Fills cfg for `device` (occupancy queries + the test knobs from the environment).
hipError_t fp_launch_config(int device, FpLaunchCfg* cfg);
inline int32_t fp_tile_frames(const FpLaunchCfg& cfg, bool fixed8k, bool f32, bool small) {
  if (!fixed8k || f32) return kFramesPerBlock;
  if (small) return 4;
  return cfg.force_generic ? kFramesPerBlock : kTile8k;
}
// fixed8k: the tables' filterbank schedule is the 8 kHz one (DspTables_fixed8k), so the
// specialized fingerprint8k_kernel runs; otherwise the generic fingerprint_kernel.
bool DspTables_fixed8k(const DspTables& t);
// tile_frames: frames per wave tile in toff/tclip: fp_tile_frames() — kFramesPerBlock for the
// generic kernel, kTile8k (or 4 for small batches) for fingerprint8k_kernel.
hipError_t launch_fingerprint(const FpLaunchCfg& cfg, const DspTables* d_tables, bool fixed8k, int32_t tile_frames,
                              const int16_t* d_pcm, const int64_t* d_sbeg, const int64_t* d_send, const int64_t* d_foff,
                              const int32_t* d_toff, const int32_t* d_tclip, int32_t ntiles, int64_t nframes,
                              int32_t* d_micro, double* d_db, hipStream_t s, const LogFix& fx,
                              int64_t single_ns = -1);
// single_ns >= 0 (8 kHz kernel): the batch is one clip of single_ns samples at d_pcm[0], frames from
// 0, so the kernel takes its tile bounds from the argument instead of a chain of layout loads
// (batch-1: the first PCM request goes out at the kernel's first instruction).
// fx: the glibc log correction table (device copy; tfp_math.hpp LogFix) used for d_db's frame
// values, so they equal glibc's 10*log10|c| bit for bit (the stored micro-units need none).
// fp32 samples (the values aubio_source_do produces: multichannel mean, 24/32-bit or float
// WAV, tfp_wav_decode_f32) through the generic kernel, 16-frame tiles; same outputs as above.
hipError_t launch_fingerprint_f32(const FpLaunchCfg& cfg, const DspTables* d_tables, const float* d_x,
                                  const int64_t* d_sbeg, const int64_t* d_send, const int64_t* d_foff,
                                  const int32_t* d_toff, const int32_t* d_tclip, int32_t ntiles, int32_t* d_micro,
                                  double* d_db, hipStream_t s, const LogFix& fx);

hipError_t launch_synth(const SynthSpecDev* d_specs, int32_t nclips, int64_t spc, int16_t* d_out, hipStream_t s);

// Index build: key = m1 (or INT32_MAX for rows that never match), value = staging index.
hipError_t launch_index_keys(const int32_t* st_m1, const int32_t* st_clip, const int32_t* rank_of_clip,
                             int64_t n, int32_t* keys, int32_t* vals, hipStream_t s);
hipError_t launch_index_gather(const int32_t* sorted_vals, const int32_t* st_m2, const int32_t* st_clip,
                               const int32_t* rank_of_clip, int64_t n, int32_t* m2s, int32_t* cols, hipStream_t s);
hipError_t launch_count_below(const int32_t* sorted_keys, int64_t n, int32_t bound, int64_t* out, hipStream_t s);
hipError_t radix_sort_pairs(void* temp, size_t* temp_bytes, const int32_t* kin, int32_t* kout, const int32_t* vin,
                            int32_t* vout, int64_t n, hipStream_t s);

// Search.
// Also zeroes zero_words[0, nzero) (the vote path's mask, max count and best keys).
hipError_t launch_prep_boxes(const double* d_q, int64_t nframes, SearchConsts sc, FrameBox* boxes, uint32_t* zero_words,
                             int32_t nzero, hipStream_t s);
// Used-key mask of all nf frames (d_mask zeroed); a key outside the vote range sets *d_maxc = INT32_MAX.
struct VoteMeta;
// Sets d_meta->ok (the vote's exactness flag, cleared later by build_A) as well.
hipError_t launch_key_mask(const double* d_q, SearchConsts sc, int64_t nf, uint32_t* d_mask /*[kKeyRange/32]*/,
                           int32_t* d_maxc /*zeroed*/, VoteMeta* d_meta, hipStream_t s);
// Row ranges of all kKeyRange keys' boxes at one tolerance (the engine caches them per index version).
hipError_t launch_key_ranges_all(const int32_t* m1s, int64_t R, double tole, int64_t* d_rng_all /*[kKeyRange][2]*/,
                                 hipStream_t s);
// Vote path bookkeeping computed on the GPU by key_mask (ok) and build_A's block 0 (read by the
// later kernels).
struct VoteMeta {
  int32_t ku;  // used keys
  int32_t kp;  // GEMM K: Ku + 1 (the packed-argmax column) rounded up to 16
  int32_t ok;  // counts exact in fp16 and keys in range: else the host redoes the batch on the scan path
  int32_t cls; // pattern-class path (Ku <= class_ku_max) instead of the Bt GEMM
};
constexpr int32_t kVoteKpMax = ((kKeyRange + 1 + 15) / 16) * 16;
// A[q][kc] per-query counts of the used keys (ascending key = column kc), derived by every block
// from the key mask; block 0 writes VoteMeta (ku, kp, cls; ok cleared for an out-of-range key);
// on the class path the grid clears the pattern maxima at the head of d_Bt.
hipError_t launch_build_A(const double* d_q, SearchConsts sc, const int64_t* d_qoff, int32_t nq, int32_t Qp,
                          const uint32_t* d_mask, const int32_t* d_maxc, VoteMeta* d_meta, int32_t class_ku_max,
                          _Float16* d_A, _Float16* d_Bt /*the class path's pattern maxima are cleared*/, int32_t Cp,
                          hipStream_t s);
hipError_t launch_build_B(const uint32_t* d_mask /*key mask words*/, const uint32_t* d_bits /*launch_key_bits*/,
                          int32_t C, const VoteMeta* d_meta, int32_t Cp, _Float16* d_Bt /*[Cp][kVoteKpMax]*/,
                          hipStream_t s);
// Partial results: d_part holds vote_chunks(Cp) x Qp keys.
int32_t vote_chunks(int32_t Cp);
hipError_t launch_vote_gemm(const _Float16* d_A, _Float16* d_Bt, int32_t Qp, int32_t Cp, const VoteMeta* d_meta,
                            const int32_t* d_tiekey, unsigned long long* d_part, unsigned long long* d_best,
                            const uint32_t* d_mask /*key mask words*/, const uint32_t* d_bits /*launch_key_bits*/,
                            int32_t C, hipStream_t s);

// ---- small-batch search (batch-1 latency path; coefs = 1, nq <= kSmallQ, <= 2048 frames per query):
// one launch after the queries' fingerprint launch, no host round trip and no copy back. Every
// block of small_vote derives the batch's used keys and per-query key counts from the query
// frames itself (a few KB of L2-resident reads) and scores its clips from the key-presence
// bitsets (launch_key_bits: bit c of key k's row = clip column c has a row in k's box, cached per
// index version and tolerance, as the boxes' row ranges are); it arg-maxes per block and writes
// its per-query maxima straight into the caller's host-mapped SmallResult, and the caller takes
// the max over the blocks once the stream is done (no publishing kernel, no device atomics).
constexpr int kSmallQ = 8;
struct SmallQueries {
  int32_t nq;
  int32_t pad;
  int64_t qoff[kSmallQ + 1];  // frame offsets of the queries in d_q (relative)
};
// Host-mapped (pinned, coherent) result of one small call: the header, then small_vote's per-block
// maxima part[block][query] (score << 32 | tie key, 0 = no hit) for the small_vote_blocks(C) blocks.
// Written only when !bad and ku > 0; valid once the stream is done.
struct SmallResult {
  int32_t ku;   // used keys (0: every frame was ignored, NOTFOUND)
  int32_t bad;  // a key outside [-512, 511]: the caller redoes the batch generally
};
constexpr int kSmallVoteClips = 1024;  // clips per small_vote block (4 per thread)
inline int32_t small_vote_blocks(int32_t C) { return (C + kSmallVoteClips - 1) / kSmallVoteClips; }
inline size_t small_result_bytes(int32_t C) {
  return sizeof(SmallResult) + sizeof(unsigned long long) * kSmallQ * (size_t)small_vote_blocks(C);
}
TFP_HD unsigned long long* small_result_parts(SmallResult* r) { return reinterpret_cast<unsigned long long*>(r + 1); }
// Key-presence bitsets: d_bits[k][w] (kKeyRange rows of W = key_bits_words(C) words), bit c of row
// k set iff column c has an index row in key k's box (d_rng_all, the cached row ranges). Cleared
// and rebuilt on the stream. rows_bound: at least the sum of the boxes' row counts (sizes the
// grid; more is harmless). win (LDS words per column window) and direct (pieces below it use
// global atomics): <= 0 / < 0 for the defaults; tests force small windows and either path.
TFP_HD int32_t key_bits_words(int32_t C) { return (C + 127) / 128 * 4; }  // rows 16-byte aligned
hipError_t launch_key_bits(const int64_t* d_rng_all, const int32_t* cols, int32_t C, int64_t rows_bound, int32_t win,
                           int64_t direct, uint32_t* d_bits, hipStream_t s);
// h_out: host-mapped memory of small_result_bytes(C) the device writes.
hipError_t launch_search_small(const double* d_q, const SmallQueries& sq, SearchConsts sc, const uint32_t* d_bits,
                               int32_t C, const int32_t* d_tiekey, SmallResult* h_out, hipStream_t s);

// A grow-only device buffer (the clip-set cache's arrays and scratch): rebuilds reuse the space, so
// no hipFree (which synchronises the device) runs between builds.
struct CacheBuf {
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t reserve(size_t n);  // grow-only, 1/8 headroom
  void release();
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// The index rows in clip order (round 6, tfp_scan.hip): every row of the m1-sorted index as
// key = t << 53 | column << 32 | (m2 ^ INT32_MIN), t = the key index (k + kKeyOffset, clamped to
// [0, kKeyRange)) of the integer k nearest its max1 (floor((m1 + 500000) / 10^6)), ascending, with
// the row's m1 beside it. For a tolerance below 1/2 the "%f" max1 box of key k lies inside the rows
// whose nearest integer is k, so the clip-set cache at such a tolerance is a filter of this order
// (rows whose m1 lies in their key's box), no sort: the order is built once (a radix sort) and
// carried across index merges (launch_order_merge, tfp_index.hip).
constexpr double kOrderMaxTol = 0.49;  // tolerances the order serves (fmt6(k +- tol) stays inside k's rows)
hipError_t launch_order_fill(const int32_t* m1s, const int32_t* m2s, const int32_t* cols, int64_t R,
                             unsigned long long* okey, int32_t* om1, hipStream_t s);
hipError_t order_sort(const unsigned long long* kin, unsigned long long* kout, const int32_t* vin, int32_t* vout, int64_t n,
                      CacheBuf* tmp, hipStream_t s);
// The clip order of an index delta's staged rows (round 6): delta clip j (uuid order; tfp_index.hpp
// DeltaClip) takes the local column j; rows are written clip after clip (unsorted: order_sort
// follows).
struct DeltaClip;
hipError_t launch_delta_order_fill(const DeltaClip* d_dc, int32_t nd, const int32_t* st_m1, const int32_t* st_m2,
                                   unsigned long long* okey, int32_t* om1, hipStream_t s);

// General path (coefs = 2 and the vote's fallbacks; tfp_scan.hip). Clip-set cache of one index
// version and tolerance: per (key, clip) group the clip's max2 values in the key's "%f" max1 box
// ("points", ascending), the groups' clusters and the sweep's per-key window directory; and, for
// the one-wave-per-frame cells form only (ensure_entries, built when that form first runs), the
// cell entries (key, cell, clip) of the max2 axis cut into cells of width w. Built from the clip
// order at tolerances up to kOrderMaxTol (build_from_order: hand-written filter / scan kernels), else
// by sorting the boxes' rows (build). Not built (valid = false) past its limits: then every frame
// takes the row scan.
struct CellCache {
  static constexpr int32_t kMaxCols = 1 << 21;  // clip columns packed in 21 bits
  int32_t* p_m2 = nullptr;                 // [S] points of each group, ascending
  uint32_t* k32 = nullptr;                 // [S] key << 21 | column of each point
  uint32_t* g_key = nullptr;               // [n1] key << 21 | column of each group, ascending
  int32_t* g_beg = nullptr;                // [n1 + 1] first point of each group
  unsigned long long* e_key = nullptr;     // [n2] key << 52 | cell << 21 | column, ascending (ensure_entries)
  int32_t* e_grp = nullptr;                // [n2] group of each entry
  int32_t* k_gbeg = nullptr;               // [kKeyRange + 1] first group of each key
  // Clusters (the sweep's form of the points): a group's points cut where consecutive points are
  // more than dgap micro-units apart, each kept as its (first, last) point. A window of width >=
  // dgap - 1 that reaches from a cluster's first to its last point holds one of its points, so
  // the sweep searches 2 bounds per cluster instead of 2 per point. dgap = max(0, floor(2 tol 1e6)
  // - 3), the least window width at this tolerance (launch_scan_wide checks every frame's).
  int32_t* c_lo = nullptr;                 // [nc] first point of each cluster
  int32_t* c_hi = nullptr;                 // [nc] last point of each cluster
  int32_t* c_beg = nullptr;                // [n1 + 1] first cluster of each group
  // the clip-major sweep's directory: kdir[k][w] = first group of key k with column >= kWin w
  static constexpr int32_t kWin = 16;
  int32_t* kdir = nullptr;                 // [kKeyRange][nwin + 1]
  int32_t nwin = 0;                        // ceil(columns / kWin)
  int64_t S = 0, n1 = 0, n2 = 0, w = 0, nc = 0, dgap = 0;
  bool valid = false;
  bool entries = false;     // e_key / e_grp built
  bool from_order = false;  // built by build_from_order (tests: tfp_index_cache_stats)
  hipError_t build(const int64_t* d_rng_all, const int64_t* h_off, const int32_t* m2s, const int32_t* cols,
                   int32_t ncols, int64_t nrows, double tole, hipStream_t s);
  // from the clip order (okey, om1: n rows) at tolerance tole <= kOrderMaxTol; d_kbox = the keys'
  // "%f" boxes at tole (launch_key_boxes)
  hipError_t build_from_order(const unsigned long long* okey, const int32_t* om1, int64_t n, const int64_t* d_kbox,
                              int32_t ncols, double tole, hipStream_t s);
  hipError_t ensure_entries(hipStream_t s);
  void invalidate() { valid = entries = from_order = false; S = n1 = n2 = nc = 0; }
  void release();
  void swap(CellCache& o);
  CellCache() = default;
  CellCache(const CellCache&) = delete;
  CellCache& operator=(const CellCache&) = delete;
  ~CellCache() { release(); }

 private:
  CacheBuf b_p_m2, b_k32, b_g_key, b_g_beg, b_e_key, b_e_grp, b_k_gbeg, b_c_lo, b_c_hi, b_c_beg, b_kdir, b_tile;
  void bind();  // the array pointers from the buffers
};
// Queries [q_begin, q_begin + nq) of the batch (frame boxes from prep_boxes, offsets d_qoff on the
// device and h_qoff on the host); d_best[q] = (count << 32 | tie key), 0 = NOTFOUND.
// d_stamp / d_score / d_touched: nq x C int32, d_tcnt: nq int32; all zero on entry and on return.
hipError_t launch_scan(const FrameBox* boxes, const int64_t* d_qoff, const int64_t* h_qoff, int32_t q_begin, int32_t nq,
                       const int32_t* m1s, const int32_t* m2s, const int32_t* cols, int64_t R, const CellCache* cells,
                       const int32_t* d_tiekey, int32_t C, int32_t* d_stamp, int32_t* d_score, int32_t* d_touched,
                       int32_t* d_tcnt, unsigned long long* d_best, hipStream_t s);

// The general path's sweep by groups (tfp_scan.hip): every query frame of the batch sorted by
// (query chunk, key, max2 window); per chunk and window of 16 clip columns, one wave counts, for
// the chunk's 128 or 256 queries at once, the frames whose window holds one of each clip group's
// points (prefix counts over the sorted frames), so its work follows the groups, not the hits.
// Needs every frame's key inside the clip-set cache.
struct WideScratch {
  static constexpr int32_t kChunk = 128;  // queries per chunk: two per lane (a word of two 16-bit counts)
  // all sized by reserve for nf frames and nq queries
  unsigned long long *ka = nullptr, *kb = nullptr;  // sort keys
  uint32_t *ua = nullptr, *ub = nullptr;
  int32_t *va = nullptr, *vb = nullptr;             // frame indices
  int32_t *L2s = nullptr, *U2s = nullptr;           // sorted windows
  uint8_t* qis = nullptr;                            // sorted frames' query within its chunk
  int32_t* fq = nullptr;                             // [nf] each frame's query
  uint32_t* P = nullptr;                             // [nf][kChunk / 2] in-chunk prefix counts, 16-bit pairs (< 2^16: every query < 65536 frames)
  uint32_t* ptot = nullptr;                          // [nchunks][256][kChunk / 2] the prefix counts' per-share totals, then their prefix
  int32_t* seg = nullptr;                            // [nchunks][2 * kKeyRange][2] sorted range
  int32_t* cbeg = nullptr;                           // [nchunks + 1] first sorted frame of each chunk
  int32_t* info = nullptr;                           // [4]: frames kept, ineligible frames, wide windows, crowd bins
  int32_t* doff = nullptr;                           // [nchunks * kKeyRange + 1] each window segment's directory offset
  int32_t* dtab = nullptr;                           // [<= 4 nf] segment directories: first frame per L2 / U2 bucket
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  void* dtmp = nullptr;                              // the directory offsets' scan
  size_t dtmp_bytes = 0;
  int64_t cap_nf = 0, cap_nch = 0, cap_dtab = 0;
  int64_t min_width = -1;                            // prepare: every max2 window is at least this wide (-1: unknown)
  bool spec = false;                                 // prepare ran without reading info back: the caller checks it with the results
  // test knobs (TFP_TEST_KNOBS; each forces a form that other batches reach on their own):
  bool points_only = false;                          // TFP_WIDE_POINTS: search points, not clusters
  bool ch128 = false;                                // TFP_WIDE_CH128: 128-query chunks only
  bool unpacked = false;                             // TFP_WIDE_UNPACKED: sort (key, frame) pairs, no packed key
  int32_t qch = kChunk;                              // prepare: queries per chunk of this batch (128, or 256 with 8-bit counts)
  int32_t* ukeys = nullptr;                          // [nchunks][kKeyRange] each chunk's used keys, ascending
  int32_t* nuk = nullptr;                            // [nchunks] their number
  bool ukeys_ready = false;                          // prepare wrote ukeys / nuk (the bin sort)
  bool libsort = false;                              // TFP_WIDE_LIBSORT: the library sort on the speculative pass too
  long long* wclk = nullptr;                         // (TFP_DEBUG_BINS: the bin sort's wave clocks)
  bool debug_bins = false;                           // TFP_DEBUG_BINS: the bin sort's counts on stderr
  // the bin sort (tfp_scan.hip wide_bin_hist ...): per (chunk, segment) frame count and L2 range,
  // per chunk and bin the frame count and first sorted frame, each window segment's first / last
  // L2 and U2
  uint32_t* segstat = nullptr;
  int32_t *ghist = nullptr, *bstart = nullptr;
  int4* segk = nullptr;  // per (chunk, window segment): {min L2, min U2, bucket shift, directory offset}
  int4* gi4 = nullptr;                               // sort groups per chunk (tfp_scan.hip wide_bin_scan)
  int32_t* gb = nullptr;
  int64_t cap_groups = 0;
  unsigned long long* part = nullptr;                // [nchunks][<= 1024 waves][kChunk] the clip-major sweep's per-wave maxima
  hipError_t reserve(int64_t nf, int32_t nq, hipStream_t s);
  void release();
  WideScratch() = default;
  WideScratch(const WideScratch&) = delete;
  WideScratch& operator=(const WideScratch&) = delete;
  ~WideScratch() { release(); }
};
// Sorts the batch's frames; *eligible = false (nothing else queued) when a frame needs the row
// scan (key outside the cache, window outside int32) or a query has 2^16 frames or more (the
// counts are 16-bit), the caller then takes launch_scan.
// speculative: no host wait for the sort's counts (the sweep's kernels read the kept-frame count
// on the device); ws->spec is then set, and the caller reads ws->info with the results: a batch
// with info[1] > 0 (a frame for the row scan) or info[2] > 0 (a window width outside the sort key's
// delta field) is redone with speculative = false. Without speculation (or when the tolerance's
// window width is unknown) the counts are read back first, as before.
hipError_t launch_scan_wide_prepare(const FrameBox* boxes, const int64_t* d_qoff, int32_t nq, int64_t nf,
                                    int64_t max_qframes, double tole, WideScratch* ws, bool* eligible, hipStream_t s,
                                    bool speculative = false, unsigned long long* d_best_zero = nullptr);
// After prepare: d_best[q] = (count << 32 | tie key) for all nq queries (d_best zeroed on entry).
// d_info_out (optional, device address of host-mapped memory): the clip-major sweep's last kernel
// copies ws->info (3 ints) there; *info_written says whether it did.
// col_base: the index column of the cache's column 0 (an index delta's cache numbers its clips
// from 0; their tie keys are d_tiekey[col_base + column]). Maxima are combined into d_best with
// an atomic max, so a second sweep over another cache adds its clips to the same results.
hipError_t launch_scan_wide(int32_t nq, int64_t nf, const CellCache* cells, const int32_t* d_tiekey, int32_t C,
                            WideScratch* ws, unsigned long long* d_best, hipStream_t s, int32_t* d_info_out = nullptr,
                            bool* info_written = nullptr, int32_t col_base = 0);

}  // namespace tfp
