// tfp_index.hpp — incremental update of the m1-sorted device index (tfp_index.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tfp_kernels.hpp"

namespace tfp {

constexpr int kMergeTile = 4096;  // old index rows per merge_write block

struct MergeScratch {
  int64_t* pos = nullptr;     // [n] insertion point of each new row
  int32_t* kept = nullptr;    // [ntiles + 1] surviving old rows per tile
  int32_t* base = nullptr;    // [ntiles + 1] exclusive scan of kept
  int64_t* jbeg = nullptr;    // [ntiles + 1] first new row whose insertion point is in each tile
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  int64_t cap_pos = 0;
  int32_t cap_tiles = 0;
  hipError_t reserve(int64_t n, int32_t ntiles);
  void release();
  MergeScratch() = default;
  MergeScratch(const MergeScratch&) = delete;
  MergeScratch& operator=(const MergeScratch&) = delete;
  ~MergeScratch() { release(); }
};

// New index = the old rows (m1s, m2s, cols)[0, R) whose remap[col] >= 0, with cols renumbered to
// remap[col], merged with the n new rows (nm1 ascending; nm2, ncol their values, ncol already in
// the new numbering); equal m1 values keep the old rows first. removed = false promises
// remap[col] >= 0 for every old row (no survivor count pass). Output into o1/o2/oc (disjoint from
// the inputs), *kept_old + n rows. Synchronous on s only when removed (to read *kept_old).
// Without removals the column map is a step function: new col = old col + the number of
// breakpoints <= it (one per inserted uuid that sorts before some old one). Up to kMergeBreaks of
// them travel as a kernel argument and replace the per-row remap gather (a random 4-byte read from
// a clip-sized table, half the pass's time at configs[2]); nbrk < 0: use d_remap.
constexpr int kMergeBreaks = 8;
struct MergeBreaks {
  int32_t n;
  int32_t p[kMergeBreaks];
};
hipError_t launch_merge_update(const int32_t* m1s, const int32_t* m2s, const int32_t* cols, int64_t R,
                               const int32_t* d_remap, bool removed, const MergeBreaks& brk, const int32_t* nm1,
                               const int32_t* nm2, const int32_t* ncol, int64_t n, MergeScratch* ms, int32_t* o1,
                               int32_t* o2, int32_t* oc, int64_t* kept_old, hipStream_t s);

// The key-presence bitsets (launch_key_bits: W words per key row, bit c = column c has a row in
// the key's box) carried across such an update instead of rebuilt from every box row:
// key_bits_remap moves every surviving old column's bits (columns < Cm of rows Wo words wide) to
// its new column (d_remap, or the breakpoints when d_remap is null) in dst (rows Wn words wide;
// removed clips' and an index delta's columns dropped), key_bits_add then sets the new rows' bits.
// A new row is in key k's box iff its m1 lies between the first and the last m1 of the box's rows
// in the merged index (d_rng_all at the bitsets' tolerance, recomputed for it): the box is an
// interval and holds the row.
hipError_t launch_key_bits_remap(const uint32_t* src, int32_t Wo, int32_t Cm, const int32_t* d_remap, const MergeBreaks& brk,
                                 uint32_t* dst, int32_t Wn, hipStream_t s);
hipError_t launch_key_bits_add(const int64_t* d_rng_all, const int32_t* m1s, const int32_t* nm1, const int32_t* ncol,
                               int64_t n, int32_t W, uint32_t* bits, hipStream_t s);

// The clip order (tfp_kernels.hpp: okey / om1, R rows) carried through the same update (round 6): the
// old rows' columns renumbered as the index's (remap or brk; removed clips' rows dropped), the
// merge's n new rows (nm1, nm2, ncol, sorted by m1, ncol in the new numbering) sorted into clip
// order alone and inserted. The D new clips: d_newcol (their new columns, ascending) and d_newat
// (each one's insertion point among the old columns: the old columns with a smaller uuid), which
// places a new clip's rows before the old columns at or after it within each key. ms: the index
// merge's scratch, free again once that merge is queued. Output into ok2 / om2, *out_rows rows;
// synchronous on s only when removed.
struct OrderScratch {
  CacheBuf nk, nk2, nv, nv2, tmp;
};
hipError_t launch_order_merge(const unsigned long long* okey, const int32_t* om1, int64_t R, const int32_t* d_remap,
                              bool removed, const MergeBreaks& brk, const int32_t* nm1, const int32_t* nm2,
                              const int32_t* ncol, int64_t n, const int32_t* d_newcol, const int32_t* d_newat, int32_t D,
                              MergeScratch* ms, OrderScratch* os, unsigned long long* ok2, int32_t* om2, int64_t* out_rows,
                              hipStream_t s);

// ---- index delta (round 4) ---------------------------------------------------------------
// The clips enrolled since the last build, searched beside the main index by the coefs = 1 vote
// paths without merging their rows into it (an enrolment then costs its own rows, not a pass over
// the DB). Their columns follow the main index's, from the next multiple of 1024 (the vote GEMM
// breaks ties inside a 1024-column chunk by position, so a chunk must hold main or delta columns
// only, each in uuid order); their key-presence bits are set from their staged rows directly.
struct DeltaClip {
  int64_t off;  // first staged row
  int32_t n;    // staged rows
  int32_t col;  // its column
};
// kbox[2 t], kbox[2 t + 1] = the "%f" box of key t - kKeyOffset at tolerance tole, in micro-units
// (the bounds key_ranges_all_kernel searches the sorted index with).
hipError_t launch_key_boxes(double tole, int64_t* d_kbox, hipStream_t s);
// Sets bit (key, column) for every delta clip and every key whose box (d_kbox) holds one of its
// staged rows' max1 (NULL max1 never does); kspan >= ceil(tole) + 1 bounds the keys a row can be in.
// The delta's columns must be clear (their words hold no main column).
hipError_t launch_delta_bits(const DeltaClip* d_dc, int32_t nd, const int32_t* st_m1, const int64_t* d_kbox, int32_t kspan,
                             int32_t W, uint32_t* bits, hipStream_t s);
// Tie keys without an override: main column c -> c + #{j : at[j] <= c} (its rank among all live
// uuids), delta column col0 + j -> at[j] + j, the columns between -> 0 (they never score).
hipError_t launch_delta_tiekey(const int32_t* d_at, int32_t nd, int32_t main_cols, int32_t col0, int32_t ncols,
                               int32_t* tiekey, hipStream_t s);

}  // namespace tfp
