// tfp_index.hpp — incremental update of the m1-sorted device index (tfp_index.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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
// key_bits_insert copies src to dst with a zero bit inserted at column p of every row (the
// breakpoints, highest first), key_bits_add then sets the new rows' bits. A new row is in key k's
// box iff its m1 lies between the first and the last m1 of the box's rows in the merged index
// (d_rng_all at the bitsets' tolerance, recomputed for it): the box is an interval and holds the row.
hipError_t launch_key_bits_insert(const uint32_t* src, uint32_t* dst, int32_t W, int32_t p, hipStream_t s);
hipError_t launch_key_bits_add(const int64_t* d_rng_all, const int32_t* m1s, const int32_t* nm1, const int32_t* ncol,
                               int64_t n, int32_t W, uint32_t* bits, hipStream_t s);

}  // namespace tfp
