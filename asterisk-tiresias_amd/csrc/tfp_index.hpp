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
hipError_t launch_merge_update(const int32_t* m1s, const int32_t* m2s, const int32_t* cols, int64_t R,
                               const int32_t* d_remap, bool removed, const int32_t* nm1, const int32_t* nm2,
                               const int32_t* ncol, int64_t n, MergeScratch* ms, int32_t* o1, int32_t* o2, int32_t* oc,
                               int64_t* kept_old, hipStream_t s);

}  // namespace tfp
