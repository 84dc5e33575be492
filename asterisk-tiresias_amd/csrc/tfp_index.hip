// tfp_index.hip — incremental maintenance of the m1-sorted device index.
//
// The reference keeps its fingerprint rows in SQLite's audio_fingerprint table with a B-tree on
// max1 (fp_handler.c:745-753); every enrolment's INSERTs (fp_handler.c:559-571) update that
// B-tree row by row, so a new clip is searchable at once for the cost of its own rows. The device
// index is the same B-tree flattened: SoA (m1s, m2s, cols) sorted by m1, col = the clip's rank
// among the live uuids (the tie-break order). An update after enrolments and removals is one
// bandwidth-bound pass over it instead of a re-sort of every staged row:
//
//   * the new rows alone are radix-sorted (their count, not the DB's);
//   * merge_pos: each new row's insertion point among the old rows (after equal m1 values);
//   * merge_count (only when clips were removed): the surviving old rows per tile of 4096,
//     then an exclusive scan over the tiles;
//   * merge_write: every tile copies its surviving old rows to their new places, with the column
//     renumbered through remap (old col -> new col: the uuid ranks shift around inserted and
//     removed clips), and writes the new rows whose insertion point falls inside it.
//
// Traffic per update: 12 B read + 12 B written per index row (+ 4 B read per row when clips were
// removed). At configs[2]'s 93.8 M rows that is ~2.3 GB, ~0.3 ms at the HBM rate, against a
// full 32-bit radix sort of all staged rows plus a host sort of every uuid.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>

#include "tfp_index.hpp"
#include "tfp_kernels.hpp"
#include "tfp_math.hpp"

namespace tfp {
namespace {

constexpr int kThreads = 256;
constexpr int kRowsPerThread = kMergeTile / kThreads;  // 16
constexpr int kPosLds = 2048;  // insertion points of one tile staged in LDS (more: searched in memory)

__device__ __forceinline__ int64_t upper_bound_m1(const int32_t* a, int64_t n, int32_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t lower_bound_pos(const int64_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// pos[j] = number of old rows with m1 <= nm1[j]: new row j goes after every equal old row.
// nm1 is sorted, so pos is non-decreasing.
__global__ void merge_pos_kernel(const int32_t* __restrict__ m1s, int64_t R, const int32_t* __restrict__ nm1, int64_t n,
                                 int64_t* __restrict__ pos) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
    pos[j] = upper_bound_m1(m1s, R, nm1[j]);
}

// jbeg[t] = the first new row whose insertion point is >= t * 4096 (t = 0..ntiles): each tile's new
// rows are [jbeg[t], jbeg[t + 1]). Searched once per tile here, so merge_write starts with two
// loads instead of a chain of dependent ones.
__global__ void merge_tiles_kernel(const int64_t* __restrict__ pos, int64_t n, int32_t ntiles, int64_t* __restrict__ jbeg) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t <= ntiles; t += (int64_t)gridDim.x * blockDim.x)
    jbeg[t] = lower_bound_pos(pos, n, t * kMergeTile);
}

// kept[t] = old rows of tile t whose clip survives (remap[col] >= 0); kept[ntiles] = 0 (the scan's
// total lands in base[ntiles]).
__global__ __launch_bounds__(kThreads) void merge_count_kernel(const int32_t* __restrict__ cols, int64_t R,
                                                               const int32_t* __restrict__ remap, int32_t ntiles,
                                                               int32_t* __restrict__ kept) {
  __shared__ int32_t wsum[kThreads / 64];
  const int64_t b0 = (int64_t)blockIdx.x * kMergeTile;
  int32_t c = 0;
  if (blockIdx.x < (unsigned)ntiles) {
    for (int k = 0; k < kRowsPerThread; k++) {
      const int64_t i = b0 + k * kThreads + threadIdx.x;
      if (i < R) c += remap[cols[i]] >= 0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t t = 0;
    for (int w = 0; w < kThreads / 64; w++) t += wsum[w];
    kept[blockIdx.x] = t;
  }
}

// One tile of old rows [b0, b0 + 4096) and the new rows inserted at points in [b0, b0 + 4096).
// base[t]: surviving old rows before tile t (nullptr: nothing removed, base = b0).
__global__ __launch_bounds__(kThreads) void merge_write_kernel(
    const int32_t* __restrict__ m1s, const int32_t* __restrict__ m2s, const int32_t* __restrict__ cols, int64_t R,
    const int32_t* __restrict__ remap, MergeBreaks brk, const int32_t* __restrict__ base, const int32_t* __restrict__ nm1,
    const int32_t* __restrict__ nm2, const int32_t* __restrict__ ncol, const int64_t* __restrict__ pos,
    const int64_t* __restrict__ jbeg, int32_t* __restrict__ o1, int32_t* __restrict__ o2, int32_t* __restrict__ oc) {
  __shared__ int32_t pref[kMergeTile + 1];          // surviving rows of the tile before each row
  __shared__ int32_t lpos[kPosLds];                 // the tile's insertion points, relative to b0
  __shared__ int32_t csum[kRowsPerThread][kThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * kMergeTile;
  const int64_t j0 = jbeg[blockIdx.x], j1 = jbeg[blockIdx.x + 1], nj = j1 - j0;
  // the tile's rows, coalesced: row b0 + k * 256 + t. Every load is issued before the first
  // remap gather (indices clamped to the last row, no branches: a branch per row made each row's
  // gather wait for its column load, 16 round trips per tile).
  int32_t r1[kRowsPerThread], r2[kRowsPerThread], rc[kRowsPerThread];
  uint32_t keep = 0;
  if (R > 0) {
#pragma unroll
    for (int k = 0; k < kRowsPerThread; k++) {
      const int64_t i = min(b0 + k * kThreads + t, R - 1);
      r1[k] = m1s[i];
      r2[k] = m2s[i];
      rc[k] = cols[i];
    }
    if (brk.n >= 0) {  // no removals: the step function of the breakpoints (kernel arguments)
#pragma unroll
      for (int k = 0; k < kRowsPerThread; k++) {
        int32_t d = 0;
        for (int j = 0; j < brk.n; j++) d += rc[k] >= brk.p[j];
        rc[k] += d;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kRowsPerThread; k++) rc[k] = remap[rc[k]];
    }
#pragma unroll
    for (int k = 0; k < kRowsPerThread; k++) keep |= (uint32_t)(b0 + k * kThreads + t < R && rc[k] >= 0) << k;
  }
  // Nothing removed (base == nullptr, every old row survives): a row's place in the tile is its own
  // index, and the tile needs no prefix (an enrolment's update: a plain streaming copy).
  const bool all_kept = base == nullptr;
  uint32_t lo[kRowsPerThread];
  if (!all_kept) {
    // in-tile exclusive prefix of the surviving rows, in row order (chunk k, then wave, then lane)
#pragma unroll
    for (int k = 0; k < kRowsPerThread; k++) {
      const uint64_t m = __ballot((keep >> k) & 1u);
      lo[k] = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (lane == 0) csum[k][wv] = __popcll(m);
    }
  }
  __syncthreads();
  if (!all_kept && t == 0) {  // 64 partial sums, in row order
    int32_t run = 0;
    for (int k = 0; k < kRowsPerThread; k++)
      for (int w = 0; w < kThreads / 64; w++) {
        const int32_t v = csum[k][w];
        csum[k][w] = run;
        run += v;
      }
    pref[kMergeTile] = run;
  }
  __syncthreads();
  const bool in_lds = nj <= kPosLds;
  if (in_lds)
    for (int64_t j = t; j < nj; j += kThreads) lpos[j] = (int32_t)(pos[j0 + j] - b0);
  if (!all_kept)
#pragma unroll
    for (int k = 0; k < kRowsPerThread; k++) pref[k * kThreads + t] = csum[k][wv] + (int32_t)lo[k];
  __syncthreads();
  auto place = [&](int32_t r) -> int32_t { return all_kept ? r : pref[r]; };
  const int64_t bb = base ? (int64_t)base[blockIdx.x] : b0;
#pragma unroll
  for (int k = 0; k < kRowsPerThread; k++) {
    if (!((keep >> k) & 1u)) continue;
    const int32_t r = k * kThreads + t;
    // new rows placed before old row b0 + r: those with insertion point <= b0 + r
    int64_t before = j0;
    if (nj) {
      int64_t a = 0, h = nj;
      while (a < h) {
        const int64_t mid = (a + h) >> 1;
        const int64_t p = in_lds ? (int64_t)lpos[mid] : pos[j0 + mid] - b0;
        if (p <= r) a = mid + 1; else h = mid;
      }
      before += a;
    }
    const int64_t o = bb + place(r) + before;
    o1[o] = r1[k];
    o2[o] = r2[k];
    oc[o] = rc[k];
  }
  for (int64_t j = t; j < nj; j += kThreads) {
    const int64_t p = in_lds ? (int64_t)lpos[j] : pos[j0 + j] - b0;  // in [0, 4096]
    const int64_t o = bb + place((int32_t)p) + j0 + j;
    o1[o] = nm1[j0 + j];
    o2[o] = nm2[j0 + j];
    oc[o] = ncol[j0 + j];
  }
}

// One word of a key row with a zero bit inserted at column p (words below p's unchanged).
// The bitsets through a column renumbering (one thread per old row word): old column c < Cm moves to
// remap[c] (-1: removed) or, without a table, to c plus the breakpoints <= c; columns >= Cm (an index
// delta's, whose clips are among the merge's new rows) are dropped. The columns keep their order, so
// a word's bits land in a few new words, each ORed in once; dst (Wn words per row) is zero on entry.
__global__ void key_bits_remap_kernel(const uint32_t* __restrict__ src, int32_t Wo, int32_t Cm, const int32_t* __restrict__ remap,
                                      MergeBreaks brk, uint32_t* __restrict__ dst, int32_t Wn) {
  const int64_t n = (int64_t)kKeyRange * Wo;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t w = (int32_t)(i % Wo);
    const int64_t k = i / Wo;
    if (32 * w >= Cm) continue;
    uint32_t x = src[i];
    if (32 * w + 32 > Cm) x &= (1u << (Cm - 32 * w)) - 1u;
    uint32_t acc = 0;
    int32_t aw = -1;
    while (x) {
      const int b = __ffs(x) - 1;
      x &= x - 1;
      const int32_t c = 32 * w + b;
      int32_t nc = c;
      if (remap) {
        nc = remap[c];
      } else {
        for (int j = 0; j < brk.n; j++) nc += c >= brk.p[j];
      }
      if (nc < 0) continue;
      if ((nc >> 5) != aw) {
        if (aw >= 0) atomicOr(&dst[k * Wn + aw], acc);
        aw = nc >> 5;
        acc = 0;
      }
      acc |= 1u << (nc & 31);
    }
    if (aw >= 0) atomicOr(&dst[k * Wn + aw], acc);
  }
}

// Per key: the new rows (sorted by m1) whose m1 lies in [m1 of the box's first row, m1 of its last].
__global__ __launch_bounds__(64) void key_bits_add_kernel(const int64_t* __restrict__ rng_all, const int32_t* __restrict__ m1s,
                                                          const int32_t* __restrict__ nm1, const int32_t* __restrict__ ncol,
                                                          int64_t n, int32_t W, uint32_t* __restrict__ bits) {
  const int key = blockIdx.x;
  const int64_t lo = rng_all[2 * key], hi = rng_all[2 * key + 1];
  if (lo >= hi || n <= 0) return;
  const int32_t vmin = m1s[lo], vmax = m1s[hi - 1];
  int64_t a = 0, b = n;  // first new row with m1 >= vmin
  while (a < b) {
    const int64_t mid = (a + b) >> 1;
    if (nm1[mid] < vmin) a = mid + 1; else b = mid;
  }
  uint32_t* row = bits + (int64_t)key * W;
  for (int64_t j = a + threadIdx.x; j < n && nm1[j] <= vmax; j += blockDim.x) {
    const int32_t c = ncol[j];
    atomicOr(&row[c >> 5], 1u << (c & 31));
  }
}


// ---- the clip order through an update (round 6) ----------------------------------------------

constexpr uint32_t kOColMask = (1u << 21) - 1u;

__device__ __forceinline__ int32_t new_at(const int32_t* __restrict__ newcol, const int32_t* __restrict__ newat, int32_t D,
                                          int32_t col) {
  int32_t lo = 0, hi = D;  // the new clip with this column
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (newcol[mid] < col) lo = mid + 1; else hi = mid;
  }
  return newat[lo < D ? lo : D - 1];
}

// The new rows' clip-order keys (t << 53 | new column << 32 | m2 bits) and m1 (the nearest-integer
// key index as tfp_scan.hip's order_key_index).
__global__ void order_new_keys_kernel(const int32_t* __restrict__ nm1, const int32_t* __restrict__ nm2,
                                      const int32_t* __restrict__ ncol, int64_t n, unsigned long long* __restrict__ nk,
                                      int32_t* __restrict__ nv) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t m1 = nm1[i];
    const int64_t v = (int64_t)m1 + 500000;
    int64_t t = (v >= 0 ? v : v - 999999) / 1000000 + kKeyOffset;
    t = t < 0 ? 0 : t >= kKeyRange ? kKeyRange - 1 : t;
    nk[i] = ((unsigned long long)t << 53) | ((unsigned long long)(uint32_t)ncol[i] << 32) | (uint32_t)(nm2[i] ^ INT32_MIN);
    nv[i] = m1;
  }
}

// pos[j] = old rows before new row j: those of a smaller key index, or of the same one and an old
// column below the new clip's insertion point (no old row shares a new row's column).
__global__ void order_pos_kernel(const unsigned long long* __restrict__ okey, int64_t R, const unsigned long long* __restrict__ nk,
                                 int64_t n, const int32_t* __restrict__ newcol, const int32_t* __restrict__ newat, int32_t D,
                                 int64_t* __restrict__ pos) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long k = nk[j];
    const int32_t at = new_at(newcol, newat, D, (int32_t)((k >> 32) & kOColMask));
    const unsigned long long v = ((k >> 53) << 53) | ((unsigned long long)(uint32_t)at << 32);
    int64_t lo = 0, hi = R;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (okey[mid] < v) lo = mid + 1; else hi = mid;
    }
    pos[j] = lo;
  }
}

// kept[t] = old order rows of tile t whose clip survives.
__global__ __launch_bounds__(kThreads) void order_count_kept_kernel(const unsigned long long* __restrict__ okey, int64_t R,
                                                                    const int32_t* __restrict__ remap, int32_t ntiles,
                                                                    int32_t* __restrict__ kept) {
  __shared__ int32_t wsum[kThreads / 64];
  const int64_t b0 = (int64_t)blockIdx.x * kMergeTile;
  int32_t c = 0;
  if (blockIdx.x < (unsigned)ntiles) {
    for (int k = 0; k < kRowsPerThread; k++) {
      const int64_t i = b0 + k * kThreads + threadIdx.x;
      if (i < R) c += remap[(okey[i] >> 32) & kOColMask] >= 0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t t = 0;
    for (int w = 0; w < kThreads / 64; w++) t += wsum[w];
    kept[blockIdx.x] = t;
  }
}

// merge_write_kernel's tile, for the clip order's (key, m1) rows.
__global__ __launch_bounds__(kThreads) void order_write_kernel(
    const unsigned long long* __restrict__ okey, const int32_t* __restrict__ om1, int64_t R, const int32_t* __restrict__ remap,
    MergeBreaks brk, const int32_t* __restrict__ base, const unsigned long long* __restrict__ nk,
    const int32_t* __restrict__ nv, const int64_t* __restrict__ pos, const int64_t* __restrict__ jbeg,
    unsigned long long* __restrict__ ok2, int32_t* __restrict__ om2) {
  __shared__ int32_t pref[kMergeTile + 1];
  __shared__ int32_t lpos[kPosLds];
  __shared__ int32_t csum[kRowsPerThread][kThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * kMergeTile;
  const int64_t j0 = jbeg[blockIdx.x], j1 = jbeg[blockIdx.x + 1], nj = j1 - j0;
  unsigned long long rk[kRowsPerThread];
  int32_t r1[kRowsPerThread];
  uint32_t keep = 0;
  if (R > 0) {
#pragma unroll
    for (int k = 0; k < kRowsPerThread; k++) {
      const int64_t i = min(b0 + k * kThreads + t, R - 1);
      rk[k] = okey[i];
      r1[k] = om1[i];
    }
#pragma unroll
    for (int k = 0; k < kRowsPerThread; k++) {
      const int32_t c = (int32_t)((rk[k] >> 32) & kOColMask);
      int32_t nc = c;
      if (brk.n >= 0) {
        for (int j = 0; j < brk.n; j++) nc += c >= brk.p[j];
      } else {
        nc = remap[c];
      }
      keep |= (uint32_t)(b0 + k * kThreads + t < R && nc >= 0) << k;
      rk[k] = (rk[k] & ~((unsigned long long)kOColMask << 32)) | ((unsigned long long)(uint32_t)(nc < 0 ? 0 : nc) << 32);
    }
  }
  const bool all_kept = base == nullptr;
  uint32_t lo[kRowsPerThread];
  if (!all_kept) {
#pragma unroll
    for (int k = 0; k < kRowsPerThread; k++) {
      const uint64_t m = __ballot((keep >> k) & 1u);
      lo[k] = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (lane == 0) csum[k][wv] = __popcll(m);
    }
  }
  __syncthreads();
  if (!all_kept && t == 0) {
    int32_t run = 0;
    for (int k = 0; k < kRowsPerThread; k++)
      for (int w = 0; w < kThreads / 64; w++) {
        const int32_t v = csum[k][w];
        csum[k][w] = run;
        run += v;
      }
    pref[kMergeTile] = run;
  }
  __syncthreads();
  const bool in_lds = nj <= kPosLds;
  if (in_lds)
    for (int64_t j = t; j < nj; j += kThreads) lpos[j] = (int32_t)(pos[j0 + j] - b0);
  if (!all_kept)
#pragma unroll
    for (int k = 0; k < kRowsPerThread; k++) pref[k * kThreads + t] = csum[k][wv] + (int32_t)lo[k];
  __syncthreads();
  auto place = [&](int32_t r) -> int32_t { return all_kept ? r : pref[r]; };
  const int64_t bb = base ? (int64_t)base[blockIdx.x] : b0;
#pragma unroll
  for (int k = 0; k < kRowsPerThread; k++) {
    if (!((keep >> k) & 1u)) continue;
    const int32_t r = k * kThreads + t;
    int64_t before = j0;  // new rows placed before old row b0 + r: insertion point <= b0 + r
    if (nj) {
      int64_t a = 0, h = nj;
      while (a < h) {
        const int64_t mid = (a + h) >> 1;
        const int64_t p = in_lds ? (int64_t)lpos[mid] : pos[j0 + mid] - b0;
        if (p <= r) a = mid + 1; else h = mid;
      }
      before += a;
    }
    const int64_t o = bb + place(r) + before;
    ok2[o] = rk[k];
    om2[o] = r1[k];
  }
  for (int64_t j = t; j < nj; j += kThreads) {
    const int64_t p = in_lds ? (int64_t)lpos[j] : pos[j0 + j] - b0;
    const int64_t o = bb + place((int32_t)p) + j0 + j;
    ok2[o] = nk[j0 + j];
    om2[o] = nv[j0 + j];
  }
}

}  // namespace

hipError_t launch_key_bits_remap(const uint32_t* src, int32_t Wo, int32_t Cm, const int32_t* d_remap, const MergeBreaks& brk,
                                 uint32_t* dst, int32_t Wn, hipStream_t s) {
  hipError_t e = hipMemsetAsync(dst, 0, sizeof(uint32_t) * (size_t)kKeyRange * Wn, s);
  if (e) return e;
  const int64_t n = (int64_t)kKeyRange * Wo;
  hipLaunchKernelGGL(key_bits_remap_kernel, dim3((unsigned)std::min<int64_t>(8192, (n + 255) / 256)), dim3(256), 0, s, src,
                     Wo, Cm, d_remap, brk, dst, Wn);
  return hipGetLastError();
}

hipError_t launch_key_bits_add(const int64_t* d_rng_all, const int32_t* m1s, const int32_t* nm1, const int32_t* ncol,
                               int64_t n, int32_t W, uint32_t* bits, hipStream_t s) {
  hipLaunchKernelGGL(key_bits_add_kernel, dim3(kKeyRange), dim3(64), 0, s, d_rng_all, m1s, nm1, ncol, n, W, bits);
  return hipGetLastError();
}

hipError_t launch_merge_update(const int32_t* m1s, const int32_t* m2s, const int32_t* cols, int64_t R,
                               const int32_t* d_remap, bool removed, const MergeBreaks& brk, const int32_t* nm1,
                               const int32_t* nm2, const int32_t* ncol, int64_t n, MergeScratch* ms, int32_t* o1,
                               int32_t* o2, int32_t* oc, int64_t* kept_old, hipStream_t s) {
  // tiles: floor(R / 4096) + 1, so the insertion points 0..R all fall in some tile
  const int64_t ntiles = R / kMergeTile + 1;
  if (ntiles >= INT32_MAX / 2) return hipErrorInvalidValue;
  hipError_t e;
  if ((e = ms->reserve(n, (int32_t)ntiles)) != hipSuccess) return e;
  if (n > 0) {
    const unsigned g = (unsigned)std::min<int64_t>(2048, (n + 255) / 256);
    hipLaunchKernelGGL(merge_pos_kernel, dim3(g), dim3(256), 0, s, m1s, R, nm1, n, ms->pos);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(merge_tiles_kernel, dim3((unsigned)std::min<int64_t>(1024, (ntiles + 256) / 256)), dim3(256), 0, s,
                     ms->pos, n, (int32_t)ntiles, ms->jbeg);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int32_t* d_base = nullptr;
  *kept_old = R;
  if (removed) {
    hipLaunchKernelGGL(merge_count_kernel, dim3((unsigned)ntiles + 1), dim3(kThreads), 0, s, cols, R, d_remap,
                       (int32_t)ntiles, ms->kept);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tb = ms->tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(ms->tmp, tb, ms->kept, ms->base, (int)ntiles + 1, s)) != hipSuccess)
      return e;
    int32_t total = 0;
    if ((e = hipMemcpyAsync(&total, ms->base + ntiles, sizeof total, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    *kept_old = total;
    d_base = ms->base;
  }
  MergeBreaks kb = brk;
  if (removed) kb.n = -1;
  hipLaunchKernelGGL(merge_write_kernel, dim3((unsigned)ntiles), dim3(kThreads), 0, s, m1s, m2s, cols, R, d_remap, kb,
                     d_base, nm1, nm2, ncol, ms->pos, ms->jbeg, o1, o2, oc);
  return hipGetLastError();
}

hipError_t launch_order_merge(const unsigned long long* okey, const int32_t* om1, int64_t R, const int32_t* d_remap,
                              bool removed, const MergeBreaks& brk, const int32_t* nm1, const int32_t* nm2,
                              const int32_t* ncol, int64_t n, const int32_t* d_newcol, const int32_t* d_newat, int32_t D,
                              MergeScratch* ms, OrderScratch* os, unsigned long long* ok2, int32_t* om2, int64_t* out_rows,
                              hipStream_t s) {
  const int64_t ntiles = R / kMergeTile + 1;
  if (ntiles >= INT32_MAX / 2 || n >= INT32_MAX || (n > 0 && D <= 0)) return hipErrorInvalidValue;
  hipError_t e;
  if ((e = ms->reserve(n, (int32_t)ntiles)) != hipSuccess) return e;
  const unsigned long long* nk = nullptr;
  const int32_t* nv = nullptr;
  if (n > 0) {
    // the new rows in clip order: keys, then a radix sort of those rows alone (their count, not the DB's)
    if ((e = os->nk.reserve(sizeof(unsigned long long) * n)) != hipSuccess || (e = os->nk2.reserve(sizeof(unsigned long long) * n)) != hipSuccess ||
        (e = os->nv.reserve(sizeof(int32_t) * n)) != hipSuccess || (e = os->nv2.reserve(sizeof(int32_t) * n)) != hipSuccess)
      return e;
    const unsigned g = (unsigned)std::min<int64_t>(2048, (n + 255) / 256);
    hipLaunchKernelGGL(order_new_keys_kernel, dim3(g), dim3(256), 0, s, nm1, nm2, ncol, n, os->nk.as<unsigned long long>(),
                       os->nv.as<int32_t>());
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tb = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, os->nk.as<unsigned long long>(), os->nk2.as<unsigned long long>(),
                                                os->nv.as<int32_t>(), os->nv2.as<int32_t>(), (int)n, 0, 63, s)) != hipSuccess ||
        (e = os->tmp.reserve(tb)) != hipSuccess)
      return e;
    tb = os->tmp.bytes;
    if ((e = hipcub::DeviceRadixSort::SortPairs(os->tmp.p, tb, os->nk.as<unsigned long long>(), os->nk2.as<unsigned long long>(),
                                                os->nv.as<int32_t>(), os->nv2.as<int32_t>(), (int)n, 0, 63, s)) != hipSuccess)
      return e;
    nk = os->nk2.as<unsigned long long>();
    nv = os->nv2.as<int32_t>();
    hipLaunchKernelGGL(order_pos_kernel, dim3(g), dim3(256), 0, s, okey, R, nk, n, d_newcol, d_newat, D, ms->pos);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(merge_tiles_kernel, dim3((unsigned)std::min<int64_t>(1024, (ntiles + 256) / 256)), dim3(256), 0, s,
                     ms->pos, n, (int32_t)ntiles, ms->jbeg);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int32_t* d_base = nullptr;
  int64_t kept = R;
  if (removed) {
    hipLaunchKernelGGL(order_count_kept_kernel, dim3((unsigned)ntiles + 1), dim3(kThreads), 0, s, okey, R, d_remap,
                       (int32_t)ntiles, ms->kept);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tb = ms->tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(ms->tmp, tb, ms->kept, ms->base, (int)ntiles + 1, s)) != hipSuccess) return e;
    int32_t total = 0;
    if ((e = hipMemcpyAsync(&total, ms->base + ntiles, sizeof total, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    kept = total;
    d_base = ms->base;
  }
  MergeBreaks kb = brk;
  if (removed) kb.n = -1;
  hipLaunchKernelGGL(order_write_kernel, dim3((unsigned)ntiles), dim3(kThreads), 0, s, okey, om1, R, d_remap, kb, d_base, nk,
                     nv, ms->pos, ms->jbeg, ok2, om2);
  *out_rows = kept + n;
  return hipGetLastError();
}

hipError_t MergeScratch::reserve(int64_t n, int32_t ntiles) {
  hipError_t e;
  if (n + 1 > cap_pos) {
    if (pos) (void)hipFree(pos);
    pos = nullptr;
    cap_pos = 0;
    if ((e = hipMalloc(&pos, sizeof(int64_t) * (n + 1))) != hipSuccess) return e;
    cap_pos = n + 1;
  }
  if (ntiles + 1 > cap_tiles) {
    for (void* p : {(void*)kept, (void*)base, (void*)jbeg, tmp})
      if (p) (void)hipFree(p);
    kept = base = nullptr;
    jbeg = nullptr;
    tmp = nullptr;
    cap_tiles = 0;
    tmp_bytes = 0;
    const int32_t cap = ntiles + 1 + ntiles / 4;  // room to grow
    if ((e = hipMalloc(&kept, sizeof(int32_t) * cap)) != hipSuccess) return e;
    if ((e = hipMalloc(&base, sizeof(int32_t) * cap)) != hipSuccess) return e;
    if ((e = hipMalloc(&jbeg, sizeof(int64_t) * cap)) != hipSuccess) return e;
    size_t tb = 0;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, kept, base, cap, (hipStream_t)0)) != hipSuccess) return e;
    if ((e = hipMalloc(&tmp, tb > 0 ? tb : 1)) != hipSuccess) return e;
    tmp_bytes = tb;
    cap_tiles = cap;
  }
  return hipSuccess;
}

void MergeScratch::release() {
  for (void* p : {(void*)pos, (void*)kept, (void*)base, (void*)jbeg, tmp})
    if (p) (void)hipFree(p);
  pos = nullptr;
  kept = base = nullptr;
  jbeg = nullptr;
  tmp = nullptr;
  cap_pos = 0;
  cap_tiles = 0;
  tmp_bytes = 0;
}

// ---- index delta --------------------------------------------------------------------------

namespace {

__global__ void key_boxes_kernel(double tole, int64_t* __restrict__ kbox) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kKeyRange) return;
  const double freq = (double)(t - kKeyOffset);
  kbox[2 * t] = fmt6_bound(freq - tole);
  kbox[2 * t + 1] = fmt6_bound(freq + tole);
}

// One block per delta clip: its rows' keys as LDS flags, then one atomicOr per (key, clip).
__global__ __launch_bounds__(256) void delta_bits_kernel(const DeltaClip* __restrict__ dc, const int32_t* __restrict__ st_m1,
                                                         const int64_t* __restrict__ kbox, int32_t kspan, int32_t W,
                                                         uint32_t* __restrict__ bits) {
  __shared__ uint32_t flags[kKeyRange / 32];
  const DeltaClip d = dc[blockIdx.x];
  for (int i = threadIdx.x; i < kKeyRange / 32; i += blockDim.x) flags[i] = 0u;
  __syncthreads();
  for (int32_t r = threadIdx.x; r < d.n; r += blockDim.x) {
    const int32_t m1 = st_m1[d.off + r];
    if (m1 == INT32_MIN) continue;  // NULL max1: never in a box
    const int64_t kc = (m1 >= 0 ? (int64_t)m1 : (int64_t)m1 - 999999) / 1000000;  // floor(m1 / 10^6)
    for (int64_t k = kc - kspan; k <= kc + kspan; k++) {
      const int64_t t = k + kKeyOffset;
      if (t < 0 || t >= kKeyRange) continue;
      if ((int64_t)m1 >= kbox[2 * t] && (int64_t)m1 <= kbox[2 * t + 1]) atomicOr(&flags[t >> 5], 1u << (t & 31));
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < kKeyRange; t += blockDim.x)
    if ((flags[t >> 5] >> (t & 31)) & 1u) atomicOr(&bits[(int64_t)t * W + (d.col >> 5)], 1u << (d.col & 31));
}

__global__ void delta_tiekey_kernel(const int32_t* __restrict__ at, int32_t nd, int32_t main_cols, int32_t col0, int32_t ncols,
                                    int32_t* __restrict__ tiekey) {
  for (int32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < ncols; c += gridDim.x * blockDim.x) {
    int32_t v = 0;
    if (c < main_cols) {
      int32_t lo = 0, hi = nd;  // #{j : at[j] <= c} (at ascending)
      while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (at[mid] <= c) lo = mid + 1; else hi = mid;
      }
      v = c + lo;
    } else if (c >= col0 && c - col0 < nd) {
      v = at[c - col0] + (c - col0);
    }
    tiekey[c] = v;
  }
}

}  // namespace

hipError_t launch_key_boxes(double tole, int64_t* d_kbox, hipStream_t s) {
  hipLaunchKernelGGL(key_boxes_kernel, dim3(kKeyRange / 64), dim3(64), 0, s, tole, d_kbox);
  return hipGetLastError();
}

hipError_t launch_delta_bits(const DeltaClip* d_dc, int32_t nd, const int32_t* st_m1, const int64_t* d_kbox, int32_t kspan,
                             int32_t W, uint32_t* bits, hipStream_t s) {
  if (nd <= 0) return hipSuccess;
  hipLaunchKernelGGL(delta_bits_kernel, dim3((unsigned)nd), dim3(256), 0, s, d_dc, st_m1, d_kbox, kspan, W, bits);
  return hipGetLastError();
}

hipError_t launch_delta_tiekey(const int32_t* d_at, int32_t nd, int32_t main_cols, int32_t col0, int32_t ncols,
                               int32_t* tiekey, hipStream_t s) {
  if (ncols <= 0) return hipSuccess;
  hipLaunchKernelGGL(delta_tiekey_kernel, dim3((unsigned)std::min<int64_t>(1024, (ncols + 255) / 256)), dim3(256), 0, s, d_at,
                     nd, main_cols, col0, ncols, tiekey);
  return hipGetLastError();
}

}  // namespace tfp
