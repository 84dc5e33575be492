// tfp_scan.hip — the search's general path on gfx950: every query frame's SQL of
// fp_search_fingerprint_info (src/fp_handler.c:308-359), for coefs = 2 (max1 AND max2 windows)
// and for the coefs = 1 batches the vote path hands back (counts beyond fp16, keys out of range).
//
// The per-frame statement inserts one row per clip that has a row in the frame's box
// (GROUP BY audio_uuid), so a frame's contribution is the SET of clips it hits. Enumerating the
// box's rows costs rows-per-clip times more than that set (a clip's frames cluster: ~50 rows per
// clip inside a 0.01 dB window at configs[2]), so the general path works on clip sets instead:
//
//   groups   per (trunc key k, clip) the clip's max2 values inside key k's max1 box
//            [fmt6(k - tol), fmt6(k + tol)], ascending (the "points" of the group);
//   cells    the max2 axis cut into cells of width w >= the widest max2 window at this
//            tolerance; entry (k, j, clip) exists iff the clip has a point in cells j or j + 1.
//
// A coefs = 2 frame with window [L2, U2] (U2 - L2 <= w) lies inside cells j(L2) and j(L2) + 1,
// so its candidates are the entries (k, j(L2), *): one per clip, each confirmed by a binary search
// in the clip's points. A frame without a max2 condition hits every group of its key. Each hit
// is a distinct clip, so frames need no per-frame dedup and run in parallel (one wave each);
// counts go to a per-query score row with atomics, and a clip's first count appends it to the
// query's touched list. Frames whose key lies outside the cache (never produced by real audio:
// |10 log10 c| <= 449 for every float c) take the row scan with per-frame stamps, one wave per
// query, frames in order. A last pass reduces (count << 32 | tie key) over each query's touched
// clips — count(*) DESC, ties to the greatest audio_uuid (:367) — and restores the scratch to 0.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "tfp_kernels.hpp"
#include "tfp_index.hpp"
#include "tfp_bsearch.hpp"
#include "tfp_math.hpp"

namespace tfp {

namespace {

constexpr int kColBits = 21;  // clip column bits in the packed keys (CellCache::kMaxCols)
constexpr uint32_t kColMask = (1u << kColBits) - 1u;

template <class T>
__device__ __forceinline__ int64_t lower_bound_t(const T* a, int64_t n, T v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t lb_i32(const int32_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int64_t ub_i32(const int32_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)a[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t cell_of(int64_t v, int64_t w) { return (v - (int64_t)INT32_MIN) / w; }

// ---- cache build --------------------------------------------------------------------------

// Every row of every key's max1 box (rng_all at this tolerance) as k << 53 | col << 32 | m2 bits.
__global__ void cells_fill_kernel(const int64_t* __restrict__ rng_all, const int64_t* __restrict__ off,
                                  const int32_t* __restrict__ m2s, const int32_t* __restrict__ cols, int64_t S,
                                  unsigned long long* __restrict__ keys) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S; i += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = kKeyRange;  // the last key whose rows start at or before i (empty boxes skipped)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (off[mid] <= i) lo = mid; else hi = mid;
    }
    const int64_t r = rng_all[2 * lo] + (i - off[lo]);
    keys[i] = ((unsigned long long)lo << 53) | ((unsigned long long)(uint32_t)cols[r] << 32) |
              (uint32_t)(m2s[r] ^ INT32_MIN);  // unsigned order of the low word == signed m2 order
  }
}

__global__ void cells_split_kernel(const unsigned long long* __restrict__ keys, int64_t S, int32_t* __restrict__ p_m2,
                                   uint32_t* __restrict__ k32) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long k = keys[i];
    p_m2[i] = (int32_t)((uint32_t)k ^ 0x80000000u);
    k32[i] = (uint32_t)(k >> 32);  // k << 21 | col
  }
}

// Two cell entries per point: its own cell j and j - 1 (so entry (k, j) covers cells j, j + 1).
__global__ void cells_entries_kernel(const int32_t* __restrict__ p_m2, const uint32_t* __restrict__ k32, int64_t S,
                                     const uint32_t* __restrict__ g_key, int64_t n1, int64_t w,
                                     unsigned long long* __restrict__ e_key, int32_t* __restrict__ e_grp) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t kc = k32[i];
    const int32_t g = (int32_t)lower_bound_t<uint32_t>(g_key, n1, kc);
    const unsigned long long key = (unsigned long long)(kc >> kColBits), col = kc & kColMask;
    const unsigned long long j = (unsigned long long)cell_of(p_m2[i], w);
    e_key[2 * i] = (key << 52) | (j << kColBits) | col;
    e_key[2 * i + 1] = (key << 52) | ((j ? j - 1 : j) << kColBits) | col;
    e_grp[2 * i] = g;
    e_grp[2 * i + 1] = g;
  }
}

// First group of every key (groups are sorted by key << 21 | column).
__global__ void key_gbeg_kernel(const uint32_t* __restrict__ g_key, int64_t n1, int32_t* __restrict__ k_gbeg) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t <= kKeyRange) k_gbeg[t] = (int32_t)lower_bound_t<uint32_t>(g_key, n1, (uint32_t)t << kColBits);
}

// Clusters of each group's points (CellCache::c_lo/c_hi/c_beg): point i starts one when it starts
// its group or lies more than dgap above its predecessor.
__global__ void cluster_flag_kernel(const int32_t* __restrict__ p_m2, const uint32_t* __restrict__ k32, int64_t S,
                                    int64_t dgap, int32_t* __restrict__ flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S; i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = i == 0 || k32[i] != k32[i - 1] || (int64_t)p_m2[i] - (int64_t)p_m2[i - 1] > dgap;
}
// cidx = exclusive prefix of the flags: point i is in cluster cidx[i] + flag[i] - 1.
__global__ void cluster_write_kernel(const int32_t* __restrict__ p_m2, const int32_t* __restrict__ flag,
                                     const int32_t* __restrict__ cidx, int64_t S, int32_t* __restrict__ c_lo,
                                     int32_t* __restrict__ c_hi) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = cidx[i] + flag[i] - 1;
    if (flag[i]) c_lo[c] = p_m2[i];
    if (i == S - 1 || flag[i + 1]) c_hi[c] = p_m2[i];
  }
}
// c_beg[g] = the cluster of group g's first point (a cluster start), c_beg[n1] = nc.
__global__ void cluster_gbeg_kernel(const int32_t* __restrict__ g_beg, const int32_t* __restrict__ cidx, int64_t n1,
                                    int64_t S, int64_t nc, int32_t* __restrict__ c_beg) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= n1; g += (int64_t)gridDim.x * blockDim.x)
    c_beg[g] = g < n1 && g_beg[g] < S ? cidx[g_beg[g]] : (int32_t)nc;
}

// kdir[k][w] = the first group of key k whose column is >= kWin w (the key's end for w = nwin):
// the clip-major sweep's per-window group ranges.
__global__ void cluster_kdir_kernel(const uint32_t* __restrict__ g_key, const int32_t* __restrict__ k_gbeg, int32_t nwin,
                                    int32_t* __restrict__ kdir) {
  const int64_t n = (int64_t)kKeyRange * (nwin + 1);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / (nwin + 1)), w = (int)(i % (nwin + 1));
    const int32_t lo = k_gbeg[k], hi = k_gbeg[k + 1];
    kdir[i] = w == nwin ? hi
                        : lo + (int32_t)lower_bound_t<uint32_t>(g_key + lo, hi - lo,
                                                                ((uint32_t)k << kColBits) | (uint32_t)(CellCache::kWin * w));
  }
}

// The sweep's frame sorts (0.6 M pairs at C3): hipCUB's dispatch (a merge sort below 2^20 items,
// 0.17 ms at C3). rocPRIM's onesweep forced instead measured slower there (6 digit passes of
// 23 us: 0.18 ms).
template <class K>
hipError_t sweep_sort_keys(void* tmp, size_t& bytes, const K* kin, K* kout, int64_t n, unsigned end_bit, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortKeys(tmp, bytes, kin, kout, (int)n, 0, (int)end_bit, s);
}
template <class K>
hipError_t sweep_sort_pairs(void* tmp, size_t& bytes, const K* kin, K* kout, const int32_t* vin, int32_t* vout, int64_t n,
                            unsigned end_bit, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, (int)n, 0, (int)end_bit, s);
}

constexpr unsigned kKeysBlocks = 512;  // wide_keys_c_kernel's grid cap (one atomic per block)
inline unsigned grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}

template <class T>
hipError_t dmalloc(T** p, int64_t n) {
  return hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * (size_t)(n > 0 ? n : 1));
}

}  // namespace

namespace {

// ---- the clip order and the cache built from it (round 6) ----------------------------------
// Tiles of 4096 items, 16 per thread of 256, item b0 + k * 256 + t (coalesced loads); a tile's
// exclusive prefix of a per-item flag in item order: chunk k, then wave, then lane.
constexpr int kOT = 256;
constexpr int kOPer = 16;
constexpr int kOTile = kOT * kOPer;

// The key index of the integer nearest m1 (micro-units): floor((m1 + 500000) / 10^6) + kKeyOffset,
// clamped to [0, kKeyRange). A clamped row lies in no box of its key (|k| > 511 dB away).
__device__ __forceinline__ uint32_t order_key_index(int32_t m1) {
  const int64_t v = (int64_t)m1 + 500000;
  const int64_t k = (v >= 0 ? v : v - 999999) / 1000000 + kKeyOffset;
  return (uint32_t)(k < 0 ? 0 : k >= kKeyRange ? kKeyRange - 1 : k);
}

__global__ void order_fill_kernel(const int32_t* __restrict__ m1s, const int32_t* __restrict__ m2s,
                                  const int32_t* __restrict__ cols, int64_t R, unsigned long long* __restrict__ okey,
                                  int32_t* __restrict__ om1) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < R; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t m1 = m1s[i];
    okey[i] = ((unsigned long long)order_key_index(m1) << 53) | ((unsigned long long)(uint32_t)cols[i] << 32) |
              (uint32_t)(m2s[i] ^ INT32_MIN);
    om1[i] = m1;
  }
}

// An index delta's staged rows as order keys: block j takes clip j (local column j), its rows after
// those of clips 0 .. j - 1.
__global__ void delta_order_fill_kernel(const DeltaClip* __restrict__ dc, const int32_t* __restrict__ st_m1,
                                        const int32_t* __restrict__ st_m2, unsigned long long* __restrict__ okey,
                                        int32_t* __restrict__ om1) {
  const int32_t j = blockIdx.x;
  __shared__ int64_t out0;
  if (threadIdx.x == 0) {
    int64_t o = 0;
    for (int32_t i = 0; i < j; i++) o += dc[i].n;
    out0 = o;
  }
  __syncthreads();
  const int64_t src = dc[j].off;
  for (int32_t i = threadIdx.x; i < dc[j].n; i += blockDim.x) {
    const int32_t m1 = st_m1[src + i];
    okey[out0 + i] = ((unsigned long long)order_key_index(m1) << 53) | ((unsigned long long)(uint32_t)j << 32) |
                     (uint32_t)(st_m2[src + i] ^ INT32_MIN);
    om1[out0 + i] = m1;
  }
}

// Is an order row with max1 m1 a point at this tolerance (m1 inside the "%f" box of its key index,
// which is order_key_index(m1) by construction: the key itself is not needed)?
__device__ __forceinline__ bool order_point(int32_t m1, const int64_t* __restrict__ kbox) {
  const uint32_t t = order_key_index(m1);
  return (int64_t)m1 >= kbox[2 * t] && (int64_t)m1 <= kbox[2 * t + 1];
}

// Block-wide exclusive prefix of one count per thread (kOT threads, thread order); *tot = the
// block's total. wsum: kOT / 64 words of LDS. Every thread of the block calls it.
__device__ __forceinline__ int32_t block_prefix(int32_t x, int32_t* wsum, int32_t* tot) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int32_t base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kOT / 64; w++) {
    const int32_t v = wsum[w];
    base += w < wv ? v : 0;
    all += v;
  }
  *tot = all;
  return base + inc - x;
}

// Which of a thread's kOPer consecutive order rows (rows r0 = b0 + kOPer t ..: 16-byte loads of
// their max1 only; the last tile's rows past n are not points) are points at this tolerance.
__device__ __forceinline__ uint32_t order_rows(const int32_t* __restrict__ om1, int64_t n, const int64_t* __restrict__ kbox,
                                               int64_t r0) {
  int32_t m1[kOPer];
  if (r0 + kOPer <= n) {
    const int4* m4 = reinterpret_cast<const int4*>(om1 + r0);
#pragma unroll
    for (int q = 0; q < kOPer / 4; q++) {
      const int4 v = m4[q];
      m1[4 * q] = v.x;
      m1[4 * q + 1] = v.y;
      m1[4 * q + 2] = v.z;
      m1[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kOPer; k++) m1[k] = r0 + k < n ? om1[r0 + k] : 0;
  }
  uint32_t bits = 0;
  // the rows are in key order: when the thread's first and last row share a key index (nearly
  // always), one box for all of them
  const uint32_t t0 = order_key_index(m1[0]);
  if (r0 + kOPer <= n && order_key_index(m1[kOPer - 1]) == t0) {
    const int64_t lo = kbox[2 * t0], hi = kbox[2 * t0 + 1];
#pragma unroll
    for (int k = 0; k < kOPer; k++) bits |= (uint32_t)((int64_t)m1[k] >= lo && (int64_t)m1[k] <= hi) << k;
    return bits;
  }
#pragma unroll
  for (int k = 0; k < kOPer; k++)
    if (r0 + k < n && order_point(m1[k], kbox)) bits |= 1u << k;
  return bits;
}

// Points per tile of the order (the tile's count into cnt[tile]).
__global__ __launch_bounds__(kOT) void order_count_kernel(const int32_t* __restrict__ om1, int64_t n,
                                                          const int64_t* __restrict__ kbox, int32_t* __restrict__ cnt) {
  __shared__ int32_t wsum[kOT / 64];
  const uint32_t bits = order_rows(om1, n, kbox, (int64_t)blockIdx.x * kOTile + kOPer * threadIdx.x);
  int32_t tot;
  (void)block_prefix(__popc(bits), wsum, &tot);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// Exclusive scan, in place, of nvec vectors of ntiles counts each (vector v at cnt + v (ntiles + 1));
// each vector's total lands in its element ntiles. One workgroup of 1024 threads: a vector of up to
// kScanLds counts goes through LDS (coalesced loads and stores; each thread then scans its
// contiguous share there), a longer one is scanned in place.
constexpr int32_t kScanLds = 30720;
__global__ __launch_bounds__(1024) void tile_scan_kernel(int32_t* __restrict__ cnt, int32_t ntiles, int32_t nvec) {
  __shared__ int32_t part[1024];
  __shared__ int32_t buf[kScanLds];
  const int t = threadIdx.x;
  const int32_t per = (ntiles + 1023) / 1024;
  const bool inlds = ntiles <= kScanLds;
  for (int32_t v = 0; v < nvec; v++) {
    int32_t* c = cnt + (int64_t)v * (ntiles + 1);
    const int32_t a = t * per, e = min(ntiles, a + per);
    int32_t sum = 0;
    if (inlds) {
      for (int32_t i = t; i < ntiles; i += 1024) buf[i] = c[i];
      __syncthreads();
      for (int32_t i = a; i < e; i++) sum += buf[i];
    } else {
      for (int32_t i = a; i < e; i++) sum += c[i];
    }
    part[t] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan of the partial sums
      const int32_t x = t >= o ? part[t - o] : 0;
      __syncthreads();
      part[t] += x;
      __syncthreads();
    }
    int32_t run = part[t] - sum;
    if (inlds) {
      for (int32_t i = a; i < e; i++) {
        const int32_t x = buf[i];
        buf[i] = run;
        run += x;
      }
      __syncthreads();
      for (int32_t i = t; i < ntiles; i += 1024) c[i] = buf[i];
    } else {
      for (int32_t i = a; i < e; i++) {
        const int32_t x = c[i];
        c[i] = run;
        run += x;
      }
    }
    if (t == 1023) c[ntiles] = part[1023];
    __syncthreads();
  }
}

// The points: every order row inside its key's box, in order (p_m2 = its m2, k32 = key << 21 | col).
// kStage (dense points: most rows of a tile): the tile's points staged in LDS and written as one
// contiguous run; sparse points are written where they fall (the 32 KB of staging would cost the
// launch occupancy for nothing).
template <bool kStage>
__global__ __launch_bounds__(kOT) void order_points_kernel(const unsigned long long* __restrict__ okey,
                                                           const int32_t* __restrict__ om1, int64_t n,
                                                           const int64_t* __restrict__ kbox, const int32_t* __restrict__ off,
                                                           int32_t* __restrict__ p_m2, uint32_t* __restrict__ k32) {
  __shared__ int32_t wsum[kOT / 64];
  __shared__ int32_t sv[kStage ? kOTile : 1];
  __shared__ uint32_t sk[kStage ? kOTile : 1];
  const int64_t r0 = (int64_t)blockIdx.x * kOTile + kOPer * threadIdx.x;
  const uint32_t bits = order_rows(om1, n, kbox, r0);
  int32_t tot;
  int32_t j = block_prefix(__popc(bits), wsum, &tot);
  // the points' keys: all of the thread's rows in 16-byte loads when most are points, else one by one
  unsigned long long key[kOPer];
  if (__popc(bits) > kOPer / 4 && r0 + kOPer <= n) {
    const ulonglong2* k2 = reinterpret_cast<const ulonglong2*>(okey + r0);
#pragma unroll
    for (int q = 0; q < kOPer / 2; q++) {
      const ulonglong2 v = k2[q];
      key[2 * q] = v.x;
      key[2 * q + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kOPer; k++) key[k] = (bits >> k) & 1u ? okey[r0 + k] : 0ull;
  }
  const int64_t o = off[blockIdx.x];
  if constexpr (!kStage) {
#pragma unroll
    for (int k = 0; k < kOPer; k++)
      if ((bits >> k) & 1u) {
        p_m2[o + j] = (int32_t)((uint32_t)key[k] ^ 0x80000000u);
        k32[o + j] = (uint32_t)(key[k] >> 32);  // key << 21 | column
        j++;
      }
    return;
  }
#pragma unroll
  for (int k = 0; k < kOPer; k++)
    if ((bits >> k) & 1u) {
      sv[j] = (int32_t)((uint32_t)key[k] ^ 0x80000000u);
      sk[j] = (uint32_t)(key[k] >> 32);
      j++;
    }
  __syncthreads();
  for (int32_t i = threadIdx.x; i < tot; i += kOT) {
    p_m2[o + i] = sv[i];
    k32[o + i] = sk[i];
  }
}

// A thread's kOPer consecutive points j0 .. (16-byte loads) with their neighbours j0 - 1 and
// j0 + kOPer: point j starts a group when its (key, column) differs from point j - 1's, a cluster
// when it starts a group or lies more than dgap above its predecessor; it ends a cluster when
// point j + 1 starts one or j is the last point. Bits of the points below S.
__device__ __forceinline__ void point_flags(const int32_t* __restrict__ p_m2, const uint32_t* __restrict__ k32, int64_t S,
                                            int64_t dgap, int64_t j0, int32_t (&v)[kOPer], uint32_t& gbits,
                                            uint32_t& cbits, uint32_t& ebits) {
  uint32_t kk[kOPer + 2];  // points j0 - 1 .. j0 + kOPer
  int32_t vv[kOPer + 2];
  if (j0 + kOPer <= S) {
    const int4* v4 = reinterpret_cast<const int4*>(p_m2 + j0);
    const uint4* k4 = reinterpret_cast<const uint4*>(k32 + j0);
#pragma unroll
    for (int q = 0; q < kOPer / 4; q++) {
      const int4 a = v4[q];
      const uint4 b = k4[q];
      vv[1 + 4 * q] = a.x, vv[2 + 4 * q] = a.y, vv[3 + 4 * q] = a.z, vv[4 + 4 * q] = a.w;
      kk[1 + 4 * q] = b.x, kk[2 + 4 * q] = b.y, kk[3 + 4 * q] = b.z, kk[4 + 4 * q] = b.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kOPer; k++) {
      vv[1 + k] = j0 + k < S ? p_m2[j0 + k] : 0;
      kk[1 + k] = j0 + k < S ? k32[j0 + k] : 0u;
    }
  }
  const bool prev = j0 > 0 && j0 - 1 < S;  // (threads past the last point read nothing)
  vv[0] = prev ? p_m2[j0 - 1] : 0;
  kk[0] = prev ? k32[j0 - 1] : ~0u;  // (point 0 starts a group: no key equals ~0)
  vv[kOPer + 1] = j0 + kOPer < S ? p_m2[j0 + kOPer] : 0;
  kk[kOPer + 1] = j0 + kOPer < S ? k32[j0 + kOPer] : 0u;
  gbits = cbits = ebits = 0;
  bool cs_next = false;
#pragma unroll
  for (int k = kOPer; k >= 0; k--) {  // k: point j0 + k - 1 (k = kOPer: the neighbour j0 + kOPer)
    const int64_t j = j0 + k;        // (the point whose flags this step forms: j0 + k)
    const bool in = j < S;
    const bool gs = in && kk[k + 1] != kk[k];
    const bool cs = in && (gs || (int64_t)vv[k + 1] - (int64_t)vv[k] > dgap);
    if (k < kOPer && in) {
      gbits |= (uint32_t)gs << k;
      cbits |= (uint32_t)cs << k;
      ebits |= (uint32_t)(cs_next || j == S - 1) << k;
    }
    cs_next = cs;
  }
#pragma unroll
  for (int k = 0; k < kOPer; k++) v[k] = vv[1 + k];
}

__global__ __launch_bounds__(kOT) void point_count_kernel(const int32_t* __restrict__ p_m2, const uint32_t* __restrict__ k32,
                                                          int64_t S, int64_t dgap, int32_t ntiles,
                                                          int32_t* __restrict__ cnt) {
  __shared__ int32_t wsum[kOT / 64];
  int32_t v[kOPer];
  uint32_t gbits, cbits, ebits;
  point_flags(p_m2, k32, S, dgap, (int64_t)blockIdx.x * kOTile + kOPer * threadIdx.x, v, gbits, cbits, ebits);
  int32_t tot;  // groups << 16 | clusters (each at most kOTile per tile)
  (void)block_prefix((__popc(gbits) << 16) | __popc(cbits), wsum, &tot);
  if (threadIdx.x == 0) {
    cnt[blockIdx.x] = tot >> 16;
    cnt[ntiles + 1 + blockIdx.x] = tot & 0xffff;
  }
}

// Groups and clusters of the points: g_key / g_beg / c_beg per group, c_lo / c_hi per cluster;
// the point S - 1 closes the arrays (g_beg[n1] = S, c_beg[n1] = nc).
__global__ __launch_bounds__(kOT) void point_groups_kernel(const int32_t* __restrict__ p_m2, const uint32_t* __restrict__ k32,
                                                           int64_t S, int64_t dgap, int32_t ntiles,
                                                           const int32_t* __restrict__ off, uint32_t* __restrict__ g_key,
                                                           int32_t* __restrict__ g_beg, int32_t* __restrict__ c_beg,
                                                           int32_t* __restrict__ c_lo, int32_t* __restrict__ c_hi) {
  __shared__ int32_t wsum[kOT / 64];
  const int64_t j0 = (int64_t)blockIdx.x * kOTile + kOPer * threadIdx.x;
  int32_t v[kOPer];
  uint32_t gbits, cbits, ebits;
  point_flags(p_m2, k32, S, dgap, j0, v, gbits, cbits, ebits);
  int32_t tot;
  const int32_t pre = block_prefix((__popc(gbits) << 16) | __popc(cbits), wsum, &tot);
  int32_t g = off[blockIdx.x] + (pre >> 16);                 // this thread's first group start
  int32_t c = off[ntiles + 1 + blockIdx.x] + (pre & 0xffff) - 1;  // the cluster of the point before j0
  const int32_t n1 = off[ntiles], nc = off[2 * (ntiles + 1) - 1];
#pragma unroll
  for (int k = 0; k < kOPer; k++) {
    const int64_t j = j0 + k;
    if ((cbits >> k) & 1u) {
      c++;
      c_lo[c] = v[k];
    }
    if ((gbits >> k) & 1u) {
      g_key[g] = k32[j];
      g_beg[g] = (int32_t)j;
      c_beg[g] = c;
      g++;
    }
    if ((ebits >> k) & 1u) c_hi[c] = v[k];
    if (j == S - 1) {
      g_beg[n1] = (int32_t)S;
      c_beg[n1] = nc;
    }
  }
}

}  // namespace

hipError_t CacheBuf::reserve(size_t n) {
  if (n <= bytes) return hipSuccess;
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
  const size_t want = std::max<size_t>(256, n + n / 8);
  const hipError_t e = hipMalloc(&p, want);
  if (e == hipSuccess) bytes = want;
  return e;
}

void CacheBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
}

hipError_t launch_order_fill(const int32_t* m1s, const int32_t* m2s, const int32_t* cols, int64_t R,
                             unsigned long long* okey, int32_t* om1, hipStream_t s) {
  if (R <= 0) return hipSuccess;
  hipLaunchKernelGGL(order_fill_kernel, dim3(grid_for(R)), dim3(256), 0, s, m1s, m2s, cols, R, okey, om1);
  return hipGetLastError();
}

hipError_t launch_delta_order_fill(const DeltaClip* d_dc, int32_t nd, const int32_t* st_m1, const int32_t* st_m2,
                                   unsigned long long* okey, int32_t* om1, hipStream_t s) {
  if (nd <= 0) return hipSuccess;
  hipLaunchKernelGGL(delta_order_fill_kernel, dim3((unsigned)nd), dim3(256), 0, s, d_dc, st_m1, st_m2, okey, om1);
  return hipGetLastError();
}

// The order's one sort (per full build; merges carry it): hipCUB's radix sort of the 63-bit keys
// with m1 beside them.
hipError_t order_sort(const unsigned long long* kin, unsigned long long* kout, const int32_t* vin, int32_t* vout, int64_t n,
                      CacheBuf* tmp, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n >= INT32_MAX) return hipErrorInvalidValue;
  size_t tb = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, vin, vout, (int)n, 0, 63, s);
  if (e != hipSuccess) return e;
  if ((e = tmp->reserve(tb)) != hipSuccess) return e;
  tb = tmp->bytes;
  return hipcub::DeviceRadixSort::SortPairs(tmp->p, tb, kin, kout, vin, vout, (int)n, 0, 63, s);
}

void CellCache::bind() {
  p_m2 = b_p_m2.as<int32_t>();
  k32 = b_k32.as<uint32_t>();
  g_key = b_g_key.as<uint32_t>();
  g_beg = b_g_beg.as<int32_t>();
  e_key = b_e_key.as<unsigned long long>();
  e_grp = b_e_grp.as<int32_t>();
  k_gbeg = b_k_gbeg.as<int32_t>();
  c_lo = b_c_lo.as<int32_t>();
  c_hi = b_c_hi.as<int32_t>();
  c_beg = b_c_beg.as<int32_t>();
  kdir = b_kdir.as<int32_t>();
}

void CellCache::release() {
  for (CacheBuf* b : {&b_p_m2, &b_k32, &b_g_key, &b_g_beg, &b_e_key, &b_e_grp, &b_k_gbeg, &b_c_lo, &b_c_hi, &b_c_beg, &b_kdir,
                      &b_tile})
    b->release();
  bind();
  invalidate();
  nwin = 0;
  w = dgap = 0;
}

void CellCache::swap(CellCache& o) {
  std::swap(b_p_m2, o.b_p_m2);
  std::swap(b_k32, o.b_k32);
  std::swap(b_g_key, o.b_g_key);
  std::swap(b_g_beg, o.b_g_beg);
  std::swap(b_e_key, o.b_e_key);
  std::swap(b_e_grp, o.b_e_grp);
  std::swap(b_k_gbeg, o.b_k_gbeg);
  std::swap(b_c_lo, o.b_c_lo);
  std::swap(b_c_hi, o.b_c_hi);
  std::swap(b_c_beg, o.b_c_beg);
  std::swap(b_kdir, o.b_kdir);
  std::swap(b_tile, o.b_tile);
  std::swap(nwin, o.nwin);
  std::swap(S, o.S);
  std::swap(n1, o.n1);
  std::swap(n2, o.n2);
  std::swap(w, o.w);
  std::swap(nc, o.nc);
  std::swap(dgap, o.dgap);
  std::swap(valid, o.valid);
  std::swap(entries, o.entries);
  std::swap(from_order, o.from_order);
  bind();
  o.bind();
}

// The per-key window directory and each key's first group (both build forms).
static hipError_t cache_directory(CellCache* c, int32_t ncols, hipStream_t s, CacheBuf* b_k_gbeg, CacheBuf* b_kdir) {
  hipError_t e;
  if ((e = b_k_gbeg->reserve(sizeof(int32_t) * (kKeyRange + 1))) != hipSuccess) return e;
  c->nwin = (ncols + CellCache::kWin - 1) / CellCache::kWin;
  if ((e = b_kdir->reserve(sizeof(int32_t) * (size_t)kKeyRange * (c->nwin + 1))) != hipSuccess) return e;
  hipLaunchKernelGGL(key_gbeg_kernel, dim3((kKeyRange + 256) / 256), dim3(256), 0, s, c->g_key, c->n1,
                     b_k_gbeg->as<int32_t>());
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(cluster_kdir_kernel, dim3(grid_for((int64_t)kKeyRange * (c->nwin + 1))), dim3(256), 0, s, c->g_key,
                     b_k_gbeg->as<int32_t>(), c->nwin, b_kdir->as<int32_t>());
  return hipGetLastError();
}

hipError_t CellCache::build_from_order(const unsigned long long* okey, const int32_t* om1, int64_t n, const int64_t* d_kbox,
                                       int32_t ncols, double tole, hipStream_t s) {
  invalidate();
  if (!(tole >= 0.0 && tole <= kOrderMaxTol) || ncols > kMaxCols || n <= 0 || n >= INT32_MAX) return hipSuccess;
  w = (int64_t)ceil(2.0 * tole * 1e6) + 4;  // >= U2 - L2 of every fmt6 max2 window at this tolerance
  dgap = std::max<int64_t>(0, (int64_t)floor(2.0 * tole * 1e6) - 3);
  const int32_t nt = (int32_t)((n + kOTile - 1) / kOTile);
  hipError_t e;
  if ((e = b_tile.reserve(sizeof(int32_t) * 2 * ((size_t)nt + 1))) != hipSuccess) return e;
  int32_t* cnt = b_tile.as<int32_t>();
  // 1. the points: a count per tile, their offsets, the filter
  hipLaunchKernelGGL(order_count_kernel, dim3((unsigned)nt), dim3(kOT), 0, s, om1, n, d_kbox, cnt);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, nt, 1);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  int32_t tot[2] = {0, 0};
  if ((e = hipMemcpyAsync(&tot[0], cnt + nt, sizeof(int32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = hipStreamSynchronize(s)) != hipSuccess)
    return e;
  S = tot[0];
  if (S <= 0) {
    S = 0;
    return hipSuccess;  // no row in any box: the row scan (which finds none either)
  }
  if ((e = b_p_m2.reserve(sizeof(int32_t) * (size_t)S)) != hipSuccess || (e = b_k32.reserve(sizeof(uint32_t) * (size_t)S)) != hipSuccess)
    return e;
  bind();
  if (4 * S > n)  // (dense: most rows are points)
    hipLaunchKernelGGL(order_points_kernel<true>, dim3((unsigned)nt), dim3(kOT), 0, s, okey, om1, n, d_kbox, cnt, p_m2, k32);
  else
    hipLaunchKernelGGL(order_points_kernel<false>, dim3((unsigned)nt), dim3(kOT), 0, s, okey, om1, n, d_kbox, cnt, p_m2, k32);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // 2. groups and clusters: two counts per tile, their offsets, then the arrays
  const int32_t nt2 = (int32_t)((S + kOTile - 1) / kOTile);
  hipLaunchKernelGGL(point_count_kernel, dim3((unsigned)nt2), dim3(kOT), 0, s, p_m2, k32, S, dgap, nt2, cnt);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, nt2, 2);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(&tot[0], cnt + nt2, sizeof(int32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = hipMemcpyAsync(&tot[1], cnt + 2 * (nt2 + 1) - 1, sizeof(int32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = hipStreamSynchronize(s)) != hipSuccess)
    return e;
  n1 = tot[0];
  nc = tot[1];
  if ((e = b_g_key.reserve(sizeof(uint32_t) * (size_t)n1)) != hipSuccess ||
      (e = b_g_beg.reserve(sizeof(int32_t) * (size_t)(n1 + 1))) != hipSuccess ||
      (e = b_c_beg.reserve(sizeof(int32_t) * (size_t)(n1 + 1))) != hipSuccess ||
      (e = b_c_lo.reserve(sizeof(int32_t) * (size_t)nc)) != hipSuccess || (e = b_c_hi.reserve(sizeof(int32_t) * (size_t)nc)) != hipSuccess)
    return e;
  bind();
  hipLaunchKernelGGL(point_groups_kernel, dim3((unsigned)nt2), dim3(kOT), 0, s, p_m2, k32, S, dgap, nt2, cnt, g_key, g_beg,
                     c_beg, c_lo, c_hi);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = cache_directory(this, ncols, s, &b_k_gbeg, &b_kdir)) != hipSuccess) return e;
  bind();
  valid = true;
  from_order = true;
  return hipSuccess;
}

hipError_t CellCache::build(const int64_t* d_rng_all, const int64_t* h_off, const int32_t* m2s, const int32_t* cols,
                            int32_t ncols, int64_t nrows, double tole, hipStream_t s) {
  invalidate();
  S = h_off[kKeyRange];
  // limits of the packed keys and of hipcub's 32-bit counts; beyond them every frame takes the
  // row scan (correct, slower)
  if (!(tole >= 0.0 && tole < 1e6) || ncols > kMaxCols || S <= 0 || 2 * S >= INT32_MAX || S > 4 * nrows + (1 << 20)) {
    S = 0;
    return hipSuccess;
  }
  w = (int64_t)ceil(2.0 * tole * 1e6) + 4;  // >= U2 - L2 of every fmt6 max2 window at this tolerance
  dgap = std::max<int64_t>(0, (int64_t)floor(2.0 * tole * 1e6) - 3);
  // (tolerances above kOrderMaxTol only: a max1 box then spans several keys' rows of the clip
  // order, so the boxes' rows are sorted here; the scratch is allocated for the build alone)
  hipError_t e;
  int64_t* d_off = nullptr;
  unsigned long long *ka = nullptr, *kb = nullptr;
  int32_t *glen = nullptr, *ga = nullptr, *gb = nullptr;
  int64_t* d_n = nullptr;
  void* tmp = nullptr;
  size_t tb = 0, t1 = 0;
  int64_t nn[2] = {0, 0};
#define TFP_TRY(x)               \
  do {                           \
    e = (x);                     \
    if (e != hipSuccess) goto out; \
  } while (0)
  TFP_TRY(dmalloc(&d_off, kKeyRange + 1));
  TFP_TRY(hipMemcpyAsync(d_off, h_off, sizeof(int64_t) * (kKeyRange + 1), hipMemcpyHostToDevice, s));
  TFP_TRY(dmalloc(&ka, S));
  TFP_TRY(dmalloc(&kb, S));
  TFP_TRY(dmalloc(&d_n, 2));
  TFP_TRY(dmalloc(&glen, S + 1));
  hipLaunchKernelGGL(cells_fill_kernel, dim3(grid_for(S)), dim3(256), 0, s, d_rng_all, d_off, m2s, cols, S, ka);
  TFP_TRY(hipGetLastError());
  // (key, col, m2) order: the groups, each group's points ascending
  TFP_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, t1, ka, kb, (int)S, 0, 63, s));
  tb = t1;
  TFP_TRY(hipcub::DeviceRunLengthEncode::Encode(nullptr, t1, k32, g_key, glen, d_n, (int)S, s));
  tb = t1 > tb ? t1 : tb;
  TFP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, glen, glen, (int)S, s));
  tb = t1 > tb ? t1 : tb;
  TFP_TRY(hipMalloc(&tmp, tb > 0 ? tb : 1));
  TFP_TRY(hipcub::DeviceRadixSort::SortKeys(tmp, tb, ka, kb, (int)S, 0, 63, s));
  TFP_TRY(b_p_m2.reserve(sizeof(int32_t) * (size_t)S));
  TFP_TRY(b_k32.reserve(sizeof(uint32_t) * (size_t)S));
  TFP_TRY(b_g_key.reserve(sizeof(uint32_t) * (size_t)S));
  bind();
  hipLaunchKernelGGL(cells_split_kernel, dim3(grid_for(S)), dim3(256), 0, s, kb, S, p_m2, k32);
  TFP_TRY(hipGetLastError());
  TFP_TRY(hipcub::DeviceRunLengthEncode::Encode(tmp, tb, k32, g_key, glen, d_n, (int)S, s));
  TFP_TRY(hipMemcpyAsync(nn, d_n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TFP_TRY(hipStreamSynchronize(s));
  n1 = nn[0];
  // group offsets: exclusive sum of the run lengths, g_beg[n1] = S
  TFP_TRY(b_g_beg.reserve(sizeof(int32_t) * (size_t)(n1 + 1)));
  bind();
  TFP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, glen, g_beg, (int)n1, s));
  {
    const int32_t S32 = (int32_t)S;  // S < 2^31
    TFP_TRY(hipMemcpyAsync(g_beg + n1, &S32, sizeof(int32_t), hipMemcpyHostToDevice, s));
    // the sweep's clusters: flags into ga, their prefix into gb
    TFP_TRY(dmalloc(&ga, S));
    TFP_TRY(dmalloc(&gb, S));
    hipLaunchKernelGGL(cluster_flag_kernel, dim3(grid_for(S)), dim3(256), 0, s, p_m2, k32, S, dgap, ga);
    TFP_TRY(hipGetLastError());
    TFP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, ga, gb, (int)S, s));
    int32_t last[2] = {0, 0};
    TFP_TRY(hipMemcpyAsync(&last[0], gb + S - 1, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    TFP_TRY(hipMemcpyAsync(&last[1], ga + S - 1, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    TFP_TRY(hipStreamSynchronize(s));  // (also: S32 was read)
    nc = (int64_t)last[0] + last[1];
  }
  TFP_TRY(b_c_lo.reserve(sizeof(int32_t) * (size_t)std::max<int64_t>(nc, 1)));
  TFP_TRY(b_c_hi.reserve(sizeof(int32_t) * (size_t)std::max<int64_t>(nc, 1)));
  TFP_TRY(b_c_beg.reserve(sizeof(int32_t) * (size_t)(n1 + 1)));
  bind();
  hipLaunchKernelGGL(cluster_write_kernel, dim3(grid_for(S)), dim3(256), 0, s, p_m2, ga, gb, S, c_lo, c_hi);
  hipLaunchKernelGGL(cluster_gbeg_kernel, dim3(grid_for(n1 + 1)), dim3(256), 0, s, g_beg, gb, n1, S, nc, c_beg);
  TFP_TRY(hipGetLastError());
  TFP_TRY(cache_directory(this, ncols, s, &b_k_gbeg, &b_kdir));
  bind();
  TFP_TRY(hipStreamSynchronize(s));  // (the scratch is freed below)
  valid = true;
out:
#undef TFP_TRY
  for (void* p : {(void*)d_off, (void*)ka, (void*)kb, (void*)glen, (void*)ga, (void*)gb, (void*)d_n, tmp})
    if (p) (void)hipFree(p);
  if (e != hipSuccess) invalidate();
  return e;
}

// The cell entries (the one-wave-per-frame cells form's candidates: two per point, its own cell j
// and j - 1, deduplicated per (key, cell, column)), built when that form first runs on this cache.
hipError_t CellCache::ensure_entries(hipStream_t s) {
  if (!valid || entries) return hipSuccess;
  if (2 * S >= INT32_MAX) return hipErrorInvalidValue;
  hipError_t e;
  unsigned long long* eb = nullptr;
  int32_t* gb = nullptr;
  int64_t* d_n = nullptr;
  void* tmp = nullptr;
  size_t tb = 0, t1 = 0;
  int64_t nn = 0;
#define TFP_TRY(x)               \
  do {                           \
    e = (x);                     \
    if (e != hipSuccess) goto out; \
  } while (0)
  TFP_TRY(b_e_key.reserve(sizeof(unsigned long long) * (size_t)(2 * S)));
  TFP_TRY(b_e_grp.reserve(sizeof(int32_t) * (size_t)(2 * S)));
  bind();
  TFP_TRY(dmalloc(&eb, 2 * S));
  TFP_TRY(dmalloc(&gb, 2 * S));
  TFP_TRY(dmalloc(&d_n, 1));
  TFP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, t1, e_key, eb, e_grp, gb, (int)(2 * S), 0, 62, s));
  tb = t1;
  TFP_TRY(hipcub::DeviceSelect::UniqueByKey(nullptr, t1, eb, gb, e_key, e_grp, d_n, (int)(2 * S), s));
  tb = t1 > tb ? t1 : tb;
  TFP_TRY(hipMalloc(&tmp, tb > 0 ? tb : 1));
  hipLaunchKernelGGL(cells_entries_kernel, dim3(grid_for(S)), dim3(256), 0, s, p_m2, k32, S, g_key, n1, w, e_key, e_grp);
  TFP_TRY(hipGetLastError());
  TFP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, e_key, eb, e_grp, gb, (int)(2 * S), 0, 62, s));
  TFP_TRY(hipcub::DeviceSelect::UniqueByKey(tmp, tb, eb, gb, e_key, e_grp, d_n, (int)(2 * S), s));
  TFP_TRY(hipMemcpyAsync(&nn, d_n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TFP_TRY(hipStreamSynchronize(s));
  n2 = nn;
  entries = true;
out:
#undef TFP_TRY
  for (void* p : {(void*)eb, (void*)gb, (void*)d_n, tmp})
    if (p) (void)hipFree(p);
  return e;
}

namespace {

// ---- search kernels -----------------------------------------------------------------------

struct CellView {
  const int32_t* p_m2;
  const int32_t* p_hi;  // the sweep: each item's last point (its cluster's; p_m2 when items are points)
  const uint32_t* g_key;
  const int32_t* g_beg;
  const unsigned long long* e_key;
  const int32_t* e_grp;
  int64_t n1, n2, w;
  int32_t valid;
};

// Does the cached clip-set path serve this frame? (else: the row scan with stamps)
__device__ __forceinline__ bool cell_frame(const FrameBox& bx, const CellView& cv) {
  const int64_t kk = (int64_t)bx.k + kKeyOffset;
  if (!cv.valid || kk < 0 || kk >= kKeyRange) return false;
  return !(bx.flags & 2) || bx.U2 - bx.L2 <= cv.w;
}

// Score one hit of query row qr on clip col; a clip's first count appends it to the touched list.
__device__ __forceinline__ void count_hit(int32_t* sc, int32_t* tl, int32_t* tcnt, int32_t col) {
  if (atomicAdd(&sc[col], 1) == 0) tl[atomicAdd(tcnt, 1)] = col;
}

// One wave per frame of the chunk's queries [q_begin, q_begin + nq).
__global__ __launch_bounds__(256) void scan_cells_kernel(const FrameBox* __restrict__ boxes,
                                                         const int64_t* __restrict__ qoff, int32_t q_begin, int32_t nq,
                                                         CellView cv, int32_t C, int32_t* __restrict__ score,
                                                         int32_t* __restrict__ touched, int32_t* __restrict__ tcnt) {
  const int64_t f0 = qoff[q_begin], nf = qoff[q_begin + nq] - f0;
  const int64_t wf = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wf >= nf) return;
  const int64_t f = f0 + wf;
  const FrameBox bx = boxes[f];
  if (!(bx.flags & 1) || !cell_frame(bx, cv)) return;
  // the frame's query: the last q with qoff[q] <= f
  int lo = 0, hi = nq;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (qoff[q_begin + mid] <= f) lo = mid; else hi = mid;
  }
  int32_t* sc = score + (int64_t)lo * C;
  int32_t* tl = touched + (int64_t)lo * C;
  int32_t* tc = tcnt + lo;
  const unsigned long long kk = (unsigned long long)((int64_t)bx.k + kKeyOffset);
  if (bx.flags & 2) {  // max1 box AND max2 window: the cell's candidates, each confirmed
    const unsigned long long j = (unsigned long long)cell_of(bx.L2, cv.w);
    const int64_t a = lower_bound_t<unsigned long long>(cv.e_key, cv.n2, (kk << 52) | (j << kColBits));
    const int64_t b = lower_bound_t<unsigned long long>(cv.e_key, cv.n2, (kk << 52) | ((j + 1) << kColBits));
    for (int64_t e = a + lane; e < b; e += 64) {
      const int32_t g = cv.e_grp[e];
      const int32_t pb = cv.g_beg[g], pn = cv.g_beg[g + 1] - pb;
      const int64_t p = lb_i32(cv.p_m2 + pb, pn, bx.L2);
      if (p < pn && (int64_t)cv.p_m2[pb + p] <= bx.U2) count_hit(sc, tl, tc, (int32_t)(cv.e_key[e] & kColMask));
    }
  } else {  // the max1 box alone: every clip with a row in it
    const int64_t a = lower_bound_t<uint32_t>(cv.g_key, cv.n1, (uint32_t)(kk << kColBits));
    const int64_t b = lower_bound_t<uint32_t>(cv.g_key, cv.n1, (uint32_t)((kk + 1) << kColBits));
    for (int64_t e = a + lane; e < b; e += 64) count_hit(sc, tl, tc, (int32_t)(cv.g_key[e] & kColMask));
  }
}

// The frames cell_frame declines, per query in frame order: the rows of the max1 box from the
// m1-sorted index (max2 filtered), deduplicated per frame by a stamp = the frame's ordinal.
__global__ __launch_bounds__(256) void scan_rows_kernel(const FrameBox* __restrict__ boxes,
                                                        const int64_t* __restrict__ qoff, int32_t q_begin, int32_t nq,
                                                        CellView cv, const int32_t* __restrict__ m1s,
                                                        const int32_t* __restrict__ m2s,
                                                        const int32_t* __restrict__ cols, int64_t R, int32_t C,
                                                        int32_t* __restrict__ stamp, int32_t* __restrict__ score,
                                                        int32_t* __restrict__ touched, int32_t* __restrict__ tcnt) {
  const int wq = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wq >= nq) return;
  const int q = q_begin + wq;
  int32_t* st = stamp + (int64_t)wq * C;
  int32_t* sc = score + (int64_t)wq * C;
  int32_t* tl = touched + (int64_t)wq * C;
  const int64_t fbeg = qoff[q], fend = qoff[q + 1];
  for (int64_t i = fbeg; i < fend; i++) {
    const FrameBox bx = boxes[i];
    if (!(bx.flags & 1) || cell_frame(bx, cv)) continue;
    const int32_t tag = (int32_t)(i - fbeg) + 1;
    const int64_t a = lb_i32(m1s, R, bx.L1), b = ub_i32(m1s, R, bx.U1);
    for (int64_t rr = a + lane; rr < b; rr += 64) {
      if (bx.flags & 2) {
        const int32_t v = m2s[rr];
        if (v == kNullMicro || (int64_t)v < bx.L2 || (int64_t)v > bx.U2) continue;
      }
      const int32_t col = cols[rr];
      if (atomicMax(&st[col], tag) < tag) count_hit(sc, tl, tcnt + wq, col);
    }
  }
}

// Per query: max over its touched clips of (count << 32 | tie key), scratch restored to zero.
__global__ __launch_bounds__(256) void scan_final_kernel(int32_t q_begin, int32_t nq, const int32_t* __restrict__ tiekey,
                                                         int32_t C, int32_t* __restrict__ stamp,
                                                         int32_t* __restrict__ score, int32_t* __restrict__ touched,
                                                         int32_t* __restrict__ tcnt, unsigned long long* __restrict__ best) {
  const int wq = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wq >= nq) return;
  int32_t* st = stamp + (int64_t)wq * C;
  int32_t* sc = score + (int64_t)wq * C;
  const int32_t* tl = touched + (int64_t)wq * C;
  const int32_t n = tcnt[wq];
  unsigned long long key = 0;
  for (int32_t j = lane; j < n; j += 64) {
    const int32_t c = tl[j];
    const unsigned long long k = ((unsigned long long)(uint32_t)sc[c] << 32) | (uint32_t)tiekey[c];
    key = k > key ? k : key;
    sc[c] = 0;
    st[c] = 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long other = __shfl_xor(key, o, 64);
    key = other > key ? other : key;
  }
  if (lane == 0) {
    best[q_begin + wq] = key;
    tcnt[wq] = 0;
  }
}

}  // namespace

hipError_t launch_scan(const FrameBox* boxes, const int64_t* d_qoff, const int64_t* h_qoff, int32_t q_begin, int32_t nq,
                       const int32_t* m1s, const int32_t* m2s, const int32_t* cols, int64_t R, const CellCache* cells,
                       const int32_t* d_tiekey, int32_t C, int32_t* d_stamp, int32_t* d_score, int32_t* d_touched,
                       int32_t* d_tcnt, unsigned long long* d_best, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  CellView cv;
  memset(&cv, 0, sizeof cv);
  if (cells && cells->valid) {
    cv.p_m2 = cells->p_m2;
    cv.g_key = cells->g_key;
    cv.g_beg = cells->g_beg;
    cv.e_key = cells->e_key;
    cv.e_grp = cells->e_grp;
    cv.n1 = cells->n1;
    cv.n2 = cells->n2;
    cv.w = cells->w;
    cv.valid = 1;
  }
  const int64_t nf = h_qoff[q_begin + nq] - h_qoff[q_begin];
  if (cv.valid && nf > 0) {
    const int64_t blocks = (nf + 3) / 4;
    if (blocks >= INT32_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(scan_cells_kernel, dim3((unsigned)blocks), dim3(256), 0, s, boxes, d_qoff, q_begin, nq, cv, C,
                       d_score, d_touched, d_tcnt);
  }
  hipLaunchKernelGGL(scan_rows_kernel, dim3((nq + 3) / 4), dim3(256), 0, s, boxes, d_qoff, q_begin, nq, cv, m1s, m2s,
                     cols, R, C, d_stamp, d_score, d_touched, d_tcnt);
  hipLaunchKernelGGL(scan_final_kernel, dim3((nq + 3) / 4), dim3(256), 0, s, q_begin, nq, d_tiekey, C, d_stamp, d_score,
                     d_touched, d_tcnt, d_best);
  return hipGetLastError();
}


// ---- wide max2 windows: sweep by groups ----------------------------------------------------
//
// A coefs = 2 frame hits clip c's group of its key iff one of the group's points v lies in its
// window [L2, U2]. Within one (chunk, key) segment the frames sorted by (L2, U2) have both bounds
// non-decreasing (both are monotone functions of the frame's max2 value), so the frames a point v
// hits are one contiguous run [A(v), B(v)] (A: first U2 >= v, B: last L2 <= v), and A(v), B(v)
// grow with v: the union over the group's ascending points is a few merged runs, and a query's
// count is its frames inside them: differences of in-segment prefix counts P[i][q]. Frames
// without a max2 condition (the ignore filter dropped it) hit every group of their key: their
// own segment, counted whole. Scores go to a per-chunk [clip][query] array (lane l = queries 2l,
// 2l + 1 as one word of two 16-bit counts, one coalesced add per group), then one pass per chunk
// takes each query's best key.

namespace {

constexpr int kWideCh = WideScratch::kChunk;
constexpr int kWideSegs = 2 * kKeyRange;  // per chunk: key k with a max2 window, k | 1024 without
static_assert(kWideCh == 128, "two queries per lane");
// Per-lane counts are pairs of 16-bit counts in one word, (query 2l) | (query 2l + 1) << 16: a count
// is at most its query's frames (< 2^16), and prefix counts only grow, so the differences and sums
// below never borrow or carry across the halves.
constexpr int kWideW = kWideCh / 2;  // words per P row and per score row
constexpr int kPartWaves = 1024;     // clip-major sweep: at most this many waves per chunk

// Bad frames (a key outside the cache's range or a window outside int32: the row scan takes the
// batch) into info[1]; with uk, the U2 (offset binary: unsigned order == signed order) of each frame
// and fv = the identity, for the two-sort form.
__global__ void wide_keys_u_kernel(const FrameBox* __restrict__ boxes, int64_t nf, uint32_t* __restrict__ uk,
                                   int32_t* __restrict__ fv, int32_t* __restrict__ info) {
  int32_t nbad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nf; i += (int64_t)gridDim.x * blockDim.x) {
    const FrameBox bx = boxes[i];
    uint32_t u = 0xffffffffu;
    if (bx.flags & 1) {
      const int64_t kk = (int64_t)bx.k + kKeyOffset;
      bool bad = kk < 0 || kk >= kKeyRange;
      if (bx.flags & 2) {
        bad = bad || bx.L2 <= (int64_t)INT32_MIN || bx.L2 > (int64_t)INT32_MAX || bx.U2 < (int64_t)INT32_MIN ||
              bx.U2 > (int64_t)INT32_MAX;
        u = (uint32_t)(int32_t)bx.U2 ^ 0x80000000u;
      } else {
        u = 0;
      }
      nbad += bad;
    }
    if (uk) {
      uk[i] = u;
      fv[i] = (int32_t)i;
    }
  }
  for (int o = 32; o > 0; o >>= 1) nbad += __shfl_xor(nbad, o, 64);
  if ((threadIdx.x & 63) == 0 && nbad) atomicAdd(&info[1], nbad);
}

// fq[f] = the query of frame f (one wave per query writes its frames' entries, coalesced): the key
// and gather passes read it instead of searching qoff per frame.
// It also zeroes the counts (info) and the segment table, which the key pass and the gather fill
// (two fill launches fewer on the timeline).
// With segstat (the bin sort's): each (chunk, segment)'s frame count, least and greatest L2 start
// at 0, ~0, 0, and ghist (each chunk's fine-bin counts, nghist words) at 0.
__global__ void wide_frame_query_kernel(const int64_t* __restrict__ qoff, int32_t nq, int32_t* __restrict__ fq,
                                        int32_t* __restrict__ info, int32_t* __restrict__ seg, int64_t nseg,
                                        unsigned long long* __restrict__ best, uint32_t* __restrict__ segstat,
                                        int32_t* __restrict__ ghist, int64_t nghist) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (int64_t)gridDim.x * blockDim.x;
  if (tid < 4) info[tid] = 0;
  for (int64_t i = tid; i < nseg; i += nt) seg[i] = 0;
  if (segstat) {  // (nseg / 2 segments of 3 words)
    for (int64_t i = tid; i < 3 * (nseg / 2); i += nt) segstat[i] = i % 3 == 1 ? 0xffffffffu : 0u;
    for (int64_t i = tid; i < nghist; i += nt) ghist[i] = 0;
  }
  if (best)  // the sweep's result keys (the caller's output buffer), maxed into from zero
    for (int64_t i = tid; i < nq; i += nt) best[i] = 0ull;
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; q < nq; q += nw) {
    const int64_t b = qoff[q] - qoff[0], e = qoff[q + 1] - qoff[0];
    for (int64_t f = b + lane; f < e; f += 64) fq[f] = (int32_t)q;
  }
}

// Composite sort key of a frame: chunk << 46 | segment key << 35 | L2 << 3 | d, with d = U2 - L2 -
// dbase in [0, 8) (U2 - L2 is fmt6(q2 + tol) - fmt6(q2 - tol): within a few micro-units of 2 tol).
// One sort by it orders each (chunk, key) segment by L2, then U2. Frames that take no part get ~0
// and sort last. fv: the frame of each position (nullptr: position i is frame i). A width outside
// [dbase, dbase + 8) counts in info[2]; the caller then sorts by U2 first and passes dbase = -1
// (d = 0: that stable pre-sort orders equal L2 by U2 instead).
constexpr int kWideDeltaBits = 3, kWideSegShift = 32 + kWideDeltaBits, kWideChunkShift = kWideSegShift + 11;
// The packed layout (every window's U2 - L2 in [dbase, dbase + 8), at most 10 chunk bits): the
// frame's query within its chunk in the low byte, chunk << 54 | segment key << 43 | L2 << 11 |
// d << 8 | query; the keys alone are sorted (no frame index to carry), and the gather reads L2,
// U2 = L2 + dbase + d and the query back from the sorted key.
constexpr int kPackSegShift = 43, kPackChunkShift = kPackSegShift + 11;
__global__ void wide_keys_c_kernel(const FrameBox* __restrict__ boxes, const int32_t* __restrict__ fq,
                                   int64_t nf, int32_t qch, bool packed, const int32_t* __restrict__ fv, int64_t dbase,
                                   unsigned long long* __restrict__ ck, int32_t* __restrict__ fo,
                                   int32_t* __restrict__ info, uint32_t* __restrict__ segstat) {
  // segstat (the bin sort's): per (chunk, segment) of this workgroup's frames, in a small LDS table
  // (a workgroup takes a contiguous range: one or two chunks, a few segments), flushed with one set
  // of global atomics per entry (same-address atomics from every wave of the grid serialise: ~80 us)
  constexpr int kSlots = 128;
  __shared__ int32_t hk[kSlots];
  __shared__ uint32_t hc[kSlots], hmn[kSlots], hmx[kSlots];
  const int lane = threadIdx.x & 63;
  if (segstat) {
    for (int j = threadIdx.x; j < kSlots; j += blockDim.x) hk[j] = -1, hc[j] = 0u, hmn[j] = 0xffffffffu, hmx[j] = 0u;
    __syncthreads();
  }
  const int64_t per = (nf + gridDim.x - 1) / gridDim.x, r1 = min(nf, per * (blockIdx.x + 1));
  int32_t kept = 0, wide = 0, nbad = 0;
  // (whole waves in every step: the segment stats' shuffles read every lane)
  for (int64_t i0 = per * blockIdx.x; i0 < r1; i0 += blockDim.x) {
    const int64_t i = i0 + threadIdx.x;
    const bool in = i < r1;
    const int32_t f = !in ? 0 : fv ? fv[i] : (int32_t)i;
    FrameBox bx = in ? boxes[f] : FrameBox{};
    unsigned long long key = ~0ull;
    const int64_t kk = (int64_t)bx.k + kKeyOffset;
    // the bad-frame check of wide_keys_u (a key or a window outside what the cache and the int32
    // windows hold: the batch takes the row scan)
    if (bx.flags & 1)
      nbad += kk < 0 || kk >= kKeyRange ||
              ((bx.flags & 2) && (bx.L2 <= (int64_t)INT32_MIN || bx.L2 > (int64_t)INT32_MAX ||
                                  bx.U2 < (int64_t)INT32_MIN || bx.U2 > (int64_t)INT32_MAX));
    if ((bx.flags & 1) && kk >= 0 && kk < kKeyRange) {
      const unsigned long long ch = (unsigned long long)(fq[f] / qch);
      const bool w2 = bx.flags & 2;
      const unsigned long long sk = w2 ? (unsigned long long)kk : (unsigned long long)kk | kKeyRange;
      const unsigned long long l2 = w2 ? (unsigned long long)((uint32_t)(int32_t)bx.L2 ^ 0x80000000u) : 0ull;
      unsigned long long d = 0;
      if (w2 && dbase >= 0) {
        const int64_t dd = bx.U2 - bx.L2 - dbase;
        if (dd < 0 || dd >= (1 << kWideDeltaBits)) wide++;
        else d = (unsigned long long)dd;
      }
      key = packed ? (ch << kPackChunkShift) | (sk << kPackSegShift) | (l2 << 11) | (d << 8) |
                         (unsigned long long)(fq[f] % qch)
                   : (ch << kWideChunkShift) | (sk << kWideSegShift) | (l2 << kWideDeltaBits) | d;
      kept++;
    }
    if (in) {
      ck[i] = key;
      if (fo) fo[i] = f;
    }
    if (segstat) {
      // (the bin sort's) this frame's (chunk, segment): its count and L2 range, one set of atomics per
      // distinct (chunk, segment) of the wave (a wave's consecutive frames share a few)
      int32_t id = key != ~0ull ? (int32_t)(key >> kPackSegShift) : -1;  // chunk << 11 | segment
      const uint32_t l2 = (uint32_t)(key >> 11);
      while (true) {
        const unsigned long long m = __ballot(id >= 0);
        if (!m) break;
        const int l = __ffsll((long long)m) - 1;
        const int32_t v = __builtin_amdgcn_readlane(id, l);
        const bool me = id == v;
        const uint32_t cnt = (uint32_t)__popcll(__ballot(me));
        uint32_t mn = me ? l2 : 0xffffffffu, mx = me ? l2 : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
          mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
        }
        if (lane == l) {
          int32_t h = (int32_t)(((uint32_t)v * 2654435761u) >> 25), probes = 0;
          for (; probes < kSlots; probes++, h = (h + 1) & (kSlots - 1)) {
            const int32_t o = atomicCAS(&hk[h], -1, v);
            if (o == -1 || o == v) break;
          }
          uint32_t *c, *a, *z;
          if (probes < kSlots) {
            c = &hc[h], a = &hmn[h], z = &hmx[h];
          } else {  // (table full: straight to the global entry)
            uint32_t* st = segstat + 3 * (int64_t)v;
            c = &st[0], a = &st[1], z = &st[2];
          }
          atomicAdd(c, cnt);
          if ((v & kKeyRange) == 0) {
            atomicMin(a, mn);
            atomicMax(z, mx);
          }
        }
        if (me) id = -1;
      }
    }
  }
  if (segstat) {
    __syncthreads();
    for (int j = threadIdx.x; j < kSlots; j += blockDim.x) {
      const int32_t v = hk[j];
      if (v < 0) continue;
      uint32_t* st = segstat + 3 * (int64_t)v;
      atomicAdd(&st[0], hc[j]);
      if ((v & kKeyRange) == 0) {
        atomicMin(&st[1], hmn[j]);
        atomicMax(&st[2], hmx[j]);
      }
    }
  }
  // one atomic per block, on a grid of at most kKeysBlocks blocks: same-address atomics serialise in
  // L2 (one per frame cost ~0.13 ms at C3, and one per wave still ~0.1 ms: 10k waves)
  __shared__ int32_t red[3][256 / 64];
  for (int o = 32; o > 0; o >>= 1) {
    kept += __shfl_xor(kept, o, 64);
    wide += __shfl_xor(wide, o, 64);
    nbad += __shfl_xor(nbad, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = kept;
    red[1][threadIdx.x >> 6] = wide;
    red[2][threadIdx.x >> 6] = nbad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t k = 0, w = 0, b = 0;
    for (int i = 0; i < 256 / 64; i++) k += red[0][i], w += red[1][i], b += red[2][i];
    if (k) atomicAdd(&info[0], k);
    if (w) atomicAdd(&info[2], w);
    if (b) atomicAdd(&info[1], b);
  }
}

// Sorted frames' windows and queries; the segment table [chunk][segment key] = [begin, end).
// (n: the kept frames, info[0] of the key pass, read on the device: no host wait for the sort)
__global__ void wide_gather_kernel(const FrameBox* __restrict__ boxes, const int32_t* __restrict__ fq,
                                   const int32_t* __restrict__ pn, const unsigned long long* __restrict__ ck,
                                   const int32_t* __restrict__ fv, int32_t qch, bool packed, int64_t dbase,
                                   int32_t* __restrict__ L2s, int32_t* __restrict__ U2s, uint8_t* __restrict__ qis,
                                   int32_t* __restrict__ seg, int64_t nch, int32_t* __restrict__ cbeg) {
  const int segshift = packed ? kPackSegShift : kWideSegShift, chshift = segshift + 11;
  const int64_t n = *pn;
  if (n == 0 && blockIdx.x == 0)  // no kept frame: every chunk empty
    for (int64_t x = threadIdx.x; x <= nch; x += blockDim.x) cbeg[x] = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long k = ck[i];
    if (packed) {
      const int32_t l2 = (int32_t)((uint32_t)(k >> 11) ^ 0x80000000u);
      L2s[i] = l2;
      U2s[i] = (int32_t)(l2 + dbase + (int64_t)((k >> 8) & 7));  // (frames without a window: never read)
      qis[i] = (uint8_t)(k & 255);
    } else {
      const int32_t f = fv[i];
      const FrameBox bx = boxes[f];
      L2s[i] = (int32_t)bx.L2;
      U2s[i] = (int32_t)bx.U2;
      qis[i] = (uint8_t)(fq[f] % qch);
    }
    const unsigned long long sg = k >> segshift;  // chunk << 11 | segment key
    if (i == 0 || (ck[i - 1] >> segshift) != sg) seg[2 * sg] = (int32_t)i;
    if (i == n - 1 || (ck[i + 1] >> segshift) != sg) seg[2 * sg + 1] = (int32_t)(i + 1);
    // chunk boundaries: cbeg[c] = the first sorted frame of chunk c (n for chunks past the last
    // frame's; chunks without kept frames take the next chunk's first frame; zeroed when n = 0)
    const int64_t c = (int64_t)(k >> chshift);
    const int64_t cp = i == 0 ? -1 : (int64_t)(ck[i - 1] >> chshift);
    for (int64_t x = cp + 1; x <= c; x++) cbeg[x] = (int32_t)i;
    if (i == n - 1)
      for (int64_t x = c + 1; x <= nch; x++) cbeg[x] = (int32_t)n;
  }
}


// Segment directories. A window segment's S frames are sorted by L2 (and U2); its directory has
// NB = 2^ceil(log2 S) buckets over each bound's range: TL[b] = the first frame whose L2 >=
// L2min + (b << shift), TU[b] the same for U2 (se if none), shift the least that fits the wider
// range into NB buckets. A point v's first U2 >= v and first L2 > v then lie inside one bucket's
// [T[b], T[b + 1]] (b = v's bucket): one table load and a search over the bucket's few frames,
// instead of a search over the whole segment.
#ifndef TFP_DIR_SCALE
#define TFP_DIR_SCALE 0
#endif
// NB = 2^(ceil(log2 S) + kDirScale): 0 since round 5 (C3 coefs=2 at tol 0.001 / 0.45: 0.804 / 0.926
// ms against 0.810 / 0.936 with 1 and 0.827 / 0.955 with 2, profiles/r05/c3_dirscale_r05h.txt;
// the fill's scattered writes shrink 4x, the sweep's bucket searches grow by about one step)
constexpr int kDirScale = TFP_DIR_SCALE;
__device__ __forceinline__ int dir_log2(int32_t S) { return (S <= 1 ? 0 : 32 - __clz(S - 1)) + kDirScale; }
__device__ __forceinline__ int dir_shift(int64_t range, int lg) {
  const int bits = range > 0 ? 64 - __clzll((unsigned long long)range) : 0;
  return bits > lg ? bits - lg : 0;
}


// Directory offsets in one workgroup: doff[t] = the exclusive prefix of the directory sizes
// (2 NB per window segment of S frames, 0 when empty) over the nch * kKeyRange window segments,
// doff[nch * kKeyRange] their total (one launch instead of a size pass and a device-wide scan). In
// rounds of 16,384 segments: the sizes loaded coalesced into LDS, each thread scans 16 consecutive
// ones, one LDS scan over the threads' sums, the offsets written coalesced.
__global__ __launch_bounds__(1024) void wide_dir_offsets_kernel(const int32_t* __restrict__ seg, int64_t nch,
                                                                int32_t* __restrict__ doff) {
  constexpr int kPer = 16, kRound = 1024 * kPer;
  __shared__ int32_t sz[kRound];
  __shared__ int32_t tsum[1024];
  const int t = threadIdx.x;
  const int64_t nseg = nch * kKeyRange;
  int32_t carry = 0;
  for (int64_t base = 0; base < nseg; base += kRound) {
#pragma unroll
    for (int j = 0; j < kPer; j++) {  // coalesced: consecutive threads, consecutive segments
      const int64_t g = base + j * 1024 + t;
      int32_t v = 0;
      if (g < nseg) {
        const int32_t* sg = seg + (g / kKeyRange) * kWideSegs * 2 + 2 * (g % kKeyRange);
        const int32_t S = sg[1] - sg[0];
        v = S > 0 ? 2 << dir_log2(S) : 0;
      }
      sz[j * 1024 + t] = v;
    }
    __syncthreads();
    int32_t sum = 0;
#pragma unroll
    for (int j = 0; j < kPer; j++) {  // this thread's 16 consecutive sizes -> exclusive prefix
      const int32_t v = sz[t * kPer + j];
      sz[t * kPer + j] = sum;
      sum += v;
    }
    tsum[t] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan of the thread sums
      const int32_t y = t >= o ? tsum[t - o] : 0;
      __syncthreads();
      tsum[t] += y;
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < kPer; j++) {
      const int i = j * 1024 + t;
      const int64_t g = base + i;
      const int owner = i / kPer;
      if (g < nseg) doff[g] = carry + (owner ? tsum[owner - 1] : 0) + sz[i];
    }
    carry += tsum[1023];
    __syncthreads();  // (the next round rewrites sz and tsum)
  }
  if (t == 0) doff[nseg] = carry;
}

// Every lane's runs written: runs up to kLane buckets by their own lane (above 8: dwords to a
// 16-byte boundary, then 16-byte stores: a sparse stretch of the value range gives a wave of 64 runs of
// tens to hundreds of buckets), longer ones (e.g. the gap below a silence-floor crowd: up to a whole
// directory) by the whole wave, 256 buckets a step. dtab 16-byte aligned. (Call with every lane.)
__device__ __forceinline__ int64_t dir_write(int32_t* __restrict__ dtab, const int32_t (&lo)[4], const int32_t (&hi)[4],
                                             const int32_t (&val)[4], const int32_t (&base)[4], int lane) {
  constexpr int32_t kLane = 256;
  int64_t nlong = 0;  // (the buckets of runs above 8: TFP_BIN_CLOCKS)
  int4* d4 = reinterpret_cast<int4*>(dtab);
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int32_t len = hi[r] - lo[r] + 1;
    if (len > 0 && len <= 8)
      for (int32_t b = lo[r]; b <= hi[r]; b++) dtab[base[r] + b] = val[r];
    if (__ballot(len > 8 && len <= kLane) && len > 8 && len <= kLane) {
      const int32_t v = val[r];
      const int64_t e = (int64_t)base[r] + hi[r] + 1;
      int64_t q = (int64_t)base[r] + lo[r];
      for (; q < e && (q & 3); q++) dtab[q] = v;
      for (const int4 v4 = make_int4(v, v, v, v); q + 4 <= e; q += 4) d4[q >> 2] = v4;
      for (; q < e; q++) dtab[q] = v;
      nlong += len;
    }
    unsigned long long m = __ballot(len > kLane);
    while (m) {
      const int l = __ffsll((long long)m) - 1;
      m &= m - 1;
      const int32_t a = __builtin_amdgcn_readlane(lo[r], l), z = __builtin_amdgcn_readlane(hi[r], l),
                    v = __builtin_amdgcn_readlane(val[r], l), o = __builtin_amdgcn_readlane(base[r], l);
      // [s, e) absolute: its unaligned head and tail (< 4 each) by lanes, the rest as int4
      const int64_t s = (int64_t)o + a, e = (int64_t)o + z + 1, s4 = (s + 3) & ~3ll, e4 = e & ~3ll;
      if (lane < s4 - s) dtab[s + lane] = v;
      if (lane < e - e4) dtab[e4 + lane] = v;
      const int4 v4 = make_int4(v, v, v, v);
      for (int64_t b = s4 / 4 + lane; b < e4 / 4; b += 64) d4[b] = v4;
      nlong += e - s;
    }
  }
  return nlong;
}
// The directories, from the sorted frames: frame i of a window segment is the first frame of the
// buckets after its predecessor's bucket up to its own (each bucket written once), the last frame
// also fills the buckets after its own with se; the first writes the segment's constants (segk).
// The runs through dir_write (a long one, a sparse stretch of the value range, by the whole wave:
// no lane loops over thousands of buckets alone).
__global__ void wide_dir_fill_kernel(const int32_t* __restrict__ pn, const unsigned long long* __restrict__ ck,
                                     int segshift, const int32_t* __restrict__ seg, const int32_t* __restrict__ L2s,
                                     const int32_t* __restrict__ U2s, const int32_t* __restrict__ doff,
                                     int32_t* __restrict__ dtab, int4* __restrict__ segk) {
  const int64_t n = *pn;
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i0 = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64; i0 < n; i0 += nw * 64) {
    const int64_t i = i0 + lane;
    // this lane's runs: [lo, hi] of table entries at base + (lo..hi), value v (up to 4: L2, U2, tails)
    int32_t lo[4] = {1, 1, 1, 1}, hi[4] = {0, 0, 0, 0}, val[4] = {0, 0, 0, 0}, base[4] = {0, 0, 0, 0};
    if (i < n) {
      // this frame's and its predecessor's bounds requested with the key (they depend on i only)
      const int32_t xl = L2s[i], xu = U2s[i], xlp = i > 0 ? L2s[i - 1] : 0, xup = i > 0 ? U2s[i - 1] : 0;
      const unsigned long long sgk = ck[i] >> segshift;  // chunk << 11 | segment key
      const int32_t skey = (int32_t)(sgk & (kWideSegs - 1));
      if (skey < kKeyRange) {  // (no max2 window: no searches, no directory)
        const int64_t ch = (int64_t)(sgk >> 11);
        const int32_t sb = seg[2 * sgk], se = seg[2 * sgk + 1];
        const int lg = dir_log2(se - sb);
        const int32_t nbk = 1 << lg;
        const int32_t l2min = L2s[sb], u2min = U2s[sb];
        const int shf = dir_shift(max((int64_t)L2s[se - 1] - l2min, (int64_t)U2s[se - 1] - u2min), lg);
        const int32_t t0 = doff[ch * kKeyRange + skey];
        if (i == sb) segk[ch * kKeyRange + skey] = make_int4(l2min, u2min, shf, t0);  // (wide_clips' constants)
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const int64_t mn = h ? u2min : l2min;
          const int32_t bi = (int32_t)(((int64_t)(h ? xu : xl) - mn) >> shf);
          const int32_t bp = i == sb ? -1 : (int32_t)(((int64_t)(h ? xup : xlp) - mn) >> shf);
          base[h] = base[2 + h] = t0 + h * nbk;
          lo[h] = bp + 1, hi[h] = bi, val[h] = (int32_t)i;
          if (i == se - 1) lo[2 + h] = bi + 1, hi[2 + h] = nbk - 1, val[2 + h] = se;
        }
      }
    }
    (void)dir_write(dtab, lo, hi, val, base, lane);
  }
}

// ---- the sweep's frame order, sorted by bins (round 5) ---------------------------------------
// The packed keys of a chunk (seg << 43 | L2 << 11 | d << 8 | query) are ordered without a
// device-wide sort. A chunk's frames are contiguous in the input, and the key pass counts each
// (chunk, segment)'s frames and L2 range (segstat). Each segment then gets nb = 2^ceil(log2(S / 8))
// bins (one without a max2 window) cut evenly over its L2 range: a bin index is monotone in the
// key, and bins hold ~8 frames where the values spread evenly. wide_bin_hist counts the bins of
// each chunk (workgroups over slices of the chunk: per-workgroup counts in LDS, one global atomic
// per bin, which also hands the workgroup its offset in the bin) and records each frame's bin and
// place in it; wide_bin_scan (a workgroup per chunk) scans the counts into each bin's first frame
// and writes the segment table, the directory offsets, the used keys and the non-empty bins;
// wide_bin_scatter moves the keys to their places; one wave sorts each bin in registers or LDS
// and writes the sorted windows, queries and segment of each frame and the directory runs of its
// window segment (wide_bin_sort, with wide_bin_scan's per-segment constants, segk).
// Chunk ch's kept frames occupy [cbeg[ch], cbeg[ch] + kept) of the sorted arrays; the rest of its
// input range holds no frame of a segment (query 0), so the prefix counts run over the
// whole range. A bin whose frames all share (segment, L2, d), or whose segment has no max2 window,
// is not sorted (any order counts the same). Any other bin above kBinCap frames sets info[2],
// which sends the speculative batch to the library sort (as a window width outside the key's delta
// field does).
constexpr int kNFine = 16384;        // bins per chunk at most (the per-segment counts halve until they fit)
#ifndef TFP_BINSORT_REVERSE
#define TFP_BINSORT_REVERSE 1
#endif
#ifndef TFP_BIN_CLOCKS
#define TFP_BIN_CLOCKS 0
#endif
constexpr int kBinCap = 512;         // frames one wave sorts in LDS (16 KB a workgroup: 8 workgroups a CU)
constexpr int kBinSortWaves = 4;     // waves per wide_bin_sort workgroup
constexpr int kGroup = 64;           // a sort group: the bins whose first frame lies in [64 g, 64 g + 64)
constexpr int kHistPer = 2;          // frames per thread of wide_bin_hist (1024 threads)
constexpr int kPlaceBits = 18;       // place of a frame in its bin (chunks of at most 2^18 frames)

// exclusive prefix of v over the workgroup (NT threads), and the total
template <int NT>
__device__ __forceinline__ int32_t block_excl(int32_t v, int32_t* ws, int32_t& total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) ws[w] = x;
  __syncthreads();
  int32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) {
    const int32_t y = ws[i];
    off += i < w ? y : 0;
    tot += y;
  }
  __syncthreads();  // (ws is reused by the next call)
  total = tot;
  return off + x - v;
}

// The chunk's bin layout from segstat, in LDS (one workgroup of NT threads, 2 segments a thread):
// base[s], nb[s] (0: unused), shift[s], l2min[s]; returns the chunk's bins. Synchronises.
template <int NT>
__device__ int32_t bin_layout(const uint32_t* __restrict__ st, int32_t* base, int32_t* nbs, int32_t* shf, uint32_t* lmn,
                              int32_t* ws) {
  static_assert(NT * 2 == kWideSegs, "two segments a thread");
  const int t = threadIdx.x;
  uint32_t cnt[2], lo[2], hi[2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const int sk = 2 * t + j;
    cnt[j] = st[3 * sk];
    lo[j] = st[3 * sk + 1];
    hi[j] = st[3 * sk + 2];
  }
  int32_t total = 0, off = 0;
  for (int extra = 3;; extra++) {  // ~2^extra frames a bin, coarser until the chunk's bins fit
    int32_t n[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int sk = 2 * t + j;
      const uint32_t per = (cnt[j] + (1u << extra) - 1) >> extra;
      n[j] = cnt[j] == 0 ? 0 : (sk >= kKeyRange || per <= 1) ? 1 : 1 << (32 - __clz(per - 1));
    }
    off = block_excl<NT>(n[0] + n[1], ws, total);
    if (total <= kNFine) {
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const int sk = 2 * t + j;
        const uint32_t range = hi[j] >= lo[j] ? hi[j] - lo[j] : 0u;
        const int32_t rb = range ? 32 - __clz(range) : 0, lg = n[j] ? 31 - __clz(n[j]) : 0;
        base[sk] = off;
        nbs[sk] = n[j];
        shf[sk] = rb > lg ? rb - lg : 0;
        lmn[sk] = sk < kKeyRange ? lo[j] : 0u;
        off += n[j];
      }
      break;
    }
  }
  __syncthreads();
  return total;
}
__device__ __forceinline__ int32_t bin_of(unsigned long long key, const int32_t* base, const int32_t* shf, const uint32_t* lmn) {
  const int sk = (int)(key >> kPackSegShift) & (kWideSegs - 1);
  return base[sk] + (sk < kKeyRange ? (int32_t)(((uint32_t)(key >> 11) - lmn[sk]) >> shf[sk]) : 0);
}

// Workgroup (ch, j): frames [cb + 2048 j, cb + 2048 (j + 1)) of chunk ch. Per bin in LDS: the
// workgroup's count (the count before a frame's add is its place among them), then one global
// atomic per non-empty bin (the workgroup's offset in the bin); each frame's bin << 18 | place in
// pos (~0: not kept; chunks under 2^18 frames, so no kept frame's word is ~0).
__global__ __launch_bounds__(1024) void wide_bin_hist_kernel(const int64_t* __restrict__ qoff, int32_t nq, int32_t qch,
                                                             const unsigned long long* __restrict__ ka,
                                                             const uint32_t* __restrict__ segstat, int32_t* __restrict__ ghist,
                                                             uint32_t* __restrict__ pos) {
  constexpr int NT = 1024;
  __shared__ int32_t base[kWideSegs], nbs[kWideSegs], shf[kWideSegs], ws[NT / 64];
  __shared__ uint32_t lmn[kWideSegs];
  __shared__ int32_t h[kNFine];
  const int t = threadIdx.x, ch = blockIdx.x;
  const int32_t q0 = ch * qch, q1 = min(nq, q0 + qch);
  const int64_t cb = qoff[q0] - qoff[0], ce = qoff[q1] - qoff[0];
  const int64_t b0 = cb + (int64_t)blockIdx.y * (NT * kHistPer);
  if (b0 >= ce) return;  // (uniform in the workgroup)
  for (int b = t; b < kNFine; b += NT) h[b] = 0;
  (void)bin_layout<NT>(segstat + (int64_t)ch * kWideSegs * 3, base, nbs, shf, lmn, ws);  // (synchronises)
  unsigned long long k[kHistPer];
  int32_t bin[kHistPer], rk[kHistPer];
#pragma unroll
  for (int j = 0; j < kHistPer; j++) {
    const int64_t i = b0 + j * NT + t;
    k[j] = i < ce ? ka[i] : ~0ull;
  }
#pragma unroll
  for (int j = 0; j < kHistPer; j++) {
    bin[j] = k[j] != ~0ull ? bin_of(k[j], base, shf, lmn) : -1;
    rk[j] = bin[j] >= 0 ? atomicAdd(&h[bin[j]], 1) : 0;
  }
  __syncthreads();
  for (int b = t; b < kNFine; b += NT) {
    const int32_t n = h[b];
    if (n) h[b] = atomicAdd(&ghist[(int64_t)ch * kNFine + b], n);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kHistPer; j++) {
    const int64_t i = b0 + j * NT + t;
    if (i < ce) pos[i] = bin[j] >= 0 ? ((uint32_t)bin[j] << kPlaceBits) | (uint32_t)(h[bin[j]] + rk[j]) : ~0u;
  }
}

// One workgroup per chunk: the bin counts scanned into each bin's first frame (bstart, relative to
// cbeg[ch]), the sort groups (gi4, gb: wide_bin_sort), the segment table, the directory offsets
// (in segk; chunk ch's directories at (4 << kDirScale) cbeg[ch]: 2 NB <= (4 << kDirScale) S per segment,
// the table's size per frame), each window segment's directory constants (segk: {min L2, min U2 =
// min L2 + dbase, bucket shift over the L2 range + 7, directory offset}), the used keys, the
// chunk's tail of non-frames, and cbeg.
__global__ __launch_bounds__(1024) void wide_bin_scan_kernel(const int64_t* __restrict__ qoff, int32_t nq, int32_t qch,
                                                             int32_t nch, const uint32_t* __restrict__ segstat,
                                                             const int32_t* __restrict__ ghist, int32_t* __restrict__ bstart,
                                                             int32_t* __restrict__ seg, int32_t* __restrict__ ukeys, int32_t* __restrict__ nuk,
                                                             int32_t* __restrict__ cbeg, uint8_t* __restrict__ qis,
                                                             int4* __restrict__ gi4,
                                                             int32_t* __restrict__ gb, int32_t gcap, int64_t dbase,
                                                             int4* __restrict__ segk) {
  constexpr int NT = 1024, FPER = kNFine / NT;
  __shared__ int32_t base[kWideSegs], nbs[kWideSegs], shf[kWideSegs], ws[NT / 64];
  __shared__ uint32_t lmn[kWideSegs];
  __shared__ int32_t start[kNFine + 1];
  __shared__ int32_t used[kKeyRange];
  const int t = threadIdx.x, ch = blockIdx.x;
  const int32_t q0 = ch * qch, q1 = min(nq, q0 + qch);
  const int64_t cb = qoff[q0] - qoff[0], ce = qoff[q1] - qoff[0];
  used[t] = 0;
  (void)bin_layout<NT>(segstat + (int64_t)ch * kWideSegs * 3, base, nbs, shf, lmn, ws);  // (synchronises)
  int32_t g[FPER], sum = 0;
#pragma unroll
  for (int j = 0; j < FPER; j++) {
    g[j] = ghist[(int64_t)ch * kNFine + FPER * t + j];
    sum += g[j];
  }
  int32_t T;
  int32_t st = block_excl<NT>(sum, ws, T);
  int32_t* bs = bstart + (int64_t)ch * (kNFine + 1);
#pragma unroll
  for (int j = 0; j < FPER; j++) {
    const int f = FPER * t + j;
    bs[f] = st;
    start[f] = st;
    st += g[j];
  }
  if (t == 0) {
    bs[kNFine] = T;
    start[kNFine] = T;
    cbeg[ch] = (int32_t)cb;
    if (ch == nch - 1) cbeg[nch] = (int32_t)ce;
  }
  __syncthreads();
  // segments: segment sk's bins [base, base + nb)
  int32_t dv[2] = {0, 0}, ns[2] = {0, 0};
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const int sk = 2 * t + j;
    if (nbs[sk]) {
      const int32_t b = start[base[sk]], e = start[base[sk] + nbs[sk]];
      if (e > b) {
        int32_t* sg = seg + ((int64_t)ch * kWideSegs + sk) * 2;
        sg[0] = (int32_t)cb + b;
        sg[1] = (int32_t)cb + e;
        used[sk & (kKeyRange - 1)] = 1;
        if (sk < kKeyRange) dv[j] = 2 << dir_log2(e - b), ns[j] = e - b;  // (the directory's entries)
      }
    }
  }
  int32_t DT;
  int32_t dof = block_excl<NT>(dv[0] + dv[1], ws, DT);  // (synchronises: used is complete)
  (void)DT;
#pragma unroll
  for (int j = 0; j < 2; j++) {
    if (dv[j]) {
      const int sk = 2 * t + j;
      const int32_t o = (4 << kDirScale) * (int32_t)cb + dof;
      const uint32_t* sst = segstat + ((int64_t)ch * kWideSegs + sk) * 3;
      const uint32_t lo = sst[1], hi = sst[2];
      const int32_t l2min = (int32_t)(lo ^ 0x80000000u);
      // (U2 min beyond int32: such frames are out of range, info[1], and the batch is redone)
      const int64_t u2min = min((int64_t)l2min + dbase, (int64_t)INT32_MAX);
      segk[(int64_t)ch * kKeyRange + sk] = make_int4(l2min, (int32_t)u2min, dir_shift((int64_t)(hi - lo) + 7, dir_log2(ns[j])), o);
    }
    dof += dv[j];
  }
  // the used keys, ascending
  int32_t NU;
  const int32_t uo = block_excl<NT>(used[t], ws, NU);
  if (used[t]) ukeys[(int64_t)ch * kKeyRange + uo] = t;
  if (t == 0) nuk[ch] = NU;
  // sort groups (wide_bin_sort): group g starts at the first bin whose first frame is >= kGroup g
  // (the bin holding frame kGroup g, or the next one). gi4[g] = {its first frame, the next group's,
  // the first frame and size of the bin holding frame kGroup g}; gb[g] = its first bin. Groups from
  // ceil(T / kGroup) on hold nothing ({T, T, 0, 0}).
  for (int32_t gi = t; gi < gcap; gi += NT) {
    const int32_t p = gi * kGroup, q = p + kGroup;
    int32_t a = T, z = T, f = kNFine, hs = 0, hn = 0;
    auto last_at = [&](int32_t x) {  // the last bin starting at or before x < T (non-empty: start[kNFine] = T > x)
      int32_t lo = 0, hi = kNFine;
      while (hi - lo > 1) {
        const int32_t mid = (lo + hi) >> 1;
        if (start[mid] <= x) lo = mid; else hi = mid;
      }
      return lo;
    };
    if (p < T) {
      const int32_t lo = last_at(p);
      f = start[lo] == p ? lo : lo + 1;
      a = start[f];
      hs = start[lo];
      hn = start[lo + 1] - hs;
      if (q < T) {
        const int32_t l2 = last_at(q);
        z = start[start[l2] == q ? l2 : l2 + 1];
      }
    }
    gi4[(int64_t)ch * gcap + gi] = make_int4(a, z, hs, hn);
    gb[(int64_t)ch * gcap + gi] = f;
  }
  // the range's tail (no kept frame): query 0
  for (int64_t i = cb + T + t; i < ce; i += NT) qis[i] = 0;
}

// Each kept frame's key to its bin's place: kb[cbeg[ch] + bstart[ch][bin] + place].
__global__ void wide_bin_scatter_kernel(int64_t nf, int32_t qch, const int32_t* __restrict__ fq,
                                        const unsigned long long* __restrict__ ka, const uint32_t* __restrict__ pos,
                                        const int32_t* __restrict__ cbeg, const int32_t* __restrict__ bstart,
                                        unsigned long long* __restrict__ kb) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nf; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t p = pos[i];
    if (p == ~0u) continue;
    const int ch = fq[i] / qch;
    kb[(int64_t)cbeg[ch] + bstart[(int64_t)ch * (kNFine + 1) + (p >> kPlaceBits)] + (p & ((1u << kPlaceBits) - 1))] = ka[i];
  }
}

__device__ __forceinline__ unsigned long long shfl_up_u64(unsigned long long v, int d) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, 64), hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {  // (l wave-uniform)
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l),
                 hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((unsigned long long)hi << 32) | lo;
}
// ascending bitonic sort of R keys per lane in registers (element i = lane + 64 r is v[r]): the
// stages with j >= 64 pair registers of one lane, the others lanes (shuffles)
template <int R>
__device__ __forceinline__ void bitonic_regs(unsigned long long (&v)[R], int lane) {
#pragma unroll
  for (int k = 2; k <= 64 * R; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int q = r ^ (j / 64);
          if (q > r) {  // (i = lane + 64 r, partner lane + 64 q: ascending when (i & k) == 0)
            const bool up = ((64 * r) & k) == 0;
            const unsigned long long a = v[r], b = v[q];
            v[r] = (a < b) == up ? a : b;
            v[q] = (a < b) == up ? b : a;
          }
        }
      } else {
        const bool lower = (lane & j) == 0;
#pragma unroll
        for (int r = 0; r < R; r++) {
          const unsigned long long o = shfl_xor_u64(v[r], j);
          const bool up = ((lane + 64 * r) & k) == 0;
          v[r] = lower == up ? (o < v[r] ? o : v[r]) : (o > v[r] ? o : v[r]);
        }
      }
    }
}
// ascending bitonic sort of S[0, N) (N a power of two, 128 .. kBinCap) by one wave in LDS (a
// wave's LDS operations complete in order: no barrier between the stages)
__device__ void bitonic_lds(unsigned long long* S, int N, int lane) {
  for (int k = 2; k <= N; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1)
      for (int t = lane; t < N / 2; t += 64) {
        const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), ip = i | j;
        const unsigned long long a = S[i], b = S[ip];
        if ((a > b) == ((i & k) == 0)) {
          S[i] = b;
          S[ip] = a;
        }
      }
}

// A window segment's directory runs for one sorted frame (wide_dir_fill's rule): frame i at
// absolute position pos writes the L2 and U2 buckets after its predecessor's (key kp; none at the
// segment's first frame) up to its own, and the segment's last frame also the buckets after its
// own (value se). sk4 = {l2min, u2min, shift, directory offset} of the segment (segk), sb / se its
// bounds. A U2 bucket is (U2 - u2min) >> shift with u2min = l2min + dbase, i.e. (L2 - l2min + d)
// >> shift: formed without dbase, it stays inside the directory even for a batch whose U2 leaves
// int32 (info[1]: redone). Returns the runs in lo / hi / val / base (empty: lo > hi).
__device__ __forceinline__ void dir_runs(int64_t pos, unsigned long long k, unsigned long long kp, int4 sk4, int32_t sb,
                                         int32_t se, int32_t (&lo)[4], int32_t (&hi)[4], int32_t (&val)[4],
                                         int32_t (&base)[4]) {
  const int64_t l2 = (int32_t)((uint32_t)(k >> 11) ^ 0x80000000u), lp = (int32_t)((uint32_t)(kp >> 11) ^ 0x80000000u);
  const int64_t dl = l2 - sk4.x, dp = lp - sk4.x;
  const int lg = dir_log2(se - sb);
  const int32_t nbk = 1 << lg;
  const int32_t bi = (int32_t)(dl >> sk4.z), bu = (int32_t)((dl + (int64_t)((k >> 8) & 7)) >> sk4.z);
  const bool first = pos == sb;
  const int32_t bp = first ? -1 : (int32_t)(dp >> sk4.z), bq = first ? -1 : (int32_t)((dp + (int64_t)((kp >> 8) & 7)) >> sk4.z);
  base[0] = base[2] = sk4.w;
  base[1] = base[3] = sk4.w + nbk;
  lo[0] = bp + 1, hi[0] = bi, val[0] = (int32_t)pos;
  lo[1] = bq + 1, hi[1] = bu, val[1] = (int32_t)pos;
  if (pos == se - 1) {
    lo[2] = bi + 1, hi[2] = nbk - 1, val[2] = se;
    lo[3] = bu + 1, hi[3] = nbk - 1, val[3] = se;
  }
}

// Sort groups: group g of a chunk is the run of bins whose first frame lies in [64 g, 64 g + 64)
// (bins are monotone in the key, so sorting a run of whole bins sorts each of them): frames
// [gi4[g].x, gi4[g].y) of the chunk, bins [gb[g], gb[g + 1]). One wave per group sorts it in
// registers (up to 256 frames, 4 a lane) or LDS, and writes each sorted frame's L2, U2 (= L2 +
// dbase + d) and query, and its window segment's directory runs (the frame before the
// group: the greatest key of the group before it). A group above kBinCap frames (a crowded bin)
// goes bin by bin: a bin whose frames all share (segment, L2, d), or whose segment has no max2
// window, needs no order, and the waves of its 64-frame windows copy it; any other bin above
// kBinCap frames sets info[2] (the batch is redone with the library sort).
__global__ __launch_bounds__(64 * kBinSortWaves) void wide_bin_sort_kernel(
    const int32_t* __restrict__ bstart, const int4* __restrict__ gi4, const int32_t* __restrict__ gb, int32_t gcap,
    const int32_t* __restrict__ cbeg, const unsigned long long* __restrict__ kb, int64_t dbase,
    const int32_t* __restrict__ seg, const int4* __restrict__ segk, int32_t* __restrict__ L2s, int32_t* __restrict__ U2s,
    uint8_t* __restrict__ qis, int32_t* __restrict__ dtab, int32_t* __restrict__ info, long long* __restrict__ wclk) {
  __shared__ unsigned long long sk[kBinSortWaves][kBinCap];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ch = blockIdx.x;
#if TFP_BINSORT_REVERSE
  // groups in descending order of dispatch: a chunk's last groups, where the silence-floor crowd
  // sorts (the longest waves), start first instead of last
  const int32_t g = (gridDim.y - 1 - blockIdx.y) * kBinSortWaves + wv;
#else
  const int32_t g = blockIdx.y * kBinSortWaves + wv;
#endif
  const int32_t* bs = bstart + (int64_t)ch * (kNFine + 1);
  if (g + 1 >= gcap) return;  // (wave-uniform)
#if TFP_BIN_CLOCKS
  // (a diagnostic build, -DTFP_BIN_CLOCKS=1 with TFP_DEBUG_BINS: each wave's clock cycles in
  // wclk[ch][g][8]: the whole wave, the key before the group, the first crowd copy, the directory
  // stores, the LDS sorts, the register sorts, the crowded-group loop; and the long runs' buckets)
  struct WaveClock {
    long long* w;
    long long t0;
    int lane;
    long long c[8];
    __device__ ~WaveClock() {
      if (w && lane == 0) {
        w[0] = clock64() - t0;
        for (int i = 1; i < 8; i++) w[i] = c[i];
      }
    }
  } wave_clock{wclk ? wclk + ((int64_t)ch * gcap + g) * 8 : nullptr, clock64(), lane, {}};
#define BCLK(i, ...)                                 \
  do {                                               \
    const long long t_ = clock64();                  \
    __VA_ARGS__;                                     \
    wave_clock.c[i] += clock64() - t_;               \
  } while (0)
#define BCLK_BEGIN(i) const long long t_##i = clock64()
#define BCLK_END(i) wave_clock.c[i] += clock64() - t_##i
#else
#define BCLK_BEGIN(i) (void)0
#define BCLK_END(i) (void)0
#define BCLK(i, ...) \
  do {               \
    __VA_ARGS__;     \
  } while (0)
#endif
  const int4 gq = gi4[(int64_t)ch * gcap + g];
  const int32_t S0 = gq.x, S1 = gq.y;
  const int64_t cb = cbeg[ch];
  unsigned long long* S = sk[wv];
  auto sk_of = [](unsigned long long k) { return (int32_t)((k >> kPackSegShift) & (kWideSegs - 1)); };
  // the key before the group in sorted order: the greatest of the bin before S0 (kb is unsorted:
  // its greatest over a range holding that whole bin, whose keys exceed those of the bins before
  // it). That bin is the previous group's last (at most kBinCap frames from S0 on) or, when that
  // group is empty, the one holding frame 64 (g - 1); a bin above kBinCap frames is a crowd of one
  // value or has no max2 window (no directory), so any of its keys will do. None at the chunk start
  // (S0 > 0 has g > 0: group 0 starts at frame 0).
  unsigned long long kprev = 0;
  BCLK_BEGIN(1);
  if (S0 > 0 && S0 < S1) {
    const int4 gr = gi4[(int64_t)ch * gcap + g - 1];
    const int32_t lo = gr.x < S0 ? max(gr.x, S0 - kBinCap) : gr.w > kBinCap ? S0 - 1 : gr.z;
    for (int32_t p = lo + lane; p < S0; p += 64) {
      const unsigned long long k = kb[cb + p];
      kprev = k > kprev ? k : kprev;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long y = shfl_xor_u64(kprev, o);
      kprev = y > kprev ? y : kprev;
    }
  }
  BCLK_END(1);
  // sorted frame p (chunk-relative) of key k after key kp: its outputs and directory runs (valid:
  // this lane has a frame; every lane calls)
  auto put = [&](int32_t p, unsigned long long k, unsigned long long kp, bool valid) {
    int32_t lo[4] = {1, 1, 1, 1}, hi[4] = {0, 0, 0, 0}, val[4] = {0, 0, 0, 0}, base[4] = {0, 0, 0, 0};
    if (valid) {
      const int64_t pos = cb + p;
      const int32_t l2 = (int32_t)((uint32_t)(k >> 11) ^ 0x80000000u), sgk = sk_of(k);
      L2s[pos] = l2;
      U2s[pos] = (int32_t)(l2 + dbase + (int64_t)((k >> 8) & 7));
      qis[pos] = (uint8_t)(k & 255);
      if (sgk < kKeyRange) {
        const int32_t* sg = seg + ((int64_t)ch * kWideSegs + sgk) * 2;
        dir_runs(pos, k, kp, segk[(int64_t)ch * kKeyRange + sgk], sg[0], sg[1], lo, hi, val, base);
      }
    }
#if TFP_BIN_CLOCKS
    BCLK(3, wave_clock.c[7] += dir_write(dtab, lo, hi, val, base, lane));
#else
    (void)dir_write(dtab, lo, hi, val, base, lane);
#endif
  };
  // frames [b, b + n) sorted in LDS, written (kp: the key before them); returns their last key
  auto sort_lds = [&](int32_t b, int32_t n, unsigned long long kp) {
    const int N = n <= 1 ? 1 : 1 << (32 - __clz(n - 1));
    for (int p = lane; p < N; p += 64) S[p] = p < n ? kb[cb + b + p] : ~0ull;
    bitonic_lds(S, N, lane);
    for (int p0 = 0; p0 < n; p0 += 64) {
      const int p = p0 + lane;
      put(b + p, p < n ? S[p] : 0ull, p == 0 ? kp : S[p > 0 ? p - 1 : 0], p < n);
    }
    return S[n - 1];
  };
  // frames [p0, p1) of big bin [b, b + nb), unsorted (kp: the key before the bin): a frame whose
  // (segment, L2, d) differs from the bin's first in a window segment sends the batch to the
  // library sort
  auto copy_big = [&](int32_t b, int32_t nb, int32_t p0, int32_t p1, unsigned long long kp) {
    const unsigned long long k0 = kb[cb + b];
    bool odd = false;
    for (int32_t q0 = p0; q0 < p1; q0 += 64) {
      const int32_t p = q0 + lane;
      const unsigned long long k = p < p1 ? kb[cb + p] : k0;
      put(p, k, p == b ? kp : k0, p < p1);
      odd = odd || ((k >> 8) != (k0 >> 8) && sk_of(k0) < kKeyRange);
    }
    if (__ballot(odd) && lane == 0) atomicAdd(&info[2], 1);
  };
  // frames 64 g .. 64 g + 63 of a bin above kBinCap that holds frame 64 g (no order needed, or the
  // batch is redone): each wave copies and checks its own (a bin starting at 64 g is this group's
  // first: its predecessor is kprev), the wave of the bin's group those before the bin's first
  // multiple of 64
  if (gq.w > kBinCap) BCLK(2, copy_big(gq.z, gq.w, max(g * kGroup, gq.z), min(g * kGroup + kGroup, gq.z + gq.w), kprev));
  const int32_t n = S1 - S0;
  if (n <= 0) return;
  // n <= 64 R: R keys a lane, sorted in registers; each frame's predecessor through the lanes
  auto sort_regs = [&](auto rr) {
    constexpr int R = decltype(rr)::value;
    unsigned long long v[R];
#pragma unroll
    for (int r = 0; r < R; r++) v[r] = 64 * r + lane < n ? kb[cb + S0 + 64 * r + lane] : ~0ull;
    bitonic_regs<R>(v, lane);
    unsigned long long pv[R];
#pragma unroll
    for (int r = 0; r < R; r++) {  // (every lane: the shuffles read whole rows)
      const unsigned long long up = shfl_up_u64(v[r], 1), last = readlane_u64(v[r > 0 ? r - 1 : 0], 63);
      pv[r] = lane ? up : r ? last : kprev;
    }
#pragma unroll
    for (int r = 0; r < R; r++) put(S0 + 64 * r + lane, v[r], pv[r], 64 * r + lane < n);
  };
  if (n <= 64) {
    BCLK(5, sort_regs(std::integral_constant<int, 1>{}));
    return;
  }
  if (n <= 128) {
    BCLK(5, sort_regs(std::integral_constant<int, 2>{}));
    return;
  }
  if (n <= 256) {
    BCLK(5, sort_regs(std::integral_constant<int, 4>{}));
    return;
  }
  if (n <= kBinCap) {
    BCLK(4, (void)sort_lds(S0, n, kprev));
    return;
  }
  // a crowded group: its bins 64 at a time, runs of small bins (contiguous frames, ascending keys)
  // sorted together up to kBinCap frames, a crowd bin copied
  unsigned long long klast = kprev;
  const int32_t fa = gb[(int64_t)ch * gcap + g];
  // the group's bins end at the first bin starting at or after S1 (the rest are empty: the last
  // group's range runs to kNFine, thousands of empty bins past a silence-floor crowd), found 64
  // probes a step
  int32_t fz = gb[(int64_t)ch * gcap + g + 1];
  for (int32_t lo = fa; fz - lo > 64;) {
    const int32_t st = (fz - lo + 63) / 64, x = lo + (lane + 1) * st;
    const int l = __ffsll((long long)__ballot(x >= fz || bs[x] >= S1)) - 1;  // (lane 63's x >= fz)
    fz = min(fz, lo + (l + 1) * st);
    lo += l * st;
  }
  int32_t pa = S0, pz = S0;  // the pending run of small bins: frames [pa, pz)
  auto flush = [&]() {
    if (pz > pa) BCLK(4, klast = sort_lds(pa, pz - pa, klast));
  };
  BCLK(6, {
  for (int32_t f0 = fa; f0 < fz; f0 += 64) {
    const int32_t bl = f0 + lane < fz ? bs[f0 + lane] : 0, nl = f0 + lane < fz ? bs[f0 + lane + 1] - bl : 0;
    for (unsigned long long mb = __ballot(nl > 0); mb; mb &= mb - 1) {
      const int sl = __ffsll((long long)mb) - 1;
      const int32_t b = __builtin_amdgcn_readlane(bl, sl), nb = __builtin_amdgcn_readlane(nl, sl);
      if (nb <= kBinCap) {
        if (b != pz || b + nb - pa > kBinCap) {
          flush();
          pa = b;
        }
        pz = b + nb;
        continue;
      }
      flush();
      pa = pz = b + nb;
      // frames that all share (segment, L2, d) need no order (a crowd of equal values: the silence
      // floor), nor do those of a segment without a max2 window: the waves of the bin's 64-frame
      // windows copy and check them, this one the frames before the bin's first multiple of 64
      copy_big(b, nb, b, min(b + nb, (b + kGroup - 1) / kGroup * kGroup), klast);
      if (lane == 0) atomicAdd(&info[3], 1);  // (crowd bins copied: tfp_sweep_stats)
      klast = kb[cb + b + nb - 1];  // (a crowd of one value: any of its keys)
    }
  }
  flush();
  });
#undef BCLK
#undef BCLK_BEGIN
#undef BCLK_END
}

// In-chunk prefix counts P[i][q] = frames of query q in [cbeg[ch], i], in three launches over
// kPortions 64-aligned shares per chunk (one wave each: a chunk's ~20 k frames at C3 spread over
// 256 waves instead of the 16 of one workgroup): each share's counts, their exclusive prefix per
// chunk, then each share's rows from its prefix. Lane l counts queries 2l and 2l + 1 (one word
// of two 16-bit counts) among 64 frames by reading their queries out of the lanes (no per-frame
// memory dependency).
constexpr int kPortions = 256;
// (checkpoint rows every 4 frames, -DTFP_PSTEP=4, write a fourth of the bytes, but wide_clips then
// adds up to 3 frames' increments per run end: C3 coefs = 2 0.86 / 0.73 / 0.81 / 0.89 ms at tol
// 0.001 / 0.01 / 0.1 / 0.45 against 0.77 / 0.71 / 0.73 / 0.83 with a row per frame,
// profiles/r06/c3_pstep_ab_r06h.txt)
#ifndef TFP_PSTEP
#define TFP_PSTEP 1
#endif
constexpr int kPStep = TFP_PSTEP;  // frames per prefix-count row (1 or 4)
static_assert(kPStep == 1 || kPStep == 4, "one row a frame, or a 4-byte word of queries a row");
__device__ __forceinline__ void portion_range(const int32_t* cbeg, int ch, int p, int32_t& b, int32_t& r0, int32_t& r1) {
  b = cbeg[ch];
  const int32_t n = cbeg[ch + 1] - b;
  const int32_t per = (n + kPortions * 64 - 1) / (kPortions * 64) * 64;
  r0 = min(n, p * per);
  r1 = min(n, r0 + per);
}
// frame x's increment for lane l. QPL = 2 (128-query chunks, 16-bit counts): 1 (query 2l), 1 << 16
// (query 2l + 1) or 0. QPL = 4 (256-query chunks, 8-bit counts, queries under 256 frames): 1 << 8j
// for query 4l + j. kPadQ pads (no lane's).
constexpr int32_t kPadQ = 4096;
template <int QPL>
__device__ __forceinline__ uint32_t prefix_inc(int32_t x, int lane) {
  if constexpr (QPL == 2) return (x >> 1) == lane ? (x & 1 ? 0x10000u : 1u) : 0u;
  else return (x >> 2) == lane ? (1u << (8 * (x & 3))) : 0u;
}
template <int QPL>
__global__ __launch_bounds__(1024) void wide_pcount_kernel(const int32_t* __restrict__ cbeg,
                                                           const uint8_t* __restrict__ qis, uint32_t* __restrict__ ptot) {
  const int lane = threadIdx.x & 63, p = blockIdx.y * 16 + (threadIdx.x >> 6);
  int32_t b, r0, r1;
  portion_range(cbeg, blockIdx.x, p, b, r0, r1);
  uint32_t cnt = 0;
  for (int32_t i = r0; i < r1; i += 64) {
    const int32_t x = i + lane < r1 ? (int32_t)qis[b + i + lane] : kPadQ;
#pragma unroll
    for (int j = 0; j < 64; j++) cnt += prefix_inc<QPL>(__builtin_amdgcn_readlane(x, j), lane);
  }
  ptot[((int64_t)blockIdx.x * kPortions + p) * 64 + lane] = cnt;
}
// Exclusive prefix of the shares' counts per chunk, in place: wave w scans shares 16w .. 16w + 15.
__global__ __launch_bounds__(1024) void wide_pscan_kernel(uint32_t* __restrict__ ptot) {
  __shared__ uint32_t tot[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* t = ptot + ((int64_t)blockIdx.x * kPortions + 16 * wv) * 64 + lane;
  uint32_t v[16], run = 0;
#pragma unroll
  for (int j = 0; j < 16; j++) v[j] = t[64 * j];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const uint32_t x = v[j];
    v[j] = run;
    run += x;
  }
  tot[wv][lane] = run;
  __syncthreads();
  uint32_t base = 0;
  for (int w = 0; w < wv; w++) base += tot[w][lane];
#pragma unroll
  for (int j = 0; j < 16; j++) t[64 * j] = base + v[j];
}
// The rows are checkpoints: frame i's row only when i % kPStep == kPStep - 1, at P[i / kPStep] (a
// fourth of the bytes written; wide_clips adds the up to kPStep - 1 frames after the checkpoint
// before a position from their queries, prefix_at).
template <int QPL>
__global__ __launch_bounds__(1024) void wide_prefix_kernel(const int32_t* __restrict__ cbeg, const uint8_t* __restrict__ qis,
                                                           const uint32_t* __restrict__ ptot, uint32_t* __restrict__ P) {
  const int lane = threadIdx.x & 63, p = blockIdx.y * 16 + (threadIdx.x >> 6);
  int32_t b, r0, r1;
  portion_range(cbeg, blockIdx.x, p, b, r0, r1);
  uint32_t run = ptot[((int64_t)blockIdx.x * kPortions + p) * 64 + lane];
  for (int32_t i = r0; i < r1; i += 64) {
    const int32_t x = i + lane < r1 ? (int32_t)qis[b + i + lane] : kPadQ;
    const int32_t bi = b + i;  // (global frame of j = 0)
    const int m = min(64, r1 - i);
#pragma unroll
    for (int j = 0; j < 64; j++) {
      run += prefix_inc<QPL>(__builtin_amdgcn_readlane(x, j), lane);
      if (j < m && ((bi + j) & (kPStep - 1)) == kPStep - 1) P[(int64_t)((bi + j) / kPStep) * kWideW + lane] = run;
    }
  }
}
// In-chunk prefix count at frame e (>= cb, the chunk's first frame) from the checkpoint rows: the
// row at e itself, or the last checkpoint before e in the chunk (none: 0) plus the increments of
// the frames after it up to e, read from their queries (one aligned 4-byte load; qis is padded).
// e is wave-uniform (every caller's is a shuffled or read-lane value): as a scalar, the queries'
// word is a scalar load and only the per-lane compare and add take vector registers.
template <int QPL>
__device__ __forceinline__ uint32_t prefix_at(const uint32_t* __restrict__ P, const uint8_t* __restrict__ qis, int32_t cb,
                                              int32_t e, int lane) {
  if constexpr (kPStep == 1) {
    return P[(int64_t)e * kWideW + lane];
  } else {
    e = __builtin_amdgcn_readfirstlane(e);
    const int32_t g = e / kPStep, f0 = g * kPStep;
    if (e == f0 + kPStep - 1) return P[(int64_t)g * kWideW + lane];
    uint32_t v = f0 - 1 >= cb ? P[(int64_t)(g - 1) * kWideW + lane] : 0u;
    const uint32_t w = *reinterpret_cast<const uint32_t*>(qis + f0);
#pragma unroll
    for (int j = 0; j < kPStep - 1; j++)
      if (f0 + j <= e && f0 + j >= cb) v += prefix_inc<QPL>((int32_t)((w >> (8 * j)) & 255u), lane);
    return v;
  }
}

// lb32 / ub32: tfp_bsearch.hpp (both ends read with the first probe)

#ifndef TFP_CLIP_DPP
#define TFP_CLIP_DPP 1  // the sweep's lane scans through DPP (A/B: 0 takes ds_bpermute shuffles; even at C3)
#endif
// Inclusive max over lanes [gst, lane] of bm (gst <= lane, per lane): four row shifts, then rows 1
// and 3 take lane 15 of the row before and rows 2 and 3 lane 31 (DPP: no LDS round trip per step).
__device__ __forceinline__ int32_t seg_max_scan(int32_t bm, int32_t gst, int lane) {
#if TFP_CLIP_DPP
  const int rl = lane & 15;
  int32_t y;
  y = __builtin_amdgcn_update_dpp(bm, bm, 0x111, 0xf, 0xf, false);  // row_shr:1
  if (rl >= 1 && lane - 1 >= gst) bm = max(bm, y);
  y = __builtin_amdgcn_update_dpp(bm, bm, 0x112, 0xf, 0xf, false);  // row_shr:2
  if (rl >= 2 && lane - 2 >= gst) bm = max(bm, y);
  y = __builtin_amdgcn_update_dpp(bm, bm, 0x114, 0xf, 0xf, false);  // row_shr:4
  if (rl >= 4 && lane - 4 >= gst) bm = max(bm, y);
  y = __builtin_amdgcn_update_dpp(bm, bm, 0x118, 0xf, 0xf, false);  // row_shr:8
  if (rl >= 8 && lane - 8 >= gst) bm = max(bm, y);
  y = __builtin_amdgcn_update_dpp(bm, bm, 0x142, 0xa, 0xf, false);  // row_bcast:15 (rows 1, 3)
  if ((lane & 16) && (lane & ~15) - 1 >= gst) bm = max(bm, y);
  y = __builtin_amdgcn_update_dpp(bm, bm, 0x143, 0xc, 0xf, false);  // row_bcast:31 (rows 2, 3)
  if (lane >= 32 && 31 >= gst) bm = max(bm, y);
  return bm;
#else
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(bm, o, 64);
    if (lane - o >= gst) bm = max(bm, y);
  }
  return bm;
#endif
}
// OR of x over the wave (DPP: row shifts, then the rows' last lanes; no LDS round trip)
__device__ __forceinline__ uint32_t wave_or_dpp(uint32_t x) {
  x |= (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x |= (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x |= (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x |= (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x |= (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x |= (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
// lane l's v from lane l - 1 (lane 0: its own)
__device__ __forceinline__ int32_t lane_before(int32_t v) {
#if TFP_CLIP_DPP
  return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xf, 0xf, false);  // wave_shr:1
#else
  return __shfl_up(v, 1, 64);
#endif
}

// ---- clip-major sweep ------------------------------------------------------------------------
// Work items are (chunk, key, clip group). A wave takes windows of kWin consecutive clip columns of
// one chunk and, for each key the chunk uses, the groups of those clips (two kdir loads per key, no
// search), so every count a clip gets in the chunk lands in the wave's own LDS row for it. After a
// window's keys the wave takes each query's best (count << 32 | tie key) over the window's clips in
// registers: no score rows in memory, no atomics, no final pass over the clips. Per-wave maxima go to
// part[ch][x][query], reduced by wide_part_max. (Round 3 also had a key-major form with score rows in
// memory; it lost its A/B and was removed in round 5.)
constexpr int kWin = CellCache::kWin;
constexpr int kClipWaves = 4;  // waves per workgroup

// The used keys of each chunk, ascending: ukeys[ch][0 .. nuk[ch]).
__global__ __launch_bounds__(1024) void wide_ukeys_kernel(const int32_t* __restrict__ seg, int32_t* __restrict__ ukeys,
                                                          int32_t* __restrict__ nuk) {
  __shared__ int32_t wcnt[16];
  const int ch = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int32_t* sg = seg + (int64_t)ch * kWideSegs * 2;
  const bool used = sg[2 * t + 1] > sg[2 * t] || sg[2 * (t | kKeyRange) + 1] > sg[2 * (t | kKeyRange)];
  const unsigned long long m = __ballot(used);
  if (lane == 0) wcnt[wv] = __popcll(m);
  __syncthreads();
  int32_t off = 0;
  for (int w = 0; w < wv; w++) off += wcnt[w];
  if (used) ukeys[(int64_t)ch * kKeyRange + off + __popcll(m & ((1ull << lane) - 1))] = t;
  if (t == 0) {
    int32_t n = 0;
    for (int w = 0; w < 16; w++) n += wcnt[w];
    nuk[ch] = n;
  }
}

// waves per SIMD the register budget is cut for (5, 6, 8: 1.185, 1.179, 1.151 ms at C3 tol 0.001;
// 8 spilled 12 VGPRs before r04: the wave index is now scalar, 49 VGPRs)
constexpr int kClipOcc = 8;
#ifndef TFP_CLIP_GROUP_MASK
#define TFP_CLIP_GROUP_MASK 1  // a batch's groups from a DPP-reduced mask of their starts (A/B: 0 binary lifting)
#endif
#ifndef TFP_CLIP_RUNQ
// a batch's run ends lane-parallel, their prefix rows this many runs at a time (A/B: 0 one by one;
// C3 tol 0.001 wide_clips 192 / 157 / 154 us at 0 / 4 / 6, 63 VGPRs at 6 and spills at 8)
#define TFP_CLIP_RUNQ 4
#endif
#ifndef TFP_CLIP_LAZY
#define TFP_CLIP_LAZY 1  // count rows written on a column's first add (A/B: 0 clears all 16 per window)
#endif
template <int QPL>
__global__ __launch_bounds__(64 * kClipWaves, kClipOcc) void wide_clips_kernel(
    int32_t xw, const int32_t* __restrict__ seg, const int32_t* __restrict__ cbeg, CellView cv,
    const int32_t* __restrict__ kdir, int32_t nwin, const int32_t* __restrict__ ukeys, const int32_t* __restrict__ nuk,
    const int32_t* __restrict__ L2s, const int32_t* __restrict__ U2s, const uint32_t* __restrict__ P,
    const uint8_t* __restrict__ qis, const int32_t* __restrict__ tiekey, int32_t C, const int4* __restrict__ segk, const int32_t* __restrict__ dtab,
    unsigned long long* __restrict__ part, const int32_t* __restrict__ stop, int32_t col_base, long long* __restrict__ wclk) {
  // stop (the bin sort's batches): info; info[2] > 0 left a bin unsorted and its directory unbuilt,
  // so the sweep reads nothing (the batch is redone; its maxima are not used)
  if (stop && stop[2] > 0) return;
  __shared__ __attribute__((aligned(16))) uint32_t accs[kClipWaves][kWin * 64];
#if TFP_BIN_CLOCKS
  // (the diagnostic build with TFP_DEBUG_BINS: each wave's clock cycles and dispatch order in wclk)
  struct ClipClock {
    long long* w;
    long long t0;
    __device__ ~ClipClock() {
      if (w && (threadIdx.x & 63) == 0) {
        w[0] = clock64() - t0;
        w[1] = t0;
      }
    }
  } clip_clock{wclk ? wclk + 2 * ((int64_t)blockIdx.x * kClipWaves + (threadIdx.x >> 6)) : nullptr, clock64()};
#else
  (void)wclk;
#endif
  // wv through readfirstlane: the wave's chunk, window range and per-chunk pointers are then scalar
  // (as per-lane values they took 64-bit VGPR pairs, and 12 VGPRs spilled at 8 waves per SIMD)
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t gw = (int64_t)blockIdx.x * kClipWaves + wv;
  const int ch = (int)(gw / xw), x = (int)(gw % xw);
  uint32_t* acc = accs[wv];
  const int32_t per = (nwin + xw - 1) / xw;
  const int32_t w0 = min(nwin, x * per), w1 = min(nwin, w0 + per);
  const int32_t nu = nuk[ch];
  const int32_t* uk = ukeys + (int64_t)ch * kKeyRange;
  const int32_t* sg = seg + (int64_t)ch * kWideSegs * 2;
  const int32_t cb = cbeg[ch];
  unsigned long long r[QPL];  // queries 64 QPL ch + QPL lane + j: best (count << 32 | tie key)
#pragma unroll
  for (int j = 0; j < QPL; j++) r[j] = 0;
  int32_t sb = 0, se = 0;
  uint32_t base = 0, fcnt = 0;
  int32_t nbk = 1, shf = 0, l2min = 0, u2min = 0;
  const int32_t* TL = dtab;
  auto find_ab = [&](int32_t va, int32_t vb, int32_t& A, int32_t& B) {
    const int64_t dv = (int64_t)vb - l2min;
    if (dv < 0) {
      B = sb - 1;
    } else {
      const int32_t b = (int32_t)min<int64_t>(dv >> shf, nbk - 1);
      const int32_t lo = TL[b], hi = b + 1 < nbk ? TL[b + 1] : se;
      B = lo + ub32(L2s + lo, hi - lo, vb) - 1;
    }
    const int64_t du = (int64_t)va - u2min;
    if (du <= 0) {
      A = sb;
    } else {
      const int32_t b = (int32_t)min<int64_t>(du >> shf, nbk - 1);
      const int32_t lo = TL[nbk + b], hi = b + 1 < nbk ? TL[nbk + b + 1] : se;
      A = lo + lb32(U2s + lo, hi - lo, va);
    }
  };
  auto close_run = [&](uint32_t& cnt, int32_t a, int32_t b) {
    cnt += prefix_at<QPL>(P, qis, cb, b, lane) - (a > sb ? prefix_at<QPL>(P, qis, cb, a - 1, lane) : base);
  };
  // The chunk's used keys' segment constants, one key per lane, loaded once per wave instead of
  // once per window and key (three dependent loads ahead of every key's groups): the window loop
  // reads them with readlane. More than 64 used keys: loaded per window and key as below.
  const bool kpre = nu <= 64;
  int32_t ksb = 0, kse = 0, kfb = 0, kfe = 0, kshf = 0, kl2 = 0, ku2 = 0, ktoff = 0;
  if (kpre && lane < nu) {
    const int kq = uk[lane];
    ksb = sg[2 * kq];
    kse = sg[2 * kq + 1];
    kfb = sg[2 * (kq | kKeyRange)];
    kfe = sg[2 * (kq | kKeyRange) + 1];
    if (kse > ksb) {
      const int4 c4 = segk[(int64_t)ch * kKeyRange + kq];
      kl2 = c4.x;
      ku2 = c4.y;
      kshf = c4.z;
      ktoff = c4.w;
    }
  }
  for (int32_t w = w0; w < w1; w++) {
    const int32_t c0 = kWin * w;
    // the used keys with groups in this window, 64 keys a step; a window in which none of them
    // has a group (up to 64 used keys: the first step's ballot) scores nothing, so its counts are
    // neither cleared nor read
    int32_t kk = 0, ga = 0, gb = 0;
    if (lane < nu) {
      kk = uk[lane];
      ga = kdir[(int64_t)kk * (nwin + 1) + w];
      gb = kdir[(int64_t)kk * (nwin + 1) + w + 1];
    }
    unsigned long long km = __ballot(gb > ga);
    if (kpre && !km) continue;
    // the window's tie keys, requested before its groups (read at its end)
    const int32_t tk = col_base + c0 + lane < C && lane < kWin ? tiekey[col_base + c0 + lane] : 0;
#if TFP_CLIP_LAZY
    // the window's columns that got a count (wave-uniform): each column's row is written by its
    // first add and read only if written, so nothing is cleared and untouched columns cost nothing
    // (at C3 -3 % per coefs = 2 batch at tol 0.001 / 0.01, even at 0.1 / 0.45; clearing the rows
    // of windows with many groups did not pay: profiles/r06/c3_window_ab_r06.txt)
    uint32_t touched = 0;
    auto add = [&](int32_t col, uint32_t cnt) {
      const int32_t j = __builtin_amdgcn_readfirstlane(col - c0);
      uint32_t* a = acc + j * 64 + lane;
      if ((touched >> j) & 1u) {
        *a += cnt;
      } else {
        *a = cnt;
        touched |= 1u << j;
      }
    };
#else
    constexpr uint32_t touched = (1u << kWin) - 1;
#pragma unroll
    for (int j = 0; j < kWin; j++) acc[j * 64 + lane] = 0u;
    auto add = [&](int32_t col, uint32_t cnt) { acc[(col - c0) * 64 + lane] += cnt; };
#endif
    for (int32_t u0 = 0; u0 < nu; u0 += 64) {
      if (u0 > 0) {
        kk = ga = gb = 0;
        if (u0 + lane < nu) {
          kk = uk[u0 + lane];
          ga = kdir[(int64_t)kk * (nwin + 1) + w];
          gb = kdir[(int64_t)kk * (nwin + 1) + w + 1];
        }
        km = __ballot(gb > ga);
      }
      while (km) {
        const int sl = __ffsll((long long)km) - 1;
        km &= km - 1;
        const int k = __builtin_amdgcn_readlane(kk, sl);
        const int32_t g1 = __builtin_amdgcn_readlane(gb, sl);
        int32_t g = __builtin_amdgcn_readlane(ga, sl);
        // the key's window segment and its frames without a max2 window
        int32_t fb, fe;
        if (kpre) {  // (u0 == 0: the key's slot is lane sl)
          sb = __builtin_amdgcn_readlane(ksb, sl);
          se = __builtin_amdgcn_readlane(kse, sl);
          fb = __builtin_amdgcn_readlane(kfb, sl);
          fe = __builtin_amdgcn_readlane(kfe, sl);
        } else {
          sb = sg[2 * k];
          se = sg[2 * k + 1];
          fb = sg[2 * (k | kKeyRange)];
          fe = sg[2 * (k | kKeyRange) + 1];
        }
        base = se > sb && sb > cb ? prefix_at<QPL>(P, qis, cb, sb - 1, lane) : 0u;
        fcnt = fe > fb ? prefix_at<QPL>(P, qis, cb, fe - 1, lane) - (fb > cb ? prefix_at<QPL>(P, qis, cb, fb - 1, lane) : 0u) : 0u;
        if (se <= sb) {  // no frame of the key has a max2 window: every group scores the rest
          for (; g < g1; g++) add((int32_t)(cv.g_key[g] & kColMask), fcnt);
          continue;
        }
        if (kpre) {
          nbk = 1 << dir_log2(se - sb);
          l2min = __builtin_amdgcn_readlane(kl2, sl);
          u2min = __builtin_amdgcn_readlane(ku2, sl);
          shf = __builtin_amdgcn_readlane(kshf, sl);
          TL = dtab + __builtin_amdgcn_readlane(ktoff, sl);
        } else {
          nbk = 1 << dir_log2(se - sb);
          const int4 c4 = segk[(int64_t)ch * kKeyRange + k];
          l2min = c4.x;
          u2min = c4.y;
          shf = c4.z;
          TL = dtab + c4.w;
        }
        // A batch of consecutive groups whose items fit the 64 lanes: lane j holds group j's item
        // range [pj0, pj1) relative to the first item pb0.
        while (g < g1) {
          const int32_t left = g1 - g;
          int32_t pj0 = 0, pj1 = INT32_MAX, colj = 0;
          const int32_t pb0 = cv.g_beg[g];
          if (lane < left) {
            pj0 = cv.g_beg[g + lane] - pb0;
            pj1 = cv.g_beg[g + lane + 1] - pb0;
            colj = (int32_t)(cv.g_key[g + lane] & kColMask);
          }
          const int nG = __popcll(__ballot(lane < left && pj1 <= 64));  // (pj1 grows with j: a prefix)
          if (nG == 0) {  // one group with more than 64 items: 64 at a time, runs merged across the steps
            const int32_t pn = __builtin_amdgcn_readlane(pj1, 0);
            uint32_t cnt = fcnt;
            int32_t carry = -2, aopen = 0;
            bool open = false;
            for (int32_t pbase = 0; pbase < pn; pbase += 64) {
              const int32_t i = pbase + lane;
              int32_t A = INT32_MAX, B = -2;
              if (i < pn) find_ab(cv.p_m2[pb0 + i], cv.p_hi[pb0 + i], A, B);
              const bool ok = A <= B;
              const int32_t bm = seg_max_scan(ok ? B : -2, 0, lane);
              int32_t pe = lane_before(bm);
              if (lane == 0) pe = -2;
              pe = max(pe, carry);
              unsigned long long starts = __ballot(ok && A > pe + 1);
              while (starts) {
                const int s2 = __ffsll((long long)starts) - 1;
                starts &= starts - 1;
                const int32_t as = __builtin_amdgcn_readlane(A, s2), ps = __builtin_amdgcn_readlane(pe, s2);
                if (open) close_run(cnt, aopen, ps);
                open = true;
                aopen = as;
              }
              carry = max(carry, __builtin_amdgcn_readlane(bm, 63));
            }
            if (open) close_run(cnt, aopen, carry);
            add(__builtin_amdgcn_readlane(colj, 0), cnt);
            g++;
            continue;
          }
          // every item of the batch on its own lane: its group (the last j < nG with pj0 <= lane, by
          // binary lifting over the lanes' starts) and its run [A, B] of the segment's frames
          const int32_t npts = __builtin_amdgcn_readlane(pj1, nG - 1);
#if TFP_CLIP_GROUP_MASK
          // the batch's group starts as one wave-uniform mask (groups are contiguous and non-empty:
          // each starts one bit past its predecessor's items), OR-reduced through DPP: a lane's
          // group, its start and the next group's start by bit counts, where a binary lifting took
          // six dependent ds_bpermute
          const unsigned long long bitj = lane < nG ? 1ull << pj0 : 0ull;
          const unsigned long long gm = ((unsigned long long)wave_or_dpp((uint32_t)(bitj >> 32)) << 32) |
                                        wave_or_dpp((uint32_t)bitj);
          const unsigned long long le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
          const int gi = __popcll(gm & le) - 1;
          const int32_t gst = 63 - __clzll(gm & le);
#else
          int gi = 0;
#pragma unroll
          for (int bit = 32; bit >= 1; bit >>= 1) {
            const int cand = gi + bit;
            const int32_t xx = __shfl(pj0, min(cand, 63), 64);
            if (cand < nG && xx <= lane) gi = cand;
          }
          const int32_t gst = __shfl(pj0, gi, 64);
#endif
          int32_t A = INT32_MAX, B = -2;
          if (lane < npts) find_ab(cv.p_m2[pb0 + lane], cv.p_hi[pb0 + lane], A, B);
          const bool ok = lane < npts && A <= B;
          const int32_t bm = seg_max_scan(ok ? B : -2, gst, lane);
          int32_t pe = lane_before(bm);
          if (lane == gst) pe = -2;
          const unsigned long long starts = __ballot(ok && A > pe + 1);
#if TFP_CLIP_RUNQ
          // Every run's end at once, lane-parallel: a run starting at lane l ends where the next run
          // of its group starts (pe there) or at its group's last item (bm). Then the runs' prefix
          // rows kQ runs at a time: their 2 kQ loads in flight together, where one run's two loads
          // each waited out a round trip before the next run's were issued (the batch's runs were
          // a chain of dependent-latency steps). Each group's count (fcnt + its runs' deltas) goes
          // to its column in group order, as before.
          const unsigned long long later = lane < 63 ? starts & (~0ull << (lane + 1)) : 0ull;
          const int nx = later ? (int)__builtin_ctzll(later) : 64;
#if TFP_CLIP_GROUP_MASK
          const unsigned long long gab = gm & ~le;
          const int32_t gend = gab ? (int32_t)__builtin_ctzll(gab) : npts;
#else
          const int32_t gend = __shfl(pj1, gi, 64);
#endif
          const int32_t pen = __shfl(pe, nx < 64 ? nx : 63, 64), bme = __shfl(bm, gend > 0 ? gend - 1 : 0, 64);
          const int32_t rend = nx < gend ? pen : bme;
          int cg = 0;
          uint32_t cnt = fcnt;
          auto flush_to = [&](int gg) {
            for (; cg < gg; cg++) {
              add(__builtin_amdgcn_readlane(colj, cg), cnt);
              cnt = fcnt;
            }
          };
          constexpr int kQ = TFP_CLIP_RUNQ;
          for (unsigned long long rm = starts; rm;) {
            int rl[kQ] = {}, nr = 0;
            uint32_t hv[kQ] = {}, lv[kQ] = {};
#pragma unroll
            for (int k = 0; k < kQ; k++) {
              if (rm) {
                const int l = __ffsll((long long)rm) - 1;
                rm &= rm - 1;
                rl[k] = l;
                nr = k + 1;
                const int32_t a = __builtin_amdgcn_readlane(A, l), b = __builtin_amdgcn_readlane(rend, l);
                hv[k] = prefix_at<QPL>(P, qis, cb, b, lane);
                lv[k] = a > sb ? prefix_at<QPL>(P, qis, cb, a - 1, lane) : base;
              }
            }
#pragma unroll
            for (int k = 0; k < kQ; k++) {
              if (k < nr) {
                flush_to(__builtin_amdgcn_readlane(gi, rl[k]));
                cnt += hv[k] - lv[k];
              }
            }
          }
          flush_to(nG);
#else
          for (int j = 0; j < nG; j++) {
            const int32_t a0 = __builtin_amdgcn_readlane(pj0, j), a1 = __builtin_amdgcn_readlane(pj1, j);
            const unsigned long long rng = (a1 >= 64 ? ~0ull : ((1ull << a1) - 1)) & ~((1ull << a0) - 1);
            unsigned long long mm = starts & rng;
            uint32_t cnt = fcnt;
            int32_t aopen = 0;
            bool open = false;
            while (mm) {
              const int s2 = __ffsll((long long)mm) - 1;
              mm &= mm - 1;
              const int32_t as = __builtin_amdgcn_readlane(A, s2), ps = __builtin_amdgcn_readlane(pe, s2);
              if (open) close_run(cnt, aopen, ps);
              open = true;
              aopen = as;
            }
            if (open) close_run(cnt, aopen, __builtin_amdgcn_readlane(bm, a1 - 1));
            add(__builtin_amdgcn_readlane(colj, j), cnt);
          }
#endif
          g += nG;
        }
      }
    }
    // the window's clips: each query's best (count << 32 | tie key)
    if (!touched) continue;  // (TFP_CLIP_LAZY)
    auto take = [&](int j) {
      const uint32_t v = acc[j * 64 + lane];
      const unsigned long long t = (uint32_t)__builtin_amdgcn_readlane(tk, j);
#pragma unroll
      for (int b = 0; b < QPL; b++) {
        const uint32_t c = QPL == 2 ? (b ? v >> 16 : v & 0xffffu) : (v >> (8 * b)) & 0xffu;
        const unsigned long long k = ((unsigned long long)c << 32) | t;
        if (c) r[b] = k > r[b] ? k : r[b];
      }
    };
    if (touched == (1u << kWin) - 1) {  // (all 16 rows read at once)
#pragma unroll
      for (int j = 0; j < kWin; j++) take(j);
    } else {
      for (uint32_t tm = touched; tm; tm &= tm - 1) take(__builtin_ctz(tm));
    }
  }
  // the workgroup's maxima (its waves share the chunk: xw is a multiple of kClipWaves), through
  // each wave's own count rows (free after its last window: 4 KB, the chunk's 64 QPL keys fit)
  constexpr int Q = 64 * QPL;
  static_assert(Q * sizeof(unsigned long long) <= kWin * 64 * sizeof(uint32_t), "maxima in the count rows");
  unsigned long long* redw = reinterpret_cast<unsigned long long*>(accs[wv]);
#pragma unroll
  for (int b = 0; b < QPL; b++) redw[QPL * lane + b] = r[b];
  __syncthreads();
  for (int t = threadIdx.x; t < Q; t += 64 * kClipWaves) {
    unsigned long long m = reinterpret_cast<const unsigned long long*>(accs[0])[t];
    for (int w2 = 1; w2 < kClipWaves; w2++) {
      const unsigned long long y = reinterpret_cast<const unsigned long long*>(accs[w2])[t];
      m = y > m ? y : m;
    }
    part[((int64_t)ch * (xw / kClipWaves) + x / kClipWaves) * Q + t] = m;
  }
}

// best[q] = max over the chunk's nb per-workgroup maxima (one workgroup per chunk: query t & 127,
// every 8th maximum from t >> 7, then the 8 slices in LDS).
template <int QPL>
__global__ __launch_bounds__(1024) void wide_part_max_kernel(const unsigned long long* __restrict__ part, int32_t nb,
                                                             int32_t nq, unsigned long long* __restrict__ best,
                                                             const int32_t* __restrict__ info, int32_t* __restrict__ info_out) {
  // (the sweep's counts into the caller's host-mapped memory, read with the results: no copy launch)
  if (info_out && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 4) info_out[threadIdx.x] = info[threadIdx.x];
  constexpr int Q = 64 * QPL, S = 1024 / Q;  // queries per chunk, slices
  __shared__ unsigned long long red[S][Q];
  // (gridDim.y workgroups per chunk, each over every gridDim.y-th slice of the maxima: a chunk's
  // 8-17 MB of maxima read by more than one CU; their results meet in an atomic max)
  const int ch = blockIdx.x, t = threadIdx.x & (Q - 1), sl = threadIdx.x / Q;
  const unsigned long long* pp = part + (int64_t)ch * nb * Q + t;
  unsigned long long m = 0;
#pragma unroll 4
  for (int32_t x = blockIdx.y * S + sl; x < nb; x += S * gridDim.y) m = pp[(int64_t)x * Q] > m ? pp[(int64_t)x * Q] : m;
  red[sl][t] = m;
  __syncthreads();
  if (sl == 0) {
    for (int j = 1; j < S; j++) m = red[j][t] > m ? red[j][t] : m;
    const int32_t q = ch * Q + t;
    if (m && q < nq) atomicMax(&best[q], m);
  }
}

}  // namespace

void WideScratch::release() {
  for (void* p : {(void*)ka, (void*)kb, (void*)ua, (void*)ub, (void*)va, (void*)vb, (void*)L2s, (void*)U2s, (void*)qis,
                  (void*)P, (void*)seg, (void*)cbeg, (void*)info, (void*)ptot, (void*)ukeys, (void*)nuk, (void*)part,
                  (void*)fq, (void*)doff, (void*)dtab, dtmp, tmp, (void*)bstart, (void*)segk, (void*)segstat,
                  (void*)ghist})
    if (p) (void)hipFree(p);
  bstart = ghist = nullptr;
  segk = nullptr;
  segstat = nullptr;
  for (void* q : {(void*)gi4, (void*)gb, (void*)wclk})
    if (q) (void)hipFree(q);
  gi4 = nullptr;
  gb = nullptr;
  wclk = nullptr;
  cap_groups = 0;
  ptot = nullptr;
  ukeys = nuk = nullptr;
  part = nullptr;
  fq = nullptr;
  doff = dtab = nullptr;
  dtmp = nullptr;
  dtmp_bytes = 0;
  cap_dtab = 0;
  ka = kb = nullptr;
  ua = ub = nullptr;
  va = vb = L2s = U2s = seg = cbeg = info = nullptr;
  P = nullptr;
  qis = nullptr;
  tmp = nullptr;
  tmp_bytes = 0;
  cap_nf = cap_nch = 0;
}

hipError_t WideScratch::reserve(int64_t nf, int32_t nq, hipStream_t s) {
  const int64_t nch = (nq + kWideCh - 1) / kWideCh;
  hipError_t e = hipSuccess;
  if (nf > cap_nf) {
    for (void* p : {(void*)ka, (void*)kb, (void*)ua, (void*)ub, (void*)va, (void*)vb, (void*)L2s, (void*)U2s, (void*)qis,
                    (void*)P, (void*)fq, tmp})
      if (p) (void)hipFree(p);
    ka = kb = nullptr;
    ua = ub = nullptr;
    va = vb = L2s = U2s = fq = nullptr;
    P = nullptr;
    qis = nullptr;
    tmp = nullptr;
    cap_nf = 0;
    if ((e = dmalloc(&ka, nf)) || (e = dmalloc(&kb, nf)) || (e = dmalloc(&ua, nf)) || (e = dmalloc(&ub, nf)) ||
        (e = dmalloc(&va, nf)) || (e = dmalloc(&vb, nf)) || (e = dmalloc(&L2s, nf)) || (e = dmalloc(&U2s, nf)) ||
        (e = dmalloc(&qis, nf + 16)) || (e = dmalloc(&P, (nf / kPStep + 2) * kWideW)) || (e = dmalloc(&fq, nf)))
      return e;
    size_t t1 = 0, t2 = 0;
    size_t t3 = 0;
    if ((e = sweep_sort_pairs<uint32_t>(nullptr, t1, ua, ub, va, vb, nf, 32, s)) ||
        (e = sweep_sort_pairs<unsigned long long>(nullptr, t2, ka, kb, va, vb, nf, 64, s)) ||
        (e = sweep_sort_keys<unsigned long long>(nullptr, t3, ka, kb, nf, 64, s)))
      return e;
    tmp_bytes = std::max(t1, std::max(t2, t3));
    if ((e = hipMalloc(&tmp, tmp_bytes > 0 ? tmp_bytes : 1))) return e;
    cap_nf = nf;
  }
  if (nch > cap_nch) {
    for (void* p : {(void*)seg, (void*)cbeg, (void*)doff, (void*)ptot, (void*)ukeys, (void*)nuk, (void*)part, dtmp,
                    (void*)bstart, (void*)segk, (void*)segstat, (void*)ghist})
      if (p) (void)hipFree(p);
    seg = cbeg = doff = ukeys = nuk = nullptr;
    bstart = ghist = nullptr;
    segk = nullptr;
    segstat = nullptr;
    ptot = nullptr;
    part = nullptr;
    dtmp = nullptr;
    dtmp_bytes = 0;
    cap_nch = 0;
    if ((e = dmalloc(&seg, nch * kWideSegs * 2)) || (e = dmalloc(&cbeg, nch + 1)) || (e = dmalloc(&doff, nch * kKeyRange + 1)) ||
        (e = dmalloc(&ptot, nch * kPortions * 64)) || (e = dmalloc(&ukeys, nch * kKeyRange)) || (e = dmalloc(&nuk, nch)) ||
        (e = dmalloc(&part, (nq + 255) / 256 * (2 * kPartWaves) * 256)) ||  // up to 2 kPartWaves waves per chunk, either chunk size
        (e = dmalloc(&bstart, nch * (kNFine + 1))) ||
        (e = dmalloc(&segstat, nch * kWideSegs * 3)) || (e = dmalloc(&ghist, nch * kNFine)) ||
        (e = dmalloc(&segk, nch * kKeyRange)))
      return e;
    size_t tb = 0;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, doff, doff, (int)(nch * kKeyRange + 1), s))) return e;
    if ((e = hipMalloc(&dtmp, tb > 0 ? tb : 1))) return e;
    dtmp_bytes = tb;
    cap_nch = nch;
  }
  // the directory table: sum over segments of 2 NB <= 4 S (NB < 2 S), so <= 4 nf entries; it first
  // holds the size pass's nch * kKeyRange + 1 entries (scanned into doff before the fill)
  const int64_t need_d = std::max<int64_t>((4 << kDirScale) * nf + 8, nch * kKeyRange + 1);
  if (need_d > cap_dtab) {
    if (dtab) (void)hipFree(dtab);
    dtab = nullptr;
    cap_dtab = 0;
    if ((e = dmalloc(&dtab, need_d))) return e;
    cap_dtab = need_d;
  }
  if (!info && (e = dmalloc(&info, 4))) return e;
  return hipSuccess;
}

hipError_t launch_scan_wide_prepare(const FrameBox* boxes, const int64_t* d_qoff, int32_t nq, int64_t nf,
                                    int64_t max_qframes, double tole, WideScratch* ws, bool* eligible, hipStream_t s,
                                    bool speculative, unsigned long long* d_best_zero) {
  *eligible = false;
  ws->spec = false;
  if (nq <= 0 || nf <= 0 || nf >= INT32_MAX / (4 << kDirScale) - 8 || (int64_t)nq / kWideCh >= (1 << 17) || max_qframes >= 65536)
    return hipSuccess;
  hipError_t e;
  // 256-query chunks (four 8-bit counts per lane word) when every query has under 256 frames and the
  // clip-major sweep will run: half the chunks, so half the (clip, key, chunk) searches
  ws->qch = (!ws->ch128 && max_qframes < 256) ? 256 : kWideCh;
  const int32_t qch = ws->qch;
  const int64_t nch = (nq + qch - 1) / qch;
  int cb = 1;  // chunk bits: every chunk number below 2^cb - 1, so no key reaches the ~0 of unused frames
  while (((int64_t)1 << cb) - 1 <= nch) cb++;
  // U2 - L2 lies within a few micro-units of 2 tol (fmt6 rounds both ends): d = U2 - L2 - dbase
  const int64_t dbase = (tole >= 0.0 && tole < 1e6) ? (int64_t)floor(2.0 * tole * 1e6) - 3 : -1;
  // the packed key (keys-only sort) whenever the delta field can hold every width (checked with
  // the results: info[2]) and the chunk number fits its 10 bits
  bool packed = dbase >= 0 && cb <= 10 && !ws->unpacked;
  const int end_bit = (packed ? kPackChunkShift : kWideChunkShift) + cb;
  speculative = speculative && dbase >= 0;
  // the bin sort on the speculative pass of a packed batch (its overflow, like a window width outside
  // the delta field, sends the batch to the non-speculative pass); the library sort otherwise
  // (and chunks of at most 2^18 frames: a frame's place in its bin takes kPlaceBits bits)
  const bool bins = packed && speculative && !ws->libsort && (int64_t)qch * max_qframes < (1 << kPlaceBits);
  ws->ukeys_ready = bins;
  hipLaunchKernelGGL(wide_frame_query_kernel, dim3((unsigned)std::min<int64_t>(2048, ((int64_t)nq * 64 + 255) / 256)), dim3(256),
                     0, s, d_qoff, nq, ws->fq, ws->info, ws->seg, nch * kWideSegs * 2, d_best_zero, bins ? ws->segstat : nullptr,
                     ws->ghist, nch * kNFine);
  // one sort by (chunk, key, L2, U2 - L2); the key pass also counts the bad frames (info[1])
  const unsigned kgrid = std::min(grid_for(nf), kKeysBlocks);
  hipLaunchKernelGGL(wide_keys_c_kernel, dim3(kgrid), dim3(256), 0, s, boxes, ws->fq, nf, qch, packed, (const int32_t*)nullptr,
                     dbase, ws->ka, packed ? (int32_t*)nullptr : ws->va, ws->info, bins ? ws->segstat : nullptr);
  if (bins) {
    ws->min_width = dbase;
    ws->spec = true;
    const int64_t maxc = std::min<int64_t>(nf, (int64_t)qch * max_qframes);
    const int64_t spc = std::max<int64_t>(1, (maxc + 1024 * kHistPer - 1) / (1024 * kHistPer));
    hipLaunchKernelGGL(wide_bin_hist_kernel, dim3((unsigned)nch, (unsigned)spc), dim3(1024), 0, s, d_qoff, nq, qch, ws->ka,
                       ws->segstat, ws->ghist, reinterpret_cast<uint32_t*>(ws->vb));
    const int64_t gcap = (maxc + kGroup - 1) / kGroup + 2;  // sort groups per chunk, and the closing entry
    if (nch * gcap > ws->cap_groups) {
      for (void* q : {(void*)ws->gi4, (void*)ws->gb})
        if (q) (void)hipFree(q);
      ws->gi4 = nullptr;
      ws->gb = nullptr;
      ws->cap_groups = 0;
      if ((e = dmalloc(&ws->gi4, nch * gcap)) || (e = dmalloc(&ws->gb, nch * gcap))) return e;
      ws->cap_groups = nch * gcap;
      if (ws->debug_bins) {
        if (ws->wclk) (void)hipFree(ws->wclk);
        ws->wclk = nullptr;
        if ((e = dmalloc(&ws->wclk, nch * gcap * 8))) return e;
        if ((e = hipMemsetAsync(ws->wclk, 0, sizeof(long long) * nch * gcap * 8, s))) return e;
      }
    }
    hipLaunchKernelGGL(wide_bin_scan_kernel, dim3((unsigned)nch), dim3(1024), 0, s, d_qoff, nq, qch, (int32_t)nch, ws->segstat,
                       ws->ghist, ws->bstart, ws->seg, ws->ukeys, ws->nuk, ws->cbeg, ws->qis, ws->gi4, ws->gb,
                       (int32_t)gcap, dbase, ws->segk);
    hipLaunchKernelGGL(wide_bin_scatter_kernel, dim3(grid_for(nf)), dim3(256), 0, s, nf, qch, ws->fq, ws->ka,
                       reinterpret_cast<const uint32_t*>(ws->vb), ws->cbeg,
                       ws->bstart, ws->kb);
    hipLaunchKernelGGL(wide_bin_sort_kernel, dim3((unsigned)nch, (unsigned)((gcap + kBinSortWaves - 1) / kBinSortWaves)),
                       dim3(64 * kBinSortWaves), 0, s, ws->bstart, ws->gi4, ws->gb, (int32_t)gcap, ws->cbeg, ws->kb, dbase, ws->seg,
                       ws->segk, ws->L2s, ws->U2s, ws->qis, ws->dtab, ws->info, ws->debug_bins ? ws->wclk : nullptr);
    if (ws->debug_bins) {  // (TFP_DEBUG_BINS: the bin sort's counts of the first chunk, on stderr)
      std::vector<int32_t> bs(kNFine + 1);
      std::vector<int4> g(gcap);
      int32_t inf[3];
      if ((e = hipMemcpyAsync(bs.data(), ws->bstart, sizeof(int32_t) * (kNFine + 1), hipMemcpyDeviceToHost, s)) ||
          (e = hipMemcpyAsync(g.data(), ws->gi4, sizeof(int4) * gcap, hipMemcpyDeviceToHost, s)) ||
          (e = hipMemcpyAsync(inf, ws->info, sizeof inf, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
        return e;
      int32_t nb = 0, big = 0, mx = 0, gbig = 0, gmx = 0, ng = 0;
      for (int f = 0; f < kNFine; f++) {
        const int32_t c = bs[f + 1] - bs[f];
        nb += c > 0, big += c > kBinCap, mx = std::max(mx, c);
      }
      for (int64_t i = 0; i + 1 < gcap; i++) {
        const int32_t c = g[i].y - g[i].x;
        ng += c > 0, gbig += c > kBinCap, gmx = std::max(gmx, c);
      }
      fprintf(stderr, "[tfp] bins chunk 0: kept %d, %d bins (largest %d, %d above %d), %d groups (largest %d, %d above); info %d %d %d\n",
              bs[kNFine], nb, mx, big, kBinCap, ng, gmx, gbig, inf[0], inf[1], inf[2]);
      // the slowest waves of every chunk, with their groups
      std::vector<long long> wc8(nch * gcap * 8), wc(nch * gcap);
      std::vector<int4> ga(nch * gcap);
      if ((e = hipMemcpyAsync(wc8.data(), ws->wclk, sizeof(long long) * nch * gcap * 8, hipMemcpyDeviceToHost, s)) ||
          (e = hipMemcpyAsync(ga.data(), ws->gi4, sizeof(int4) * nch * gcap, hipMemcpyDeviceToHost, s)) ||
          (e = hipStreamSynchronize(s)))
        return e;
      std::vector<int64_t> ord(nch * gcap);
      for (int64_t i = 0; i < nch * gcap; i++) ord[i] = i, wc[i] = wc8[i * 8];
      std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return wc[a] > wc[b]; });
      double sum = 0, nlong = 0;
      for (long long v : wc) sum += (double)v;
      for (int64_t i = 0; i < nch * gcap; i++) nlong += (double)wc8[i * 8 + 7];
      fprintf(stderr, "[tfp] bin sort waves: %lld, mean %.0f cycles, long-run buckets %.0f\n", (long long)(nch * gcap),
              sum / (double)(nch * gcap), nlong);
      for (int i = 0; i < 12 && i < (int)ord.size(); i++) {
        const int4 q = ga[ord[i]];
        const long long* c = &wc8[ord[i] * 8];
        fprintf(stderr,
                "[tfp]   ch %lld g %lld: %lld cycles (kprev %lld, crowd copy %lld, dir %lld, lds %lld, regs %lld, crowd loop %lld; long-run buckets %lld), "
                "frames [%d, %d) (%d), first bin %d of %d\n",
                (long long)(ord[i] / gcap), (long long)(ord[i] % gcap), c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], q.x, q.y,
                q.y - q.x, q.z, q.w);
      }
    }
  } else {
    size_t tb = ws->tmp_bytes;
    if (packed) {
      if ((e = sweep_sort_keys<unsigned long long>(ws->tmp, tb, ws->ka, ws->kb, nf, end_bit, s))) return e;
    } else {
      if ((e = sweep_sort_pairs<unsigned long long>(ws->tmp, tb, ws->ka, ws->kb, ws->va, ws->vb, nf, end_bit, s))) return e;
    }
    const int32_t* order = ws->vb;
    if (speculative) {
      // every window at least dbase wide and no frame for the row scan, as the caller checks after
      // the results (info[1], info[2]); the kept-frame count stays on the device
      ws->min_width = dbase;
      ws->spec = true;
    } else {
      int32_t info[3] = {0, 0, 0};
      if ((e = hipMemcpyAsync(info, ws->info, sizeof info, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s))) return e;
      if (info[1] > 0) return hipSuccess;  // a frame for the row scan: the caller takes launch_scan
      ws->min_width = info[2] == 0 && dbase >= 0 ? dbase : -1;  // every window's U2 - L2 >= dbase
      if (info[2] > 0 || dbase < 0) {
        // a window width outside the delta field: sort by U2 first, then stably by (chunk, key, L2)
        if ((e = hipMemsetAsync(ws->info, 0, 3 * sizeof(int32_t), s))) return e;
        hipLaunchKernelGGL(wide_keys_u_kernel, dim3(grid_for(nf)), dim3(256), 0, s, boxes, nf, ws->ua, ws->va, ws->info);
        tb = ws->tmp_bytes;
        if ((e = sweep_sort_pairs<uint32_t>(ws->tmp, tb, ws->ua, ws->ub, ws->va, ws->vb, nf, 32, s))) return e;
        packed = false;  // (the U2 pre-sort's order: frame indices carried)
        hipLaunchKernelGGL(wide_keys_c_kernel, dim3(std::min(grid_for(nf), kKeysBlocks)), dim3(256), 0, s, boxes, ws->fq, nf, qch,
                           false, ws->vb, (int64_t)-1, ws->ka, (int32_t*)nullptr, ws->info, (uint32_t*)nullptr);
        tb = ws->tmp_bytes;
        if ((e = sweep_sort_pairs<unsigned long long>(ws->tmp, tb, ws->ka, ws->kb, ws->vb, ws->va, nf, kWideChunkShift + cb, s)))
          return e;
        order = ws->va;
      }
    }
    // (info[0] = the kept frames, read by the kernels below on the device; seg zeroed with the
    // frame -> query map)
    hipLaunchKernelGGL(wide_gather_kernel, dim3(grid_for(nf)), dim3(256), 0, s, boxes, ws->fq, ws->info, ws->kb, order, qch,
                       packed, dbase, ws->L2s, ws->U2s, ws->qis, ws->seg, nch, ws->cbeg);
    // the window segments' directories (sizes, offsets, then filled from the sorted frames)
    const int64_t nd = nch * kKeyRange + 1;
    (void)nd;
    hipLaunchKernelGGL(wide_dir_offsets_kernel, dim3(1), dim3(1024), 0, s, ws->seg, nch, ws->doff);
    hipLaunchKernelGGL(wide_dir_fill_kernel, dim3(grid_for(nf)), dim3(256), 0, s, ws->info, ws->kb,
                       packed ? kPackSegShift : kWideSegShift, ws->seg, ws->L2s, ws->U2s, ws->doff, ws->dtab, ws->segk);
  }
  if (qch == 256) {
    hipLaunchKernelGGL(wide_pcount_kernel<4>, dim3((unsigned)nch, kPortions / 16), dim3(1024), 0, s, ws->cbeg, ws->qis, ws->ptot);
    hipLaunchKernelGGL(wide_pscan_kernel, dim3((unsigned)nch), dim3(1024), 0, s, ws->ptot);
    hipLaunchKernelGGL(wide_prefix_kernel<4>, dim3((unsigned)nch, kPortions / 16), dim3(1024), 0, s, ws->cbeg, ws->qis, ws->ptot,
                       ws->P);
  } else {
    hipLaunchKernelGGL(wide_pcount_kernel<2>, dim3((unsigned)nch, kPortions / 16), dim3(1024), 0, s, ws->cbeg, ws->qis, ws->ptot);
    hipLaunchKernelGGL(wide_pscan_kernel, dim3((unsigned)nch), dim3(1024), 0, s, ws->ptot);
    hipLaunchKernelGGL(wide_prefix_kernel<2>, dim3((unsigned)nch, kPortions / 16), dim3(1024), 0, s, ws->cbeg, ws->qis, ws->ptot,
                       ws->P);
  }
  if ((e = hipGetLastError())) return e;
  *eligible = true;
  return hipSuccess;
}

hipError_t launch_scan_wide(int32_t nq, int64_t nf, const CellCache* cells, const int32_t* d_tiekey, int32_t C,
                            WideScratch* ws, unsigned long long* d_best, hipStream_t s, int32_t* d_info_out,
                            bool* info_written, int32_t col_base) {
  if (info_written) *info_written = false;
  if (nq <= 0 || !cells || !cells->valid || !cells->k_gbeg) return hipErrorInvalidValue;
  (void)nf;
  const int64_t nch = (nq + ws->qch - 1) / ws->qch;
  if (!cells->kdir) return hipErrorInvalidValue;
  CellView cv;
  memset(&cv, 0, sizeof cv);
  cv.g_key = cells->g_key;
  // clusters when every window of the batch is at least dgap wide (CellCache), else points
  if (cells->c_beg && !ws->points_only && (cells->dgap == 0 || (ws->min_width >= 0 && ws->min_width >= cells->dgap))) {
    cv.p_m2 = cells->c_lo;
    cv.p_hi = cells->c_hi;
    cv.g_beg = cells->c_beg;
  } else {
    cv.p_m2 = cells->p_m2;
    cv.p_hi = cells->p_m2;
    cv.g_beg = cells->g_beg;
  }
  cv.valid = 1;
  // xw waves per chunk (a multiple of the workgroup's), ~32 k waves in all
  int64_t xw = std::max<int64_t>(1, 32768 / nch);
  // (256-query chunks: half the chunks, so up to twice the waves per chunk, ~32 k in all)
  const int64_t xcap = std::min<int64_t>(2 * kPartWaves, (int64_t)kPartWaves * (ws->qch / kWideCh));
  xw = std::min<int64_t>(xw, std::min<int64_t>(xcap, cells->nwin));
  xw = std::max<int64_t>(kClipWaves, (xw + kClipWaves - 1) / kClipWaves * kClipWaves);
  // (TFP_DEBUG_BINS with a -DTFP_BIN_CLOCKS=1 build: the sweep's wave clocks in the bin sort's clock buffer)
  long long* clk = TFP_BIN_CLOCKS && ws->debug_bins && ws->wclk && 2 * nch * xw <= 8 * ws->cap_groups ? ws->wclk : nullptr;
  if (!ws->ukeys_ready) hipLaunchKernelGGL(wide_ukeys_kernel, dim3((unsigned)nch), dim3(1024), 0, s, ws->seg, ws->ukeys, ws->nuk);
  if (ws->qch == 256) {
    hipLaunchKernelGGL(wide_clips_kernel<4>, dim3((unsigned)(nch * xw / kClipWaves)), dim3(64 * kClipWaves), 0, s, (int32_t)xw,
                       ws->seg, ws->cbeg, cv, cells->kdir, cells->nwin, ws->ukeys, ws->nuk, ws->L2s, ws->U2s, ws->P, ws->qis, d_tiekey,
                       C, ws->segk, ws->dtab, ws->part, ws->ukeys_ready ? ws->info : nullptr, col_base, clk);
    hipLaunchKernelGGL(wide_part_max_kernel<4>, dim3((unsigned)nch, 8), dim3(1024), 0, s, ws->part, (int32_t)(xw / kClipWaves),
                       nq, d_best, ws->info, d_info_out);
  } else {
    hipLaunchKernelGGL(wide_clips_kernel<2>, dim3((unsigned)(nch * xw / kClipWaves)), dim3(64 * kClipWaves), 0, s, (int32_t)xw,
                       ws->seg, ws->cbeg, cv, cells->kdir, cells->nwin, ws->ukeys, ws->nuk, ws->L2s, ws->U2s, ws->P, ws->qis, d_tiekey,
                       C, ws->segk, ws->dtab, ws->part, ws->ukeys_ready ? ws->info : nullptr, col_base, clk);
    hipLaunchKernelGGL(wide_part_max_kernel<2>, dim3((unsigned)nch, 4), dim3(1024), 0, s, ws->part, (int32_t)(xw / kClipWaves),
                       nq, d_best, ws->info, d_info_out);
  }
  if (clk) {  // (TFP_DEBUG_BINS) the sweep's wave clocks: their spread
    const int64_t nw = nch * xw;
    std::vector<long long> wc(2 * nw);
    hipError_t e;
    if ((e = hipMemcpyAsync(wc.data(), clk, sizeof(long long) * 2 * nw, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
      return e;
    std::vector<long long> c(nw);
    for (int64_t i = 0; i < nw; i++) c[i] = wc[2 * i];
    std::vector<long long> o = c;
    std::sort(o.begin(), o.end());
    double sum = 0;
    for (long long v : c) sum += (double)v;
    fprintf(stderr, "[tfp] clip sweep waves: %lld, mean %.0f, p50 %lld, p90 %lld, p99 %lld, max %lld cycles\n", (long long)nw,
            sum / (double)nw, o[nw / 2], o[nw * 9 / 10], o[nw * 99 / 100], o[nw - 1]);
    // the slowest waves' chunk and window share
    std::vector<int64_t> ix(nw);
    for (int64_t i = 0; i < nw; i++) ix[i] = i;
    std::partial_sort(ix.begin(), ix.begin() + std::min<int64_t>(8, nw), ix.end(), [&](int64_t a, int64_t b) { return c[a] > c[b]; });
    for (int i = 0; i < 8 && i < nw; i++)
      fprintf(stderr, "[tfp]   wave %lld (chunk %lld, share %lld): %lld cycles\n", (long long)ix[i], (long long)(ix[i] / xw),
              (long long)(ix[i] % xw), c[ix[i]]);
  }
  if (info_written) *info_written = d_info_out != nullptr;
  return hipGetLastError();
}

}  // namespace tfp
