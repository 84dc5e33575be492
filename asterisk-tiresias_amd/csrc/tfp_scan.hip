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

#include "tfp_kernels.hpp"
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

void CellCache::release() {
  for (void* p : {(void*)p_m2, (void*)g_key, (void*)g_beg, (void*)e_key, (void*)e_grp})
    if (p) (void)hipFree(p);
  p_m2 = nullptr;
  g_key = nullptr;
  g_beg = nullptr;
  e_key = nullptr;
  e_grp = nullptr;
  S = n1 = n2 = 0;
  valid = false;
}

hipError_t CellCache::build(const int64_t* d_rng_all, const int64_t* h_off, const int32_t* m2s, const int32_t* cols,
                            int32_t ncols, int64_t nrows, double tole, hipStream_t s) {
  release();
  S = h_off[kKeyRange];
  // limits of the packed keys and of hipcub's 32-bit counts; beyond them every frame takes the
  // row scan (correct, slower)
  if (!(tole >= 0.0 && tole < 1e6) || ncols > kMaxCols || S <= 0 || 2 * S >= INT32_MAX || S > 4 * nrows + (1 << 20)) {
    S = 0;
    return hipSuccess;
  }
  w = (int64_t)ceil(2.0 * tole * 1e6) + 4;  // >= U2 - L2 of every fmt6 max2 window at this tolerance
  hipError_t e;
  int64_t* d_off = nullptr;
  unsigned long long *ka = nullptr, *kb = nullptr, *ea = nullptr, *eb = nullptr;
  uint32_t* k32 = nullptr;
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
  hipLaunchKernelGGL(cells_fill_kernel, dim3(grid_for(S)), dim3(256), 0, s, d_rng_all, d_off, m2s, cols, S, ka);
  TFP_TRY(hipGetLastError());
  // (key, col, m2) order: the groups, each group's points ascending
  TFP_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, t1, ka, kb, (int)S, 0, 63, s));
  tb = t1;
  TFP_TRY(hipcub::DeviceRunLengthEncode::Encode(nullptr, t1, k32, k32, glen, d_n, (int)S, s));
  tb = t1 > tb ? t1 : tb;
  TFP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, t1, ea, eb, ga, gb, (int)(2 * S), 0, 62, s));
  tb = t1 > tb ? t1 : tb;
  TFP_TRY(hipcub::DeviceSelect::UniqueByKey(nullptr, t1, eb, gb, ea, ga, d_n + 1, (int)(2 * S), s));
  tb = t1 > tb ? t1 : tb;
  TFP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, glen, glen, (int)S, s));
  tb = t1 > tb ? t1 : tb;
  TFP_TRY(hipMalloc(&tmp, tb > 0 ? tb : 1));
  TFP_TRY(hipcub::DeviceRadixSort::SortKeys(tmp, tb, ka, kb, (int)S, 0, 63, s));
  TFP_TRY(dmalloc(&p_m2, S));
  TFP_TRY(dmalloc(&k32, S));
  hipLaunchKernelGGL(cells_split_kernel, dim3(grid_for(S)), dim3(256), 0, s, kb, S, p_m2, k32);
  TFP_TRY(hipGetLastError());
  (void)hipFree(ka);
  (void)hipFree(kb);
  ka = kb = nullptr;
  TFP_TRY(dmalloc(&g_key, S));
  TFP_TRY(dmalloc(&glen, S + 1));
  TFP_TRY(hipcub::DeviceRunLengthEncode::Encode(tmp, tb, k32, g_key, glen, d_n, (int)S, s));
  TFP_TRY(hipMemcpyAsync(nn, d_n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TFP_TRY(hipStreamSynchronize(s));
  n1 = nn[0];
  // group offsets: exclusive sum of the run lengths, g_beg[n1] = S
  TFP_TRY(dmalloc(&g_beg, n1 + 1));
  TFP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, glen, g_beg, (int)n1, s));
  TFP_TRY(hipMemcpyAsync(g_beg + n1, &S, sizeof(int32_t), hipMemcpyHostToDevice, s));  // S < 2^31
  (void)hipFree(glen);
  glen = nullptr;
  TFP_TRY(dmalloc(&ea, 2 * S));
  TFP_TRY(dmalloc(&eb, 2 * S));
  TFP_TRY(dmalloc(&ga, 2 * S));
  TFP_TRY(dmalloc(&gb, 2 * S));
  hipLaunchKernelGGL(cells_entries_kernel, dim3(grid_for(S)), dim3(256), 0, s, p_m2, k32, S, g_key, n1, w, ea, ga);
  TFP_TRY(hipGetLastError());
  TFP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, ea, eb, ga, gb, (int)(2 * S), 0, 62, s));
  TFP_TRY(hipcub::DeviceSelect::UniqueByKey(tmp, tb, eb, gb, ea, ga, d_n + 1, (int)(2 * S), s));
  TFP_TRY(hipMemcpyAsync(nn + 1, d_n + 1, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TFP_TRY(hipStreamSynchronize(s));
  n2 = nn[1];
  e_key = ea;
  e_grp = ga;
  ea = nullptr;
  ga = nullptr;
  valid = true;
out:
#undef TFP_TRY
  for (void* p : {(void*)d_off, (void*)ka, (void*)kb, (void*)ea, (void*)eb, (void*)k32, (void*)glen, (void*)ga,
                  (void*)gb, (void*)d_n, tmp})
    if (p) (void)hipFree(p);
  if (e != hipSuccess) release();
  return e;
}

namespace {

// ---- search kernels -----------------------------------------------------------------------

struct CellView {
  const int32_t* p_m2;
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

}  // namespace tfp
