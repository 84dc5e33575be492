// tfp_bsearch.hpp — the sweep's searches in a directory bucket of sorted window bounds
// (tfp_scan.hip find_ab; tests/native/check_bsearch.cpp checks them against std::lower_bound /
// std::upper_bound).
//
// A bucket may hold a crowd of equal values (the silence floor: thousands of frames of one chunk
// at C3), and a wave's search takes as many dependent probes as its slowest lane. The first probe
// reads both ends (two independent loads, one latency): a bucket that lies wholly on one side of v
// (a crowd always does) ends the search there instead of after log2 n probes, and otherwise the
// answer lies strictly inside, as after a bisection step.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define TFP_BS_HD __host__ __device__ inline
#else
#define TFP_BS_HD static inline
#endif

namespace tfp {

// first i in [0, n) with a[i] > v (n if none); a ascending
TFP_BS_HD int32_t ub32(const int32_t* a, int32_t n, int32_t v) {
  if (n <= 0) return 0;
  const int32_t x0 = a[0], xl = a[n - 1];
  // all <= v: n; all > v: 0; else a[0] <= v < a[n - 1] and the answer lies in [1, n - 1]
  int32_t lo = xl <= v ? n : x0 > v ? 0 : 1;
  int32_t hi = (xl <= v || x0 > v) ? lo : n - 1;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// first i in [0, n) with a[i] >= v (n if none); a ascending
TFP_BS_HD int32_t lb32(const int32_t* a, int32_t n, int32_t v) {
  if (n <= 0) return 0;
  const int32_t x0 = a[0], xl = a[n - 1];
  // all >= v: 0; all < v: n; else a[0] < v <= a[n - 1] and the answer lies in [1, n - 1]
  int32_t lo = x0 >= v ? 0 : xl < v ? n : 1;
  int32_t hi = (x0 >= v || xl < v) ? lo : n - 1;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

}  // namespace tfp
