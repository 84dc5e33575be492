// tfp_log.hpp — the 8 kHz throughput kernel's band log (device code; included by tfp_kernels.hip
// and tests/native/check_log_fast.hip): aubio_log10_fast (tfp_math.hpp) with fewer instructions.
//
//   * glibc log10f's argument split (k = unbiased exponent, i = k < 0, m = the mantissa with
//     exponent 0x7f - i, y = k + i; the 2^25 rescale of subnormals) is v_frexp: a = mt 2^e with
//     mt in [0.5, 1), so k = e - 1 and, with c = (e >= 1), m = mt 2^c and y = e - c, exactly;
//   * logf's y0 = logc + k Ln2 (k in {-1, 0, 1} on [0.5, 2)) comes from a 64-entry table indexed
//     by bits 19..24 of tmp = bits(m) - 0x3f330000, built with the same double operations, and
//     so does invc 2^-k: logf's z = m 2^-k (its exponent-field subtraction) then times invc is the
//     same real product as m times invc 2^-k, both exact scalings, so r rounds identically.
// tests/native/check_log_fast.hip compares it with aubio_log10_fast on the GPU for every
// non-negative finite float.
#pragma once
#include <hip/hip_runtime.h>

#include "tfp_math.hpp"

namespace tfp {

constexpr int kLogf2Entries = 64;

// Entry idx of the 64-entry table: (invc 2^-k, y0) of logf_glibc's table entry idx & 15 and its
// exponent k = bits 23..24 of tmp as a signed field (idx >> 4: 0 -> 0, 1 -> 1, 3 -> -1; 2 is
// unused). y0 = logc + (double)k * Ln2, the two roundings of logf_glibc.
__device__ inline LogfEntry logf2_entry(int idx, const LogfEntry* T16) {
  const double Ln2 = 0x1.62e42fefa39efp-1;
  const LogfEntry e = T16[idx & 15];
  const int k = ((idx >> 4) ^ 2) - 2;
  return LogfEntry{e.invc * (k == 1 ? 0.5 : k == -1 ? 2.0 : 1.0), e.logc + (double)k * Ln2};
}

// == aubio_log10_fast(x) for every x >= +0 (finite; the filterbank sums). T64: logf2_entry(0..63).
// In two halves, so a caller with several logs can issue all their table reads before it needs
// any of them: log_reduce (argument split + table index) and log_finish.
struct LogArg {
  float y;       // glibc's y = k + i
  float m;       // glibc's x, logf's argument in [0.5, 2)
  uint32_t idx;  // table index
};
__device__ __forceinline__ LogArg log_reduce(float x) {
  const float c = (float)2.e-42;
  const float a = x > c ? x : c;  // aubio's clamp (a double compare, equal to this for any non-NaN x)
  const int e = __builtin_amdgcn_frexp_expf(a);
  const float mt = __builtin_amdgcn_frexp_mantf(a);
  const int c1 = min(max(e, 0), 1);
  const float m = __builtin_amdgcn_ldexpf(mt, c1);  // glibc's x (exact)
  const uint32_t ix = f2u(m);
  const uint32_t tmp = ix - 0x3f330000u;
  return LogArg{(float)(e - c1), m, (tmp >> 19) & 63u};
}
__device__ __forceinline__ float log_finish(const LogArg& g, const LogfEntry& en) {
  const float ivln10 = 4.3429449201e-01f, log10_2hi = 3.0102920532e-01f, log10_2lo = 7.9034151668e-07f;
  const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
  const double r = (double)g.m * en.invc - 1.0;  // en.invc holds invc 2^-k
  const double r2 = r * r;
  double yy = A1 * r + A2;
  yy = A0 * r2 + yy;
  yy = yy * r2 + (en.logc + r);  // en.logc holds y0
  const float l = (float)yy;
  const float zz = g.y * log10_2lo + ivln10 * l;
  return zz + g.y * log10_2hi;
}
__device__ __forceinline__ float aubio_log10_frexp(float x, const LogfEntry* T64) {
  const LogArg g = log_reduce(x);
  return log_finish(g, T64[g.idx]);
}

}  // namespace tfp
