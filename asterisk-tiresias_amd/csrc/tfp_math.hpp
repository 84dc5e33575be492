// tfp_math.hpp — exact scalar math shared by the host engine and the gfx950 kernels.
//
// Everything here is written with IEEE-754 basic operations only (+ - * / sqrt, fma where
// written explicitly, rint), so it evaluates bit-identically on x86-64 and on gfx950 when
// built with -ffp-contract=off (see Makefile). No libm/ocml calls.
//
// Functions and the reference behaviour they reproduce:
//   tfp_log10f()   == glibc 2.35 log10f, bit for bit, for every positive float.
//                     The reference applies it per mel band via aubio's fvec_log10
//                     (libaubio mathutils.c, called from aubio_mfcc_do; call site
//                     /root/reference/src/fp_handler.c:642). glibc 2.35 log10f is the fdlibm
//                     float wrapper around ARM-optimized-routines logf; both are restated
//                     below. Verified exhaustively on all 2^24 mantissas of [0.5,2) for logf
//                     and on 713 M sampled floats for log10f (tests/test_math_exact.py).
//   tfp_log10()    glibc 2.35 log10 wrapper (fdlibm e_log10.c) around an own near-CR log;
//                  used for `10*log10(fabs(c))` (/root/reference/src/fp_handler.c:651).
//                  Its callers only consume fmt6()/trunc of 10*log10(); agreement with glibc
//                  at that granularity is checked exhaustively over all floats c.
//   tfp_fmt6()     printf("%f") of a double = round-half-even of the EXACT binary value to
//                  6 decimals, returned as integer micro-units. The reference stores every
//                  fingerprint value through "%f" (/root/reference/src/db_ctx_handler.c:479-481)
//                  and prints search bounds through "%f" (/root/reference/src/fp_handler.c:308-314,
//                  339-347); SQLite then compares the parsed decimals, which orders exactly as
//                  these integers do.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define TFP_HD __host__ __device__ inline
#else
#define TFP_HD static inline
#endif

namespace tfp {

TFP_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
TFP_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
TFP_HD uint64_t d2u(double d) { return __builtin_bit_cast(uint64_t, d); }
TFP_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }

// Micro-unit sentinel for a value the reference stores as SQL NULL (json_real(±inf) → NULL,
// /root/reference/src/fp_handler.c:651 + jansson). Valid fingerprints are within ±4.6e8.
constexpr int32_t kNullMicro = INT32_MIN;

// ---------------------------------------------------------------------------------------
// glibc 2.35 logf (ARM optimized-routines, LOGF_TABLE_BITS = 4), restated. The double-typed
// evaluation below is the non-FMA form; on [0.5,2) it equals the FMA form bit for bit
// (checked exhaustively), which is the only range tfp_log10f() feeds it.
struct LogfEntry { double invc, logc; };
#if defined(__HIPCC__) || defined(__HIP__)
__host__ __device__
#endif
inline const LogfEntry* logf_table() {
  static constexpr LogfEntry T[16] = {
      {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
      {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
      {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
      {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
      {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
      {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
      {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
      {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
  };
  return T;
}

// Valid for positive normal finite x (tfp_log10f only passes [0.5, 2)). T: the 16-entry table
// (device code passes a copy staged in LDS).
TFP_HD float logf_glibc(float x, const LogfEntry* T = logf_table()) {
  const double Ln2 = 0x1.62e42fefa39efp-1;
  const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
  const uint32_t ix = f2u(x);
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) & 15u);
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & 0xff800000u);
  const LogfEntry e = T[i];
  const double z = (double)u2f(iz);
  const double r = z * e.invc - 1.0;
  const double y0 = e.logc + (double)k * Ln2;
  const double r2 = r * r;
  double y = A1 * r + A2;
  y = A0 * r2 + y;
  y = y * r2 + (y0 + r);
  return (float)y;
}

// glibc 2.35 log10f = fdlibm e_log10f.c float wrapper (all float arithmetic).
TFP_HD float log10f_glibc(float x, const LogfEntry* T = logf_table()) {
  const float two25 = 3.3554432000e+07f, ivln10 = 4.3429449201e-01f;
  const float log10_2hi = 3.0102920532e-01f, log10_2lo = 7.9034151668e-07f;
  int32_t hx = (int32_t)f2u(x);
  int32_t k = 0;
  if (hx < 0x00800000) {
    if ((hx & 0x7fffffff) == 0) return -u2f(0x7f800000u);  // -inf
    if (hx < 0) return u2f(0x7fc00000u);                    // NaN
    k -= 25;
    x *= two25;
    hx = (int32_t)f2u(x);
  }
  if (hx >= 0x7f800000) return x + x;
  k += (hx >> 23) - 127;
  const int32_t i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
  hx = (hx & 0x007fffff) | ((0x7f - i) << 23);
  const float y = (float)(k + i);
  x = u2f((uint32_t)hx);
  const float z = y * log10_2lo + ivln10 * logf_glibc(x, T);
  return z + y * log10_2hi;
}

// aubio fvec_log10: LOG10(MAX(VERY_SMALL_NUMBER, x)), VERY_SMALL_NUMBER = 2.e-42 (a double
// literal, so the comparison is done in double and the clamp value is (float)2e-42).
TFP_HD float aubio_log10_clamped(float x, const LogfEntry* T = logf_table()) {
  const double v = 2.e-42;
  const double xd = (double)x;
  const float a = (float)((v > xd) ? v : xd);
  return log10f_glibc(a, T);
}

// aubio_log10_clamped for the filterbank sums (finite, >= -0), branch-free. For any non-NaN
// float x the double-precision clamp (2e-42 > (double)x ? (float)2e-42 : x) equals
// max(x, (float)2e-42), after which the only special case of log10f left is a subnormal
// argument (rescaled by 2^25 under a select). Bit-identical to aubio_log10_clamped on every
// non-negative float (tests/native/check_math.cpp #5, exhaustive log committed).
TFP_HD float aubio_log10_fast(float x, const LogfEntry* T = logf_table()) {
  const float two25 = 3.3554432000e+07f, ivln10 = 4.3429449201e-01f;
  const float log10_2hi = 3.0102920532e-01f, log10_2lo = 7.9034151668e-07f;
  const float c = (float)2.e-42;
  float a = x > c ? x : c;
  const bool den = f2u(a) < 0x00800000u;
  a = den ? a * two25 : a;
  int32_t hx = (int32_t)f2u(a);
  const int32_t k = (den ? -25 : 0) + (hx >> 23) - 127;
  const int32_t i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
  hx = (hx & 0x007fffff) | ((0x7f - i) << 23);
  const float y = (float)(k + i);
  const float z = y * log10_2lo + ivln10 * logf_glibc(u2f((uint32_t)hx), T);
  return z + y * log10_2hi;
}

// ---------------------------------------------------------------------------------------
// Near-correctly-rounded natural log for x in [0.5, 2): reduce to [sqrt(1/2), sqrt(2)),
// log(m) = 2 atanh(s), s = (m-1)/(m+1) kept as a double-double, series tail in double.
// Relative error ~2^-59, so it rounds to the CR double except within ~2^-59 of a midpoint.
TFP_HD double log_acc(double x) {
  const double SQRT2 = 0x1.6a09e667f3bcdp+0, SQRT1_2 = 0x1.6a09e667f3bcdp-1;
  const double LN2_HI = 0x1.62e42fefa3800p-1;   // 43 significant bits: j*LN2_HI exact
  const double LN2_LO = 0x1.ef35793c7673p-45;
  double j = 0.0;
  if (x > SQRT2) { x = x * 0.5; j = 1.0; }
  else if (x < SQRT1_2) { x = x * 2.0; j = -1.0; }
  const double f = x - 1.0;                       // exact (Sterbenz)
  const double dh = 2.0 + f;
  const double dl = (2.0 - dh) + f;               // exact (Fast2Sum, |2| >= |f|)
  const double sh = f / dh;
  double r = __builtin_fma(-sh, dh, f);           // exact remainder f - sh*dh
  r = r - sh * dl;
  const double sl = r / dh;
  const double w = sh * sh;
  // p = sum_{n=1..11} 2/(2n+1) w^n
  double p = 2.0 / 23.0;
  p = p * w + 2.0 / 21.0;
  p = p * w + 2.0 / 19.0;
  p = p * w + 2.0 / 17.0;
  p = p * w + 2.0 / 15.0;
  p = p * w + 2.0 / 13.0;
  p = p * w + 2.0 / 11.0;
  p = p * w + 2.0 / 9.0;
  p = p * w + 2.0 / 7.0;
  p = p * w + 2.0 / 5.0;
  p = p * w + 2.0 / 3.0;
  p = p * w;
  const double tail = sh * p;
  const double hi = 2.0 * sh;                     // exact
  const double lo = 2.0 * sl + tail + j * LN2_LO;
  const double a = j * LN2_HI;                    // exact
  const double s = a + hi;                        // TwoSum(a, hi)
  const double bb = s - a;
  const double err = (a - (s - bb)) + (hi - bb);
  return s + (err + lo);
}

// glibc's inner log differs from log_acc on 58,054 of the 2^24 reduced arguments the wrapper
// below can see for a float input (the double of a float has 29 zero low mantissa bits; the
// reduced argument is its mantissa in [1, 2) or [0.5, 1)). LogFix lists them, keyed
// i << 23 | mantissa23 (i = 1 for [0.5, 1)), with glibc's value: built on the host from glibc
// itself (tfp_tables.cpp build_log_fix), ascending keys. n = 0: no table (log_acc everywhere).
// hashed: key/val are instead the 2^kLogFixHashBits slots of tfp_tables.cpp log_fix_hash (the
// device copy: at load 0.44 a lookup, hit or miss, reads one or two adjacent keys).
constexpr int kLogFixHashBits = 17;
constexpr uint32_t kLogFixEmpty = 0xffffffffu;
TFP_HD uint32_t log_fix_slot(uint32_t k) { return (k * 0x9E3779B1u) >> (32 - kLogFixHashBits); }
struct LogFix {
  const uint32_t* key;
  const double* val;
  int32_t n;
  int32_t hashed = 0;
  const uint32_t* bits = nullptr;  // (hashed) the keys present, one bit each over the 2^24 domain
};

TFP_HD double log_fixed(double x, int32_t i, const LogFix& fx) {
  if (fx.n > 0 && (d2u(x) & 0x1fffffffull) == 0) {  // (a float's double: the table's domain)
    const uint32_t k = ((uint32_t)i << 23) | (uint32_t)((d2u(x) >> 29) & 0x7fffffu);
    if (fx.hashed) {
      // one load decides for the 99.65 % of arguments without an entry (the probes of a miss are
      // dependent loads: they cost more than the log itself)
      if (fx.bits && !((fx.bits[k >> 5] >> (k & 31)) & 1u)) return log_acc(x);
      for (uint32_t h = log_fix_slot(k);; h = (h + 1) & ((1u << kLogFixHashBits) - 1)) {
        const uint32_t s = fx.key[h];
        if (s == k) return fx.val[h];
        if (s == kLogFixEmpty) break;
      }
      return log_acc(x);
    }
    int32_t lo = 0, hi = fx.n;
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      if (fx.key[mid] < k) lo = mid + 1; else hi = mid;
    }
    if (lo < fx.n && fx.key[lo] == k) return fx.val[lo];
  }
  return log_acc(x);
}

// glibc 2.35 log10 = fdlibm e_log10.c wrapper; the inner log is log_acc() above, or glibc's own
// value where the LogFix table lists it (then the result is glibc's, bit for bit, for every
// double of a float: tests/native/check_logfix.cpp).
TFP_HD double log10_glibc_wrapper(double x, const LogFix& fx = LogFix{nullptr, nullptr, 0}) {
  const double two54 = 1.80143985094819840000e+16;
  const double ivln10 = 4.34294481903251816668e-01;
  const double log10_2hi = 3.01029995663611771306e-01;
  const double log10_2lo = 3.69423907715893078616e-13;
  uint64_t bits = d2u(x);
  int32_t hx = (int32_t)(bits >> 32);
  const uint32_t lx = (uint32_t)bits;
  int32_t k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -u2d(0x7ff0000000000000ull);
    if (hx < 0) return u2d(0x7ff8000000000000ull);
    k -= 54;
    x *= two54;
    bits = d2u(x);
    hx = (int32_t)(bits >> 32);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  const int32_t i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
  hx = (hx & 0x000fffff) | ((0x3ff - i) << 20);
  const double y = (double)(k + i);
  x = u2d(((uint64_t)(uint32_t)hx << 32) | (d2u(x) & 0xffffffffull));
  const double z = y * log10_2lo + ivln10 * log_fixed(x, i, fx);
  return z + y * log10_2hi;
}

// `10 * log10(fabs((double)c))` of /root/reference/src/fp_handler.c:651. Without a LogFix table
// the value may differ from glibc's in its last bit (152,867 floats), never in its "%f" micro-units
// or its truncation (what the stored rows and the max1 keys use); with the table it is glibc's.
TFP_HD double db_of_coef(float c, const LogFix& fx = LogFix{nullptr, nullptr, 0}) {
  const double a = (double)c;
  return 10.0 * log10_glibc_wrapper(a < 0.0 ? -a : a, fx);
}

// ---------------------------------------------------------------------------------------
// printf("%f") micro-units: round-half-even of the exact value x*1e6. Valid for |x| < 2^52/1e6
// (fingerprints are |x| < 460). two_prod(x, 1e6) = p + e exactly; only when p lands exactly on
// a half-integer does the sign of e decide.
TFP_HD int64_t fmt6(double x) {
  const double p = x * 1e6;
  const double e = __builtin_fma(x, 1e6, -p);
  double n = __builtin_rint(p);
  const double d = p - n;  // exact
  if (d == 0.5 || d == -0.5) {
    if (e > 0.0) n = p + 0.5;
    else if (e < 0.0) n = p - 0.5;
  }
  return (int64_t)n;
}

// fmt6 for a search bound that may be arbitrarily large (user tolerance): saturates far
// outside the range of any stored value, which preserves every comparison.
constexpr int64_t kBoundSat = (int64_t)1 << 60;
TFP_HD int64_t fmt6_bound(double x) {
  if (!(x < 1e12)) return kBoundSat;     // also +inf
  if (!(x > -1e12)) return -kBoundSat;   // also -inf
  return fmt6(x);
}

// Fingerprint value as stored: NULL when 10*log10|c| is ±inf/NaN (c == 0), else fmt6.
TFP_HD int32_t micro_of_db(double q) {
  const double inf = u2d(0x7ff0000000000000ull);
  if (!(q > -inf && q < inf)) return kNullMicro;
  return (int32_t)fmt6(q);
}

}  // namespace tfp
