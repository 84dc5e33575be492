// tfp_split.hpp — the 8 kHz kernel's real split per conjugate pair, as packed pairs over the two
// bins (device code; included by tfp_kernels.hip and tests/native/check_fast_sqrt.hip).
//
// A lane holds Z[k] = y and Z[256 - k] = p of the 256-point complex FFT. The spec's split
// ("Canonical FFT") of bin k is E = (a + Px, b - Py), O = (a - Px, b + Py),
// T = (O.re wy + O.im wx, O.im wy - O.re wx) with w = w512^k, S = E + T = 2X, and bin k' = 256 - k
// uses the exact sign flips E' = (E.re, -E.im), O' = (-O.re, O.im) with w' = w512^k'. Below,
// lane 0 of every packed value is bin k and lane 1 is bin k': each v_pk_* lane performs exactly
// the spec's scalar operation for its bin (x - y == x + (-y) and (-a) b == -(a b) bitwise, a
// product times +-1 is exact, so fma(a, +-1, c) is the plain c +- a), and no value is negated
// or moved between register halves.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tfp {

typedef float cf2 __attribute__((ext_vector_type(2)));

// (|S_k|^2, |S_k'|^2) with S = 2X: (fl(S.re^2) + fl(S.im^2)) per bin.
//   WX = (re w512^k, re w512^k'), WY = (im w512^k, im w512^k').
__device__ __forceinline__ cf2 split_pair_sq(cf2 y, cf2 p, cf2 WX, cf2 WY) {
  const cf2 E = __builtin_elementwise_fma(p, cf2{1.f, -1.f}, y);  // (a + Px, b - Py)
  const cf2 O = __builtin_elementwise_fma(p, cf2{-1.f, 1.f}, y);  // (a - Px, b + Py)
  const cf2 A1 = cf2{O.x, O.x} * WY;  // (O.re wy, O.re wy')
  const cf2 A2 = cf2{O.y, O.y} * WX;  // (O.im wx, O.im wx')
  const cf2 A3 = cf2{O.y, O.y} * WY;  // (O.im wy, O.im wy')
  const cf2 A4 = cf2{O.x, O.x} * WX;  // (O.re wx, O.re wx')
  // T.re = O.re wy + O.im wx;      T'.re = (-O.re) wy' + O.im wx'
  const cf2 TR = __builtin_elementwise_fma(A1, cf2{1.f, -1.f}, A2);
  // T.im = O.im wy - O.re wx;      T'.im = O.im wy' - (-O.re) wx'
  const cf2 TI = __builtin_elementwise_fma(A4, cf2{-1.f, 1.f}, A3);
  const cf2 SR = cf2{E.x, E.x} + TR;                                        // E.re + T.re, E.re + T'.re
  const cf2 SI = __builtin_elementwise_fma(cf2{E.y, E.y}, cf2{1.f, -1.f}, TI);  // E.im + T.im, -E.im + T'.im
  return SR * SR + SI * SI;
}

// Both bins: n = m + med3(bits(rp), 0, 1) + med3(bits(rm), 0, 1) on the bit patterns (med3 = 1 iff
// the float is > 0, not a negative NaN). One asm block: the compiler's own form of the clamps is a
// compare, a select and an add-with-carry per bin, and every separate asm block gets a hazard
// s_nop before its VALU consumer; here the only consumers are the caller's ds_writes. a0 is
// early-clobber too: it is written before the last instruction reads m1 (sharing a register
// with m1, which the allocator chose under the 12-wave build's 168-VGPR budget, it gave bin
// 256 - k the bits of bin k).
__device__ __forceinline__ void step_tuckerman(uint32_t m0, uint32_t m1, cf2 rp, cf2 rm, float& n0, float& n1) {
  uint32_t a0, a1, t0, t1, u0, u1;
  asm("v_med3_i32 %2, %6, 0, 1\n\t"
      "v_med3_i32 %3, %8, 0, 1\n\t"
      "v_med3_i32 %4, %7, 0, 1\n\t"
      "v_med3_i32 %5, %9, 0, 1\n\t"
      "v_add3_u32 %0, %10, %2, %3\n\t"
      "v_add3_u32 %1, %11, %4, %5"
      : "=&v"(a0), "=v"(a1), "=&v"(t0), "=&v"(t1), "=&v"(u0), "=&v"(u1)
      : "v"(rp.x), "v"(rp.y), "v"(rm.x), "v"(rm.y), "v"(m0), "v"(m1));
  n0 = __builtin_bit_cast(float, a0);
  n1 = __builtin_bit_cast(float, a1);
}
// The kernel's rare-bin key of a pair: min over both bins of bits(|S|^2) - 1 (exact zeros wrap to
// the top), so a wave holds a bin with 0 < |S|^2 < thr iff its min key < bits(thr) - 1. The
// elements go through scalars first: clang's __builtin_bit_cast of an ext_vector element
// expression (`sq.y`) reads element 0, which left every bin 256 - k out of the test.
__device__ __forceinline__ uint32_t rare_key_pair(cf2 sq) {
  const float a = sq.x, b = sq.y;
  return min(__builtin_bit_cast(uint32_t, a) - 1u, __builtin_bit_cast(uint32_t, b) - 1u);
}

// Correctly rounded sqrtf of x (= SSE sqrtss, glibc's sqrtf) for x = 0 and x in [2^-100, 2^100):
// v_sqrt_f32 (within 1 ulp) moved to the neighbour whose Tuckerman interval holds x:
//   +1 ulp when x - yp y > 0, -1 ulp when x - ym y <= 0 (ym, yp: y's neighbours),
// on the bit patterns as ym + med3(bits(rp), 0, 1) + med3(bits(rm), 0, 1) — a float's bits
// order as a signed integer, +0 is 0. x = 0: y = 0, rp = +0, ym's bits wrap to a NaN whose
// negation (the fma's neg modifier) is positive, so rm is a positive NaN: 0xffffffff + 0 + 1 = 0.
// (tests/native/check_fast_sqrt.hip runs this on the GPU over every float in range.)
// (v_sqrt_f32 returns 0 for denormal x, so the caller sends 0 < x < 2^-98 to its slow path by x.)
__device__ __forceinline__ void sqrt_pair_cr(cf2 x, float& n0, float& n1) {
  const uint32_t b0 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_sqrtf(x.x));
  const uint32_t b1 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_sqrtf(x.y));
  const uint32_t m0 = b0 - 1u, m1 = b1 - 1u;
  const cf2 yy = {__builtin_bit_cast(float, b0), __builtin_bit_cast(float, b1)};
  const cf2 ym = {__builtin_bit_cast(float, m0), __builtin_bit_cast(float, m1)};
  const cf2 yp = {__builtin_bit_cast(float, b0 + 1u), __builtin_bit_cast(float, b1 + 1u)};
  const cf2 rm = __builtin_elementwise_fma(-ym, yy, x);
  const cf2 rp = __builtin_elementwise_fma(-yp, yy, x);
  step_tuckerman(m0, m1, rp, rm, n0, n1);
}

}  // namespace tfp
