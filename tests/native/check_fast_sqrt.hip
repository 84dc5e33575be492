// check_fast_sqrt.hip — exhaustive gfx950 check of the 8 kHz kernel's sqrt sequence
// (asterisk-tiresias_amd/csrc/tfp_split.hpp: sqrt_pair_cr) over every non-negative finite float:
//   * x = 0 and x in [2^-100, 2^100): the result equals the correctly rounded sqrtf, bitwise;
//   * 0 < x < 2^-98 (denormals included): the kernel's rare-bin flag (tfp_split.hpp:
//     rare_key_pair(pair) < bits(2^-98) - 1) is raised, so those bins take the spec-order slow
//     path, and it is not raised for x = 0 or the fast range; the pair key is checked with the
//     candidate in either element (bin k or bin 256 - k). Also counted: x whose v_sqrt_f32 is 0
//     (denormal inputs, flushed).
// The device's IEEE __builtin_sqrtf is the reference; it is pinned to the host's sqrtf (SSE
// sqrtss, glibc) on a strided sample copied back. Prints the counts; exit status 0 iff all are 0.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../asterisk-tiresias_amd/csrc/tfp_split.hpp"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 2;                                                                \
    }                                                                          \
  } while (0)

constexpr uint32_t kInf = 0x7f800000u;     // x bits in [0, kInf): every non-negative finite float
constexpr uint32_t kHalf = kInf / 2;       // lane 0 takes b, lane 1 takes b + kHalf
constexpr uint32_t kSampleStride = 1021;   // host pin of the device reference

struct Counts {
  unsigned long long fast_mismatch, rare_missed, rare_spurious, zero_bad, sqrt_flushed, checked, up, down;
};

__global__ void check_kernel(Counts* c, uint32_t rare_m1, float* sample) {
  unsigned long long bad = 0, missed = 0, spur = 0, zbad = 0, flushed = 0, n = 0, up = 0, down = 0;
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < kHalf; b += gridDim.x * blockDim.x) {
    const uint32_t bx[2] = {b, b + kHalf};
    const tfp::cf2 x = {__builtin_bit_cast(float, bx[0]), __builtin_bit_cast(float, bx[1])};
    float r[2];
    tfp::sqrt_pair_cr(x, r[0], r[1]);
    for (int i = 0; i < 2; i++) {
      const float xi = i ? x.y : x.x;
      const float ref = __builtin_sqrtf(xi);
      if (bx[i] % kSampleStride == 0) sample[bx[i] / kSampleStride] = ref;
      const bool fast = xi == 0.f || (xi >= 0x1p-100f && xi < 0x1p100f);
      if (fast && __builtin_bit_cast(uint32_t, r[i]) != __builtin_bit_cast(uint32_t, ref)) bad++;
      if (xi == 0.f && __builtin_bit_cast(uint32_t, r[i]) != 0u) zbad++;
      if (xi > 0.f && __builtin_amdgcn_sqrtf(xi) == 0.f) flushed++;
      if (fast && xi > 0.f) {  // which neighbour of v_sqrt_f32's result the correct rounding takes
        const uint32_t y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_sqrtf(xi)), c = __builtin_bit_cast(uint32_t, ref);
        up += c == y + 1u;
        down += c == y - 1u;
      }
      n++;
    }
    // fingerprint8k_kernel's rare test on the pair, with x.x (the low half's candidate; x.y is
    // never in (0, 2^-98)) as bin k and as bin 256 - k
    const bool want = (x.x > 0.f && x.x < 0x1p-98f) || (x.y > 0.f && x.y < 0x1p-98f);
    const bool f01 = tfp::rare_key_pair(x) < rare_m1, f10 = tfp::rare_key_pair(tfp::cf2{x.y, x.x}) < rare_m1;
    missed += (want && !f01) + (want && !f10);
    spur += (!want && f01) + (!want && f10);
  }
  if (bad) atomicAdd(&c->fast_mismatch, bad);
  if (missed) atomicAdd(&c->rare_missed, missed);
  if (zbad) atomicAdd(&c->zero_bad, zbad);
  if (spur) atomicAdd(&c->rare_spurious, spur);
  if (flushed) atomicAdd(&c->sqrt_flushed, flushed);
  if (up) atomicAdd(&c->up, up);
  if (down) atomicAdd(&c->down, down);
  atomicAdd(&c->checked, n);
}

int main() {
  // the kernel's threshold: bits(2^-98) - 1 (fingerprint8k_kernel's rare_m1)
  const float thr = 0x1p-98f;
  uint32_t rare_m1;
  memcpy(&rare_m1, &thr, 4);
  rare_m1 -= 1u;
  Counts* d_c;
  float* d_s;
  const size_t ns = kInf / kSampleStride + 1;
  CK(hipMalloc(&d_c, sizeof(Counts)));
  CK(hipMemset(d_c, 0, sizeof(Counts)));
  CK(hipMalloc(&d_s, ns * sizeof(float)));
  hipLaunchKernelGGL(check_kernel, dim3(8192), dim3(256), 0, 0, d_c, rare_m1, d_s);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  Counts c;
  CK(hipMemcpy(&c, d_c, sizeof c, hipMemcpyDeviceToHost));
  float* hs = new float[ns];
  CK(hipMemcpy(hs, d_s, ns * sizeof(float), hipMemcpyDeviceToHost));
  unsigned long long ref_bad = 0, nsample = 0;
  for (uint64_t b = 0; b < kInf; b += kSampleStride) {
    float x;
    const uint32_t bb = (uint32_t)b;
    memcpy(&x, &bb, 4);
    const float h = sqrtf(x);
    if (memcmp(&h, &hs[b / kSampleStride], 4) != 0) ref_bad++;
    nsample++;
  }
  delete[] hs;
  printf("checked %llu floats [0, inf): fast_mismatch %llu, zero_bad %llu, rare_missed %llu, "
         "rare_spurious %llu; v_sqrt_f32 returns 0 for %llu positive inputs; "
         "device sqrtf vs host sqrtf on %llu samples: %llu differ; v_sqrt_f32 one below the correctly rounded "
         "result on %llu fast-range inputs, one above on %llu\n",
         c.checked, c.fast_mismatch, c.zero_bad, c.rare_missed, c.rare_spurious, c.sqrt_flushed, nsample, ref_bad, c.up,
         c.down);
  (void)hipFree(d_c);
  (void)hipFree(d_s);
  const bool ok = c.checked == 2ull * kHalf && !c.fast_mismatch && !c.zero_bad && !c.rare_missed && !c.rare_spurious &&
                  !ref_bad;
  printf("%s\n", ok ? "OK" : "FAIL");
  return ok ? 0 : 1;
}
