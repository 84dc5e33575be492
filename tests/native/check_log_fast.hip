// check_log_fast.hip — exhaustive gfx950 check of the 8 kHz throughput kernel's band log
// (asterisk-tiresias_amd/csrc/tfp_log.hpp: aubio_log10_frexp) against aubio_log10_fast
// (tfp_math.hpp; itself bit-identical to aubio's clamped glibc log10f on every non-negative float,
// tests/native/check_math.cpp) over every non-negative finite float, both evaluated on the GPU.
// Prints the mismatch count and the first mismatches; exit status 0 iff there are none.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../asterisk-tiresias_amd/csrc/tfp_log.hpp"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 2;                                                                \
    }                                                                          \
  } while (0)

constexpr uint32_t kInf = 0x7f800000u;  // x bits in [0, kInf)

__global__ void table_kernel(tfp::LogfEntry* t64) {
  if (threadIdx.x < tfp::kLogf2Entries) t64[threadIdx.x] = tfp::logf2_entry(threadIdx.x, tfp::logf_table());
}

__global__ void check_kernel(const tfp::LogfEntry* t64, unsigned long long* counts, uint32_t* first) {
  __shared__ tfp::LogfEntry T16[16], T64[tfp::kLogf2Entries];
  if (threadIdx.x < 16) T16[threadIdx.x] = tfp::logf_table()[threadIdx.x];
  if (threadIdx.x < tfp::kLogf2Entries) T64[threadIdx.x] = t64[threadIdx.x];
  __syncthreads();
  unsigned long long bad = 0, n = 0;
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < kInf; b += gridDim.x * blockDim.x) {
    const float x = __builtin_bit_cast(float, b);
    const float r0 = tfp::aubio_log10_fast(x, T16), r1 = tfp::aubio_log10_frexp(x, T64);
    if (__builtin_bit_cast(uint32_t, r0) != __builtin_bit_cast(uint32_t, r1)) {
      const unsigned long long i = atomicAdd(&counts[0], 1ull);
      if (i < 8) first[i] = b;
      bad++;
    }
    n++;
  }
  atomicAdd(&counts[1], n);
  (void)bad;
}

int main() {
  tfp::LogfEntry* d_t;
  unsigned long long* d_c;
  uint32_t* d_f;
  CK(hipMalloc(&d_t, sizeof(tfp::LogfEntry) * tfp::kLogf2Entries));
  CK(hipMalloc(&d_c, 2 * sizeof(unsigned long long)));
  CK(hipMalloc(&d_f, 8 * sizeof(uint32_t)));
  CK(hipMemset(d_c, 0, 2 * sizeof(unsigned long long)));
  CK(hipMemset(d_f, 0, 8 * sizeof(uint32_t)));
  hipLaunchKernelGGL(table_kernel, dim3(1), dim3(64), 0, 0, d_t);
  CK(hipGetLastError());
  hipLaunchKernelGGL(check_kernel, dim3(8192), dim3(256), 0, 0, d_t, d_c, d_f);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  unsigned long long c[2];
  uint32_t f[8];
  CK(hipMemcpy(c, d_c, sizeof c, hipMemcpyDeviceToHost));
  CK(hipMemcpy(f, d_f, sizeof f, hipMemcpyDeviceToHost));
  printf("checked %llu floats [0, inf): aubio_log10_frexp != aubio_log10_fast on %llu\n", c[1], c[0]);
  for (unsigned long long i = 0; i < c[0] && i < 8; i++) printf("  x bits 0x%08x\n", f[i]);
  (void)hipFree(d_t);
  (void)hipFree(d_c);
  (void)hipFree(d_f);
  const bool ok = c[1] == kInf && c[0] == 0;
  printf("%s\n", ok ? "OK" : "FAIL");
  return ok ? 0 : 1;
}
