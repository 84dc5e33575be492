// Is (float) v_sqrt_f64((double) x) the correctly rounded sqrtf for every non-negative float?
// (A double sqrt within a few double ulps of the exact root rounds to the correctly rounded float,
// because no float's square root lies that close to a float rounding midpoint; this checks the
// hardware instruction's accuracy end to end.) Also times both forms per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off sqrt_f64_check.hip -o sqrt_f64_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float sqrtf_fast_cr(float x) {  // the kernel's current sequence
  float y = __builtin_amdgcn_sqrtf(x);
  const float ym = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) - 1u);
  const float yp = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) + 1u);
  const float rm = __builtin_fmaf(-ym, y, x);
  const float rp = __builtin_fmaf(-yp, y, x);
  y = rm <= 0.f ? ym : y;
  y = rp > 0.f ? yp : y;
  return y;
}
__device__ __forceinline__ float sqrt_via_f64(float x) { return (float)__builtin_amdgcn_sqrt((double)x); }

__global__ void check(unsigned long long* bad, unsigned int* first) {
  const uint64_t n = 0x7f800000ull;  // all non-negative finite floats (and +0)
  unsigned long long mine = 0;
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (uint64_t)gridDim.x * blockDim.x) {
    const float x = __builtin_bit_cast(float, (uint32_t)u);
    const float ref = __builtin_sqrtf(x);  // IEEE sqrt (LLVM's correctly rounded expansion)
    const float got = sqrt_via_f64(x);
    if (__builtin_bit_cast(uint32_t, ref) != __builtin_bit_cast(uint32_t, got)) {
      mine++;
      atomicMin(first, (unsigned int)u);
    }
  }
  if (mine) atomicAdd(bad, mine);
}

template <int V>
__global__ void timing(float* out, int iters, long long* cyc) {
  float x0 = 1.0f + threadIdx.x * 1e-3f, x1 = x0 + 0.5f, x2 = x0 + 0.25f, x3 = x0 + 0.125f;
  float a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    if (V == 0) { a0 += sqrtf_fast_cr(x0); a1 += sqrtf_fast_cr(x1); a2 += sqrtf_fast_cr(x2); a3 += sqrtf_fast_cr(x3); }
    else { a0 += sqrt_via_f64(x0); a1 += sqrt_via_f64(x1); a2 += sqrt_via_f64(x2); a3 += sqrt_via_f64(x3); }
    x0 += 1e-7f; x1 += 1e-7f; x2 += 1e-7f; x3 += 1e-7f;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3;
}

int main() {
  unsigned long long* d_bad;
  unsigned int* d_first;
  (void)hipMalloc(&d_bad, 8);
  (void)hipMalloc(&d_first, 4);
  (void)hipMemset(d_bad, 0, 8);
  const unsigned int big = 0xffffffffu;
  (void)hipMemcpy(d_first, &big, 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, d_bad, d_first);
  unsigned long long bad = 0;
  unsigned int first = 0;
  (void)hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&first, d_first, 4, hipMemcpyDeviceToHost);
  printf("(float)v_sqrt_f64 vs IEEE sqrtf over all 2139095040 non-negative finite floats: %llu mismatches", bad);
  if (bad) printf(" (first at bits 0x%08x)", first);
  printf("\n");

  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = cus * 2, iters = 4096;  // 2 waves / SIMD
  float* d_out;
  long long* d_cyc;
  (void)hipMalloc(&d_out, sizeof(float) * grid * 256);
  (void)hipMalloc(&d_cyc, sizeof(long long) * grid * 4);
  long long* h = new long long[grid * 4];
  const char* names[2] = {"v_sqrt_f32 + 2 fma residuals (current)", "cvt + v_sqrt_f64 + cvt"};
  for (int v = 0; v < 2; v++) {
    for (int rep = 0; rep < 2; rep++) {
      if (v == 0) hipLaunchKernelGGL(timing<0>, dim3(grid), dim3(256), 0, 0, d_out, iters, d_cyc);
      else hipLaunchKernelGGL(timing<1>, dim3(grid), dim3(256), 0, 0, d_out, iters, d_cyc);
    }
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d_cyc, sizeof(long long) * grid * 4, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < grid * 4; i++) s += h[i];
    const double per = s / (grid * 4) / (iters * 4.0);
    printf("%-40s %6.2f cycles per sqrt per wave, %5.2f per SIMD (2 waves)\n", names[v], per, per / 2);
  }
  return bad != 0;
}
