// Over the split's fast-path range x in [2^-98, 2^18] (|S|^2 of int16 PCM, fingerprint8k_kernel):
//  (a) which way raw v_sqrt_f32 misses the correctly rounded sqrtf (up / down counts),
//  (b) whether (float) v_sqrt_f64((double) x) equals the correctly rounded sqrtf.
// Reference: LLVM's IEEE sqrtf expansion (__builtin_sqrtf). Build:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off sqrt_range_check.hip -o sqrt_range_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void check(uint32_t lo, uint32_t hi, unsigned long long* cnt) {
  unsigned long long up = 0, down = 0, far = 0, f64bad = 0;
  for (uint64_t u = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= hi; u += (uint64_t)gridDim.x * blockDim.x) {
    const float x = __builtin_bit_cast(float, (uint32_t)u);
    const uint32_t ref = __builtin_bit_cast(uint32_t, __builtin_sqrtf(x));
    const uint32_t raw = __builtin_bit_cast(uint32_t, __builtin_amdgcn_sqrtf(x));
    const uint32_t d64 = __builtin_bit_cast(uint32_t, (float)__builtin_amdgcn_sqrt((double)x));
    if (raw + 1 == ref) up++;
    else if (raw == ref + 1) down++;
    else if (raw != ref) far++;
    if (d64 != ref) f64bad++;
  }
  atomicAdd(&cnt[0], up);
  atomicAdd(&cnt[1], down);
  atomicAdd(&cnt[2], far);
  atomicAdd(&cnt[3], f64bad);
}

int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 32);
  (void)hipMemset(d, 0, 32);
  const uint32_t lo = 0x0e800000u, hi = 0x48800000u;  // 2^-98 .. 2^18
  hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, lo, hi, d);
  unsigned long long h[4];
  (void)hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
  printf("x in [2^-98, 2^18]: %u floats\n", hi - lo + 1);
  printf("raw v_sqrt_f32 vs CR sqrtf: %llu one ulp low (needs +1), %llu one ulp high (needs -1), %llu further off\n", h[0], h[1], h[2]);
  printf("(float) v_sqrt_f64((double) x) vs CR sqrtf: %llu mismatches\n", h[3]);
  return 0;
}
