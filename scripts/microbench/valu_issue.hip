// VALU issue-cost microbenchmark (gfx950): cycles per instruction per wave for independent
// streams of one instruction type, at 1, 2 and 4 waves per SIMD (blocks of 256 threads, 1..4
// blocks per CU). Informs the fingerprint kernel's packing decisions (DESIGN.md perf log).
// Build: hipcc --offload-arch=gfx950 -O3 valu_issue.hip -o valu_issue
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define R8(x) x x x x x x x x
#define BODY(name, ins)                                                                            \
  __global__ void name(long long* out, int iters) {                                             \
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,       \
          a6 = a0 + 6, a7 = a0 + 7;                                                              \
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3;                                                   \
    long long t0 = __builtin_amdgcn_s_memtime();                                                 \
    for (int i = 0; i < iters; i++) { ins }                                                      \
    long long t1 = __builtin_amdgcn_s_memtime();                                                 \
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;   \
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)(d0 + d1 + d2 + d3) == 12345.f) out[0] = 0; \
  }

// 32 instructions per iteration, 8 independent destinations
#define ADD8 asm volatile("v_add_f32 %0, %0, %1\n v_add_f32 %1, %1, %2\n v_add_f32 %2, %2, %3\n v_add_f32 %3, %3, %4\n v_add_f32 %4, %4, %5\n v_add_f32 %5, %5, %6\n v_add_f32 %6, %6, %7\n v_add_f32 %7, %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
BODY(k_add, ADD8 ADD8 ADD8 ADD8)

#define ADDI8 asm volatile("v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(1.0f));
BODY(k_add_indep, ADDI8 ADDI8 ADDI8 ADDI8)

#define CHAIN8 asm volatile("v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1" : "+v"(a0) : "v"(a1));
BODY(k_chain, CHAIN8 CHAIN8 CHAIN8 CHAIN8)

#define PK8 asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pc));
#define PKBODY(name, ins)                                                                          \
  __global__ void name(long long* out, int iters) {                                             \
    typedef float f2 __attribute__((ext_vector_type(2)));                                         \
    f2 p0 = {(float)threadIdx.x, 1.f}, p1 = p0 + 1.f, p2 = p0 + 2.f, p3 = p0 + 3.f, pc = {1.f, 2.f}; \
    long long t0 = __builtin_amdgcn_s_memtime();                                                 \
    for (int i = 0; i < iters; i++) { ins }                                                      \
    long long t1 = __builtin_amdgcn_s_memtime();                                                 \
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;   \
    f2 s = p0 + p1 + p2 + p3;                                                                    \
    if (s.x + s.y == 12345.f) out[0] = 0;                                                        \
  }
PKBODY(k_pk_add, PK8 PK8 PK8 PK8)
#define PKM8 asm volatile("v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4\n v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pc));
PKBODY(k_pk_mul, PKM8 PKM8 PKM8 PKM8)

#define MOV8 asm volatile("v_mov_b32 %0, %1\n v_mov_b32 %1, %2\n v_mov_b32 %2, %3\n v_mov_b32 %3, %4\n v_mov_b32 %4, %5\n v_mov_b32 %5, %6\n v_mov_b32 %6, %7\n v_mov_b32 %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
BODY(k_mov, MOV8 MOV8 MOV8 MOV8)

#define D8 asm volatile("v_add_f64 %0, %0, %1\n v_add_f64 %1, %1, %2\n v_add_f64 %2, %2, %3\n v_add_f64 %3, %3, %0\n v_add_f64 %0, %0, %1\n v_add_f64 %1, %1, %2\n v_add_f64 %2, %2, %3\n v_add_f64 %3, %3, %0" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));
BODY(k_add_f64, D8 D8 D8 D8)
#define DF8 asm volatile("v_fma_f64 %0, %0, %1, %2\n v_fma_f64 %1, %1, %2, %3\n v_fma_f64 %2, %2, %3, %0\n v_fma_f64 %3, %3, %0, %1\n v_fma_f64 %0, %0, %1, %2\n v_fma_f64 %1, %1, %2, %3\n v_fma_f64 %2, %2, %3, %0\n v_fma_f64 %3, %3, %0, %1" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));
BODY(k_fma_f64, DF8 DF8 DF8 DF8)

#define SQ8 asm volatile("v_sqrt_f32 %0, %1\n v_sqrt_f32 %1, %2\n v_sqrt_f32 %2, %3\n v_sqrt_f32 %3, %4\n v_sqrt_f32 %4, %5\n v_sqrt_f32 %5, %6\n v_sqrt_f32 %6, %7\n v_sqrt_f32 %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
BODY(k_sqrt, SQ8 SQ8 SQ8 SQ8)

#define CV8 asm volatile("v_cvt_f64_f32 %0, %4\n v_cvt_f64_f32 %1, %5\n v_cvt_f64_f32 %2, %6\n v_cvt_f64_f32 %3, %7\n v_cvt_f32_f64 %4, %0\n v_cvt_f32_f64 %5, %1\n v_cvt_f32_f64 %6, %2\n v_cvt_f32_f64 %7, %3" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
BODY(k_cvt, CV8 CV8 CV8 CV8)

typedef void (*K)(long long*, int);
int main(int argc, char** argv) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  struct { const char* n; K k; } ks[] = {{"v_add_f32 (8 chains)", k_add},     {"v_add_f32 independent", k_add_indep},
                                         {"v_add_f32 1 chain", k_chain},       {"v_pk_add_f32", k_pk_add},
                                         {"v_pk_mul_f32", k_pk_mul},           {"v_mov_b32", k_mov},
                                         {"v_add_f64", k_add_f64},             {"v_fma_f64", k_fma_f64},
                                         {"v_sqrt_f32", k_sqrt},               {"v_cvt_f64_f32/f32_f64", k_cvt}};
  const int iters = 2000;
  long long* d;
  hipMalloc(&d, sizeof(long long) * cus * 4 * 4);
  long long* h = (long long*)malloc(sizeof(long long) * cus * 4 * 4);
  printf("cycles per instruction per wave (s_memtime), waves/SIMD = 1, 2, 4; SIMD issue interval = cyc / waves\n");
  for (auto& k : ks) {
    printf("%-26s", k.n);
    for (int w : {1, 2, 4}) {
      const int grid = cus * w;
      hipLaunchKernelGGL(k.k, dim3(grid), dim3(256), 0, 0, d, iters);  // warm
      hipLaunchKernelGGL(k.k, dim3(grid), dim3(256), 0, 0, d, iters);
      hipDeviceSynchronize();
      hipMemcpy(h, d, sizeof(long long) * grid * 4, hipMemcpyDeviceToHost);
      double s = 0;
      for (int i = 0; i < grid * 4; i++) s += h[i];
      const double cpi = s / (grid * 4) / (iters * 32.0);
      printf("  %d: %6.2f cyc (SIMD %5.2f)", w, cpi, cpi / w);
    }
    printf("\n");
  }
  return 0;
}
