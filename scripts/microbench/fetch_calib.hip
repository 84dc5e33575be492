// FETCH_SIZE calibration for fingerprint8k_kernel's PCM reads (round 5): MI355X_MICROARCH.md's HBM
// section calibrates FETCH_SIZE for 16-B/lane streaming reads only ("other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern"). The kernel now reads
// PCM with 4-B buffer loads: a wave's pass reads 4 frames x 16 sample pairs per lane, lane (g, L)
// at byte 512 g + 4 L + {1024 + 128 n1 (n1 < 8), 128 (n1 - 8)} of the pass's 2,560-byte window
// (hops f - 1 .. f + 3; frames overlap by half). This kernel walks a buffer of known size with
// exactly that pattern (each wave over consecutive 2,048-byte hop steps: every byte read from
// memory once, twice through L2) and one 16-B/lane streaming pass over the same size for the known
// factor, so FETCH_SIZE(dword pattern) / FETCH_SIZE(16-B stream) x 2 is the correction.
// Build: hipcc --offload-arch=gfx950 -O3 fetch_calib.hip -o fetch_calib
// Run under: rocprofv3 --pmc FETCH_SIZE --kernel-include-regex calib -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int64_t kBytes = 512ll << 20;  // 512 MiB: past the 256 MiB Infinity Cache
constexpr int kPass = 2048;              // bytes a pass advances (4 hops of 256 int16 samples)

__global__ __launch_bounds__(256) void calib_dword_pattern(const int16_t* __restrict__ pcm, int64_t nbytes, uint32_t* sink) {
  const int lane = threadIdx.x & 63, grp = lane >> 4, L = lane & 15;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t npass = nbytes / kPass;
  const int64_t per = (npass + nw - 1) / nw;  // each wave a contiguous run of passes
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(pcm), (short)0, (int)nbytes, 0x00020000);
  uint32_t acc = 0;
  for (int64_t p = w * per; p < min(npass, (w + 1) * per); p++) {
    // frame grp of the pass starts at hop p*4 + grp - 1 (the first hop of the buffer before it reads 0)
    const int32_t fs = (int32_t)(p * kPass) + 512 * (grp - 1) + 4 * L;
#pragma unroll
    for (int n1 = 0; n1 < 16; n1++) {
      // bytes: 2 (256 + 32 n1) for n1 < 8 (hop f), 2 (32 (n1 - 8)) for n1 >= 8 (hop f - 1)
      acc ^= __builtin_amdgcn_raw_buffer_load_b32(rs, fs + (n1 < 8 ? 512 + 64 * n1 : 64 * (n1 - 8)), 0, 0);
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void calib_stream16(const int4* __restrict__ src, int64_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
    const int4 v = src[i];
    acc ^= (uint32_t)(v.x ^ v.y ^ v.z ^ v.w);
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  int16_t* buf = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&buf, kBytes) || hipMalloc(&sink, 4) || hipMemset(buf, 1, kBytes)) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  for (int r = 0; r < 3; r++) {
    hipLaunchKernelGGL(calib_dword_pattern, dim3(2048), dim3(256), 0, 0, buf, kBytes, sink);
    hipLaunchKernelGGL(calib_stream16, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const int4*>(buf), kBytes / 16, sink);
  }
  if (hipDeviceSynchronize()) {
    fprintf(stderr, "kernel failed\n");
    return 1;
  }
  printf("read %lld bytes per kernel, 3 launches each\n", (long long)kBytes);
  (void)hipFree(buf);
  (void)hipFree(sink);
  return 0;
}
