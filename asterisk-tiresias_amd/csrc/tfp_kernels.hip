// tfp_kernels.hip — gfx950 kernels of the tiresias hot path.
//
//  fingerprint_kernel  create_audio_fingerprints' per-hop loop (fp_handler.c:632-661) for a
//                      batch of clips: framing + hanningz window + 512-pt real FFT magnitude +
//                      40-band Slaney mel + log10 + DCT rows 0/1 + 10*log10|c| + "%f" rounding.
//  prep/scan/vote      fp_search_fingerprint_info's per-frame SQL and scoring
//                      (fp_handler.c:287-374) over the m1-sorted enrolled index.
//
// Numerics: built with -ffp-contract=off; every float/double operation below is the one the
// oracle (oracle/oracle.c) performs, in the same order, so results are bit-identical.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "tfp_kernels.hpp"
#include "tfp_math.hpp"
#include "tfp_synth.hpp"

namespace tfp {

// ------------------------------------------------------------------------------------
// Canonical FFT building blocks (spec: DESIGN.md §FFT; oracle: dft4/dft16/fft256).

__device__ __forceinline__ float2 cmul(float2 a, float wr, float wi) {
  float2 r;
  r.x = a.x * wr - a.y * wi;
  r.y = a.x * wi + a.y * wr;
  return r;
}

__device__ __forceinline__ void dft4(float2 a0, float2 a1, float2 a2, float2 a3, float2& X0, float2& X1,
                                     float2& X2, float2& X3) {
  const float t0r = a0.x + a2.x, t0i = a0.y + a2.y;
  const float t1r = a0.x - a2.x, t1i = a0.y - a2.y;
  const float t2r = a1.x + a3.x, t2i = a1.y + a3.y;
  const float t3r = a1.x - a3.x, t3i = a1.y - a3.y;
  X0.x = t0r + t2r; X0.y = t0i + t2i;
  X2.x = t0r - t2r; X2.y = t0i - t2i;
  X1.x = t1r + t3i; X1.y = t1i - t3r;
  X3.x = t1r - t3i; X3.y = t1i + t3r;
}

// 16-point DFT in registers: n = 4 n1 + n2, k = k1 + 4 k2, W16^e = tw256[16 e].
__device__ __forceinline__ void dft16(const DspTables* __restrict__ T, const float2 (&in)[16], float2 (&out)[16]) {
  float2 A[4][4];
#pragma unroll
  for (int n2 = 0; n2 < 4; n2++) dft4(in[n2], in[4 + n2], in[8 + n2], in[12 + n2], A[n2][0], A[n2][1], A[n2][2], A[n2][3]);
#pragma unroll
  for (int n2 = 1; n2 < 4; n2++)
#pragma unroll
    for (int k1 = 1; k1 < 4; k1++) {
      const int e = 16 * n2 * k1;
      A[n2][k1] = cmul(A[n2][k1], T->tw256_re[e], T->tw256_im[e]);
    }
#pragma unroll
  for (int k1 = 0; k1 < 4; k1++) dft4(A[0][k1], A[1][k1], A[2][k1], A[3][k1], out[k1], out[k1 + 4], out[k1 + 8], out[k1 + 12]);
}

// ------------------------------------------------------------------------------------
// Fingerprint kernel. Block = 16 frames of one clip; lane group (16 lanes) = one frame.
//   LDS: PCM tile of 17 hops (frame t's window = hops t, t+1) + one 16x17 complex scratch per frame.
constexpr int kTileSamples = (kFramesPerBlock + 1) * kHop;
constexpr int kScratch = 16 * 17;  // float2 per frame

__global__ __launch_bounds__(256) void fingerprint_kernel(const DspTables* __restrict__ T, const int16_t* __restrict__ pcm,
                                                          const int64_t* __restrict__ soff, const int64_t* __restrict__ foff,
                                                          const int32_t* __restrict__ toff, int32_t nclips,
                                                          int32_t* __restrict__ micro, double* __restrict__ db) {
  __shared__ int16_t tile[kTileSamples];
  __shared__ float2 work[kFramesPerBlock][kScratch];

  const int b = blockIdx.x;
  int lo = 0, hi = nclips;  // clip c with toff[c] <= b < toff[c+1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (toff[mid] <= b) lo = mid; else hi = mid;
  }
  const int c = lo;
  const int64_t s0 = soff[c], ns = soff[c + 1] - s0;
  const int64_t nf = (ns + kHop - 1) / kHop;
  const int64_t f0 = (int64_t)(b - toff[c]) * kFramesPerBlock;
  const int tid = threadIdx.x;

  // Stage hops f0-1 .. f0+15 (zeros before the clip and past its end: aubio_source_do pads).
  const int64_t base = (f0 - 1) * kHop;
  for (int i = tid; i < kTileSamples; i += 256) {
    const int64_t s = base + i;
    tile[i] = (s >= 0 && s < ns) ? pcm[s0 + s] : (int16_t)0;
  }
  __syncthreads();

  const int t = tid >> 4, L = tid & 15;
  const int16_t* win = tile + t * kHop;
  float2* W = work[t];

  // z[m] = x[2m] + i x[2m+1], x = fftshift(window * [old | new]); lane L holds m = 16 n1 + L.
  float2 z[16], Y[16];
#pragma unroll
  for (int n1 = 0; n1 < 16; n1++) {
    const int j = (32 * n1 + 2 * L + 256) & 511;
    const float a = (float)win[j] * (1.0f / 32768.0f);
    const float bb = (float)win[j + 1] * (1.0f / 32768.0f);
    z[n1].x = a * T->window[j];
    z[n1].y = bb * T->window[j + 1];
  }
  dft16(T, z, Y);
#pragma unroll
  for (int k1 = 1; k1 < 16; k1++) Y[k1] = cmul(Y[k1], T->tw256_re[L * k1], T->tw256_im[L * k1]);
#pragma unroll
  for (int k1 = 0; k1 < 16; k1++) W[L * 17 + k1] = Y[k1];
  __syncthreads();
#pragma unroll
  for (int n2 = 0; n2 < 16; n2++) z[n2] = W[n2 * 17 + L];
  dft16(T, z, Y);  // Y[k2] = Z[L + 16 k2]
  __syncthreads();
#pragma unroll
  for (int k2 = 0; k2 < 16; k2++) W[L + 16 * k2] = Y[k2];
  __syncthreads();
  float2 P[16];
#pragma unroll
  for (int k2 = 0; k2 < 16; k2++) P[k2] = W[(256 - (L + 16 * k2)) & 255];
  // |X[k]| of the 512-point real FFT, k = L + 16 k2 (k = 0 and 256 from Z[0]).
  float nrm[16];
  float nrm256 = 0.f;
#pragma unroll
  for (int k2 = 0; k2 < 16; k2++) {
    const int k = L + 16 * k2;
    const float a = Y[k2].x, bq = Y[k2].y, cc = P[k2].x, d = P[k2].y;
    if (k == 0) {
      nrm[k2] = fabsf(a + bq);
      nrm256 = fabsf(a - bq);
    } else {
      const float Er = a + cc, Ei = bq - d, Or = a - cc, Oi = bq + d;
      const float wr = T->tw512_re[k], wi = T->tw512_im[k];
      const float tr = wr * Oi + wi * Or;
      const float ti = wr * Or - wi * Oi;
      const float Xr = 0.5f * (Er + tr);
      const float Xi = 0.5f * (Ei - ti);
      // sqrtf, correctly rounded as SSE sqrtss is: v_sqrt_f32 is not, but the double root of
      // a float rounds to the correctly rounded float root (no float input has its root within
      // 2^-50 of a float midpoint, and the f64 sqrt sequence is accurate to < 1 ulp).
      const float s2 = Xr * Xr + Xi * Xi;
      nrm[k2] = (float)__builtin_sqrt((double)s2);
    }
  }
  __syncthreads();
  float* N = reinterpret_cast<float*>(W);  // norms at [0, 257), band logs at [260, 300)
#pragma unroll
  for (int k2 = 0; k2 < 16; k2++) N[L + 16 * k2] = nrm[k2];
  if (L == 0) N[256] = nrm256;
  __syncthreads();
  // Filterbank (sequential ascending-bin sums, as fmat_vecmul) + fvec_log10.
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int jf = L + 16 * r;
    if (jf < kFilters) {
      const int st = T->mel_start[jf], len = T->mel_len[jf], off = T->mel_off[jf];
      float acc = 0.f;
      for (int q = 0; q < len; q++) acc = acc + N[st + q] * T->mel_w[off + q];
      N[260 + jf] = aubio_log10_clamped(acc);
    }
  }
  __syncthreads();
  const int64_t f = f0 + t;
  if (L < kCoefs && f < nf) {
    float acc = 0.f;
    for (int i = 0; i < kFilters; i++) acc = acc + N[260 + i] * T->dct[L][i];
    const double q = db_of_coef(acc);
    const int64_t g = foff[c] + f;
    micro[2 * g + L] = micro_of_db(q);
    if (db) db[2 * g + L] = q;
  }
}

hipError_t launch_fingerprint(const DspTables* d_tables, const int16_t* d_pcm, const int64_t* d_soff,
                              const int64_t* d_foff, const int32_t* d_toff, int32_t nclips, int32_t ntiles,
                              int32_t* d_micro, double* d_db, hipStream_t s) {
  if (ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(fingerprint_kernel, dim3(ntiles), dim3(256), 0, s, d_tables, d_pcm, d_soff, d_foff, d_toff,
                     nclips, d_micro, d_db);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// Synthetic PCM.
__global__ void synth_kernel(const SynthSpecDev* __restrict__ specs, int64_t spc, int16_t* __restrict__ out) {
  const int c = blockIdx.y;
  const SynthSpecDev sp = specs[c];
  const SynthClip p = synth_clip(sp.seed, sp.clip);
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < spc; s += (int64_t)gridDim.x * blockDim.x)
    out[(int64_t)c * spc + s] = synth_sample(p, sp.offset + s);
}

hipError_t launch_synth(const SynthSpecDev* d_specs, int32_t nclips, int64_t spc, int16_t* d_out, hipStream_t s) {
  if (nclips <= 0 || spc <= 0) return hipSuccess;
  int64_t bx = (spc + 255) / 256;
  if (bx > 256) bx = 256;
  hipLaunchKernelGGL(synth_kernel, dim3((unsigned)bx, nclips), dim3(256), 0, s, d_specs, spc, d_out);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// Index build (sorted by max1, the B-tree idx_audio_fingerprint_max1 of fp_handler.c:745-753).
__global__ void index_keys_kernel(const int32_t* __restrict__ m1, const int32_t* __restrict__ clip,
                                  const int32_t* __restrict__ rank, int64_t n, int32_t* keys, int32_t* vals) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t v = m1[i];
    const bool live = rank[clip[i]] >= 0 && v != kNullMicro;  // NULL max1 never satisfies max1 >= ...
    keys[i] = live ? v : INT32_MAX;
    vals[i] = (int32_t)i;
  }
}

hipError_t launch_index_keys(const int32_t* st_m1, const int32_t* st_clip, const int32_t* rank_of_clip, int64_t n,
                             int32_t* keys, int32_t* vals, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(index_keys_kernel, dim3(2048), dim3(256), 0, s, st_m1, st_clip, rank_of_clip, n, keys, vals);
  return hipGetLastError();
}

__global__ void index_gather_kernel(const int32_t* __restrict__ sv, const int32_t* __restrict__ m2,
                                    const int32_t* __restrict__ clip, const int32_t* __restrict__ rank, int64_t n,
                                    int32_t* m2s, int32_t* cols) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t j = sv[i];
    m2s[i] = m2[j];
    cols[i] = rank[clip[j]];
  }
}

hipError_t launch_index_gather(const int32_t* sorted_vals, const int32_t* st_m2, const int32_t* st_clip,
                               const int32_t* rank_of_clip, int64_t n, int32_t* m2s, int32_t* cols, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(index_gather_kernel, dim3(2048), dim3(256), 0, s, sorted_vals, st_m2, st_clip, rank_of_clip, n,
                     m2s, cols);
  return hipGetLastError();
}

__device__ __forceinline__ int64_t lower_bound_i32(const int32_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int64_t upper_bound_i32(const int32_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)a[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ void count_below_kernel(const int32_t* keys, int64_t n, int32_t bound, int64_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *out = lower_bound_i32(keys, n, bound);
}

hipError_t launch_count_below(const int32_t* sorted_keys, int64_t n, int32_t bound, int64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(count_below_kernel, dim3(1), dim3(64), 0, s, sorted_keys, n, bound, out);
  return hipGetLastError();
}

hipError_t radix_sort_pairs(void* temp, size_t* temp_bytes, const int32_t* kin, int32_t* kout, const int32_t* vin,
                            int32_t* vout, int64_t n, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, kin, kout, vin, vout, (int)n, 0, 32, s);
}

// ------------------------------------------------------------------------------------
// Search: per query frame box (fp_handler.c:287-351).
__global__ void prep_boxes_kernel(const double* __restrict__ q, int64_t n, SearchConsts sc, FrameBox* __restrict__ boxes) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double q1 = q[2 * i], q2 = q[2 * i + 1];
    const double v1 = __builtin_isfinite(q1) ? q1 : 0.0;  // ast_json_real_get(NULL) = 0.0
    // (int) truncation, :290 — out of int range gives INT_MIN as x86 cvttsd2si does
    const int32_t ki = (v1 > -2147483649.0 && v1 < 2147483648.0) ? (int32_t)v1 : INT32_MIN;
    const double freq = (double)ki;
    FrameBox bx;
    bx.k = ki;
    bx.flags = 1;
    bx.L2 = bx.U2 = 0;
    if (sc.has_low && freq < sc.thr_low) bx.flags = 0;
    if (sc.has_high && freq > sc.thr_high) bx.flags = 0;
    const double lo = freq - sc.tole, hi = freq + sc.tole;
    if (!__builtin_isfinite(lo) || !__builtin_isfinite(hi)) bx.flags = 0;  // "%f" -> nan/inf: SQL error
    bx.L1 = fmt6_bound(lo);
    bx.U1 = fmt6_bound(hi);
    if (sc.coefs == 2 && bx.flags) {
      const double f2 = __builtin_isfinite(q2) ? q2 : 0.0;
      bool skip = false;
      if (sc.has_low && f2 < sc.thr_low) skip = true;
      else if (sc.has_high && f2 > sc.thr_high) skip = true;
      if (!skip) {
        const double lo2 = f2 - sc.tole, hi2 = f2 + sc.tole;
        if (!__builtin_isfinite(lo2) || !__builtin_isfinite(hi2)) bx.flags = 0;
        else {
          bx.L2 = fmt6_bound(lo2);
          bx.U2 = fmt6_bound(hi2);
          bx.flags |= 2;
        }
      }
    }
    boxes[i] = bx;
  }
}

hipError_t launch_prep_boxes(const double* d_q, int64_t nframes, SearchConsts sc, FrameBox* boxes, hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  int64_t g = (nframes + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(prep_boxes_kernel, dim3((unsigned)g), dim3(256), 0, s, d_q, nframes, sc, boxes);
  return hipGetLastError();
}

// ---- coefs = 1: vote matrix. score[q][clip] = sum_k N[q][k] * B[k][clip], where N counts the
// query's non-ignored frames with trunc key k and B[k][clip] = 1 iff the clip has a row in
// [fmt6(k - tol), fmt6(k + tol)] — exactly the per-frame "group by audio_uuid" hit count.
__global__ void key_hist_kernel(const FrameBox* __restrict__ boxes, const int64_t* __restrict__ qoff, int32_t nq,
                                int32_t* __restrict__ counts, uint32_t* __restrict__ mask, int32_t* __restrict__ maxc) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  int32_t local_max = 0;
  for (int64_t i = qoff[q]; i < qoff[q + 1]; i++) {
    const FrameBox bx = boxes[i];
    if (!(bx.flags & 1)) continue;
    const int64_t idx = (int64_t)bx.k + kKeyOffset;
    if (idx < 0 || idx >= kKeyRange) {  // not a fingerprint-range key: send the batch to the scan path
      local_max = INT32_MAX;
      continue;
    }
    const int32_t v = ++counts[(int64_t)q * kKeyRange + idx];
    local_max = v > local_max ? v : local_max;
    atomicOr(&mask[idx >> 5], 1u << (idx & 31));
  }
  if (local_max) atomicMax(maxc, local_max);
}

hipError_t launch_key_hist(const FrameBox* boxes, const int64_t* d_qoff, int32_t nq, int32_t* d_counts, uint32_t* d_mask,
                           int32_t* d_maxcount, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(key_hist_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, boxes, d_qoff, nq, d_counts, d_mask,
                     d_maxcount);
  return hipGetLastError();
}

__global__ void build_A_kernel(const int32_t* __restrict__ counts, int32_t nq, int32_t Qp, const int32_t* __restrict__ keycols,
                               int32_t Ku, int32_t Kp, _Float16* __restrict__ A) {
  const int64_t total = (int64_t)Qp * Kp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(i / Kp), col = (int)(i % Kp);
    int32_t v = 0;
    if (q < nq && col < Ku) v = counts[(int64_t)q * kKeyRange + keycols[col]];
    A[i] = (_Float16)(float)v;  // exact: v <= 2048 (checked by the host)
  }
}

hipError_t launch_build_A(const int32_t* d_counts, int32_t nq, int32_t Qp, const int32_t* d_keycols, int32_t Ku,
                          int32_t Kp, _Float16* d_A, hipStream_t s) {
  const int64_t total = (int64_t)Qp * Kp;
  int64_t g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(build_A_kernel, dim3((unsigned)g), dim3(256), 0, s, d_counts, nq, Qp, d_keycols, Ku, Kp, d_A);
  return hipGetLastError();
}

__global__ void build_B_kernel(const int32_t* __restrict__ m1s, int64_t R, const int32_t* __restrict__ cols,
                               const int64_t* __restrict__ kb, int32_t Kp, _Float16* __restrict__ Bt) {
  const int col = blockIdx.x;
  const int64_t lo = lower_bound_i32(m1s, R, kb[2 * col]);
  const int64_t hi = upper_bound_i32(m1s, R, kb[2 * col + 1]);
  for (int64_t r = lo + threadIdx.x; r < hi; r += blockDim.x) Bt[(int64_t)cols[r] * Kp + col] = (_Float16)1.0f;
}

hipError_t launch_build_B(const int32_t* m1s, int64_t R, const int32_t* cols, const int64_t* d_kbounds, int32_t Ku,
                          int32_t Kp, _Float16* d_Bt, hipStream_t s) {
  if (Ku <= 0) return hipSuccess;
  hipLaunchKernelGGL(build_B_kernel, dim3(Ku), dim3(256), 0, s, m1s, R, cols, d_kbounds, Kp, d_Bt);
  return hipGetLastError();
}

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int kVoteColsPerBlock = 1024;

// Wave = 32 queries x (32-clip sub-tiles of the block's 1024-clip chunk); 4 waves = 128 queries
// share each B fragment through L1. Fused argmax: per row the max (score, column); columns are
// the clips in ascending uuid order, so a later column wins a tie (SQLite returns the greatest
// audio_uuid). Result key = score << 32 | tiekey[column], merged with atomicMax.
__global__ __launch_bounds__(256) void vote_gemm_kernel(const _Float16* __restrict__ A, const _Float16* __restrict__ Bt,
                                                        int32_t Qp, int32_t Cp, int32_t Kp,
                                                        const int32_t* __restrict__ tiekey,
                                                        unsigned long long* __restrict__ best) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int q0 = (blockIdx.y * 4 + wave) * 32;
  if (q0 >= Qp) return;
  const int cbeg = blockIdx.x * kVoteColsPerBlock;
  const int cend = min(cbeg + kVoteColsPerBlock, Cp);
  int bs[16], bc[16];
#pragma unroll
  for (int i = 0; i < 16; i++) { bs[i] = 0; bc[i] = 0; }
  const _Float16* arow = A + (int64_t)(q0 + r) * Kp + 8 * h;
  for (int c0 = cbeg; c0 < cend; c0 += 32) {
    floatx16 acc;
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = 0.f;
    const _Float16* brow = Bt + (int64_t)(c0 + r) * Kp + 8 * h;
    for (int kb = 0; kb < Kp; kb += 16) {
      const half8 a = *reinterpret_cast<const half8*>(arow + kb);
      const half8 bv = *reinterpret_cast<const half8*>(brow + kb);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bv, acc, 0, 0, 0);
    }
    const int col = c0 + r;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int s = (int)acc[i];
      if (s > 0 && s >= bs[i]) { bs[i] = s; bc[i] = col; }
    }
  }
#pragma unroll
  for (int i = 0; i < 16; i++) {
    unsigned long long key = bs[i] > 0 ? (((unsigned long long)(unsigned)bs[i] << 32) | (unsigned)tiekey[bc[i]]) : 0ull;
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) {
      const unsigned long long o = __shfl_xor(key, off, 64);
      key = o > key ? o : key;
    }
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    if (r == 0 && key) atomicMax(&best[q0 + row], key);
  }
}

hipError_t launch_vote_gemm(const _Float16* d_A, const _Float16* d_Bt, int32_t Qp, int32_t Cp, int32_t Kp,
                            const int32_t* d_tiekey, unsigned long long* d_best, hipStream_t s) {
  if (Qp <= 0 || Cp <= 0) return hipSuccess;
  dim3 grid((Cp + kVoteColsPerBlock - 1) / kVoteColsPerBlock, (Qp / 32 + 3) / 4);
  hipLaunchKernelGGL(vote_gemm_kernel, grid, dim3(256), 0, s, d_A, d_Bt, Qp, Cp, Kp, d_tiekey, d_best);
  return hipGetLastError();
}

// ---- general path (any coefs / tolerance): one wave per query, frames in order; per frame the
// rows with max1 in [L1, U1] (binary search on the sorted index) filtered by the max2 box; each
// clip counts once per frame (stamp), i.e. the per-frame GROUP BY audio_uuid of :353.
__global__ __launch_bounds__(256) void scan_kernel(const FrameBox* __restrict__ boxes, const int64_t* __restrict__ qoff,
                                                   int32_t q_begin, int32_t nq, const int32_t* __restrict__ m1s,
                                                   const int32_t* __restrict__ m2s, const int32_t* __restrict__ cols,
                                                   int64_t R, const int32_t* __restrict__ tiekey, int32_t Cp,
                                                   int32_t* __restrict__ stamp, int32_t* __restrict__ score,
                                                   unsigned long long* __restrict__ best) {
  const int wq = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wq >= nq) return;
  const int q = q_begin + wq;
  int32_t* st = stamp + (int64_t)wq * Cp;
  int32_t* sc = score + (int64_t)wq * Cp;
  const int64_t fbeg = qoff[q], fend = qoff[q + 1];
  for (int64_t i = fbeg; i < fend; i++) {
    const FrameBox bx = boxes[i];
    if (!(bx.flags & 1)) continue;
    const int64_t lo = lower_bound_i32(m1s, R, bx.L1);
    const int64_t hi = upper_bound_i32(m1s, R, bx.U1);
    const int32_t tag = (int32_t)(i - fbeg) + 1;
    for (int64_t rr = lo + lane; rr < hi; rr += 64) {
      if (bx.flags & 2) {
        const int32_t v = m2s[rr];
        if (v == kNullMicro || (int64_t)v < bx.L2 || (int64_t)v > bx.U2) continue;
      }
      const int32_t col = cols[rr];
      const int32_t old = atomicMax(&st[col], tag);
      if (old < tag) {
        const int32_t s = atomicAdd(&sc[col], 1) + 1;
        atomicMax(&best[q], ((unsigned long long)(unsigned)s << 32) | (unsigned)tiekey[col]);
      }
    }
  }
}

hipError_t launch_scan(const FrameBox* boxes, const int64_t* d_qoff, int32_t q_begin, int32_t nq, const int32_t* m1s,
                       const int32_t* m2s, const int32_t* cols, int64_t R, const int32_t* d_tiekey, int32_t Cp,
                       int32_t* d_stamp, int32_t* d_score, unsigned long long* d_best, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(scan_kernel, dim3((nq + 3) / 4), dim3(256), 0, s, boxes, d_qoff, q_begin, nq, m1s, m2s, cols, R,
                     d_tiekey, Cp, d_stamp, d_score, d_best);
  return hipGetLastError();
}

}  // namespace tfp
