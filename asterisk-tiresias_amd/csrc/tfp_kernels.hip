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
#include <type_traits>

#include "tfp_kernels.hpp"
#include "tfp_log.hpp"
#include "tfp_math.hpp"
#include "tfp_split.hpp"
#include "tfp_synth.hpp"

namespace tfp {

// ------------------------------------------------------------------------------------
// Canonical FFT building blocks (spec: DESIGN.md §FFT; oracle: dft4/dft16/fft256).

// Complex values as (re, im) register pairs: every operation below is a v_pk_*_f32 whose lanes
// perform exactly the scalar IEEE operations of the canonical spec (x + (-y) == x - y, products
// and sums commute). Per-lane signs ride on an exact fma: fma(p, (1, -1), c) rounds c + p.x and
// c - p.y once each — the plain add and subtract — so (re, im) sign patterns cost no moves.
typedef float cf __attribute__((ext_vector_type(2)));

__device__ __forceinline__ cf swap(cf a) { return __builtin_shufflevector(a, a, 1, 0); }
__device__ __forceinline__ cf addsub(cf c, cf p) { return __builtin_elementwise_fma(p, cf{1.f, -1.f}, c); }  // (c.x + p.x, c.y - p.y)
__device__ __forceinline__ cf subadd(cf c, cf p) { return __builtin_elementwise_fma(p, cf{-1.f, 1.f}, c); }  // (c.x - p.x, c.y + p.y)

// a * w: (a.x wr - a.y wi, a.x wi + a.y wr)
__device__ __forceinline__ cf cmul(cf a, cf w) {
  const cf p = a * cf{w.x, w.x};        // (a.x wr, a.y wr)
  const cf q = swap(a) * cf{w.y, w.y};  // (a.y wi, a.x wi)
  return subadd(p, q);
}

__device__ __forceinline__ void dft4(cf a0, cf a1, cf a2, cf a3, cf& X0, cf& X1, cf& X2, cf& X3) {
  const cf t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, t3 = a1 - a3;
  X0 = t0 + t2;
  X2 = t0 - t2;
  X1 = addsub(t1, swap(t3));  // (t1r + t3i, t1i - t3r)
  X3 = subadd(t1, swap(t3));  // (t1r - t3i, t1i + t3r)
}

// 16-point DFT in registers: n = 4 n1 + n2, k = k1 + 4 k2, W16^e = tw256[16 e].
__device__ __forceinline__ void dft16(const cf (&w16)[10], const cf (&in)[16], cf (&out)[16]) {
  cf A[4][4];
#pragma unroll
  for (int n2 = 0; n2 < 4; n2++) dft4(in[n2], in[4 + n2], in[8 + n2], in[12 + n2], A[n2][0], A[n2][1], A[n2][2], A[n2][3]);
#pragma unroll
  for (int n2 = 1; n2 < 4; n2++)
#pragma unroll
    for (int k1 = 1; k1 < 4; k1++) A[n2][k1] = cmul(A[n2][k1], w16[n2 * k1]);
#pragma unroll
  for (int k1 = 0; k1 < 4; k1++) dft4(A[0][k1], A[1][k1], A[2][k1], A[3][k1], out[k1], out[k1 + 4], out[k1 + 8], out[k1 + 12]);
}

// ------------------------------------------------------------------------------------
// Fingerprint kernel (persistent, wave-independent).
//   * A workgroup stages the DSP tables in LDS once; afterwards its 4 waves never wait on each
//     other: each wave walks 16-frame tiles on its own (tile = 16 consecutive frames of a clip).
//   * FFT stage: 16 lanes per frame, 4 frames per pass, 4 passes per tile. The 256-point complex
//     FFT is 16x16 Cooley-Tukey with the transpose through a padded (16x17) LDS square; the real
//     split, |X|, the filterbank and the log10 stay on the frame's 16 lanes. Each frame leaves its
//     40 band logs in the wave's log buffer.
//   * Tail: once per tile, 32 lanes (frame, coef) run the DCT row, 10*log10|c| and "%f" rounding.
//   * PCM: each pass's 5 hops are fetched with coalesced 16-byte loads one pass ahead (registers),
//     then staged in the wave's LDS scratch.
//   * Filterbank: a lane's 3 filters (slot schedule, see DspTables) are summed interleaved.
#ifndef TFP_FP_WAVES
#define TFP_FP_WAVES 2  // waves per SIMD the register budget is cut for (A/B: scripts/ab_waves.sh)
#endif
#ifndef TFP_FP_BLOCK_WAVES
#define TFP_FP_BLOCK_WAVES 4  // waves per workgroup (LDS: tables once per block + per-wave scratch)
#endif
constexpr int kBlockWaves = TFP_FP_BLOCK_WAVES;
constexpr int kBlockThreads = 64 * kBlockWaves;
constexpr int kWaveFrames = 16;     // frames per wave tile (== kFramesPerBlock: tile offsets)
constexpr int kFrameStride = 272;   // complex per frame scratch: 16x17 padded square (2 x 272 floats
                                    // = 32 mod 64 banks: frames g, g+1 of a b64 read take opposite halves)
constexpr int kSq = 17;             // padded row of the transpose square (affine addresses, no conflicts)
constexpr int kLogStride = 41;      // floats per frame row in the log buffer (bank-conflict free)
constexpr int kMsLds = 960;         // filterbank slot-schedule weights kept in LDS (8 kHz: 16 x 60)

struct LdsTables {
  float window[kWin];              // hanningz * 2^-15 (window_s)
  cf lane_tw[15][16];              // lane_tw[k1-1][L] = w256^(L*k1), k1 = 1..15
  cf w16[10];                      // W16^e = tw256[16 e] (dft16's internal twiddles)
  cf tw512[kBins];                 // w512^k for the real split
  float dct[kCoefs][kFilters];
  int32_t ms_len[3], ms_woff[3];
  int32_t ms_filter[3][16], ms_start[3][16];
  LogfEntry logf[16];
  LogfEntry logf2[kLogf2Entries];  // (invc, y0) for aubio_log10_frexp (tfp_log.hpp)
  int32_t c_defer, c_real[2];  // slot-2 log deferral (DspTables::ms_c_defer)
  union {
    alignas(16) float ms_w[kMsLds];                  // slot schedule (fingerprint_kernel, fingerprint8k_kernel<1>)
    alignas(16) float fbw[kFbSteps * kFbPatterns];  // frame-pair schedule (fingerprint8k_kernel<4>): [step / 4][pattern][step % 4]
  };
};

constexpr int kPassSamples = 5 * kHop;           // one pass = 4 frames = hops f-1 .. f+3
constexpr int kPassChunks = kPassSamples / 8;     // 16-byte chunks per pass (160)
constexpr int kChunkRounds = (kPassChunks + 63) / 64;
constexpr int kHopStride = kHop + 32;  // staged hop stride in samples: frames 0/1 (and 2/3) of a
                                       // 32-lane half read disjoint LDS bank halves

// The pass's staged PCM aliases the FFT scratch: it is read into registers (z) before the first
// write of the transpose square, and restaged only after the filterbank has read |X|.
struct WaveLds {
  union {
    cf scratch[4][kFrameStride];
    alignas(16) int16_t pcm[5 * kHopStride];
    alignas(16) float pcmf[5 * kHopStride];  // fp32-sample launches of the generic kernel
  };
  float logs[kWaveFrames * kLogStride];
};
static_assert(sizeof(float) * 5 * kHopStride <= sizeof(cf) * 4 * kFrameStride, "pcm alias fits");
static_assert(16 * kSq <= kFrameStride && 16 + 500 <= 2 * kFrameStride, "square and |X| rows (ms_maxbin <= 500) fit");

// The 8 kHz kernel's per-wave scratch: the transpose square stored column-major with a row pitch
// of 18 complex (lane L writes Y[k1] to [k1][L]; reads its column as 8 contiguous ds_read_b128,
// conflict-free: lane L's 16-B pieces start at dword 36 L + 4 j, 16 distinct bank quads per lane
// group), frames 288 complex apart; the odd frames' |X| rows 48 floats in, which gives the
// filterbank reads the banks of the 272-complex layout (frames 0, 48, 0, 48 mod 64).
//
// The throughput kernel's filterbank runs once per two passes over frame pairs: a pass writes
// each pair's |X| rows interleaved ([bin][2 frames], kFbRow floats per pair, the two pairs' rows
// 32 banks apart), the even pass into xeven and the odd pass into the scratch (free after its
// transpose), and 64 lanes = 4 pairs x 16 patterns (DspTables::fb_*) then sum all 8 frames.
// Its raw sums land in logs as [2 (t % 8) + t / 8][kFbNf] for tile frame t (a pair's frames of
// both double passes a few rows apart: immediate offsets), logged once per tile.
typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int kSq8 = 18;
constexpr int kFrameStride8 = 16 * kSq8;
constexpr int kFbRow = 544;  // 258 bins x 2 frames, padded to 32 mod 64 banks
constexpr int kFbNf = 34;    // non-empty filters at 8 kHz (DspTables::fb_nfilters), all below the empty ones
struct WaveLds8 {
  union {
    cf scratch[4][kFrameStride8];
    alignas(16) int16_t pcm[5 * kHopStride];
  };
  alignas(16) float xeven[2 * kFbRow];
  float logs[kWaveFrames * kLogStride];
};
static_assert(2 * 5 * kHopStride <= sizeof(cf) * 4 * kFrameStride8 && 48 + 260 <= 2 * kFrameStride8, "8 kHz scratch");
static_assert(2 * kFbRow <= 2 * 4 * kFrameStride8 && 2 * kFbRowBins <= kFbRow && kWaveFrames * kFbNf <= kWaveFrames * kLogStride,
              "frame-pair rows");
static_assert(kFbSegs == 4, "fb_seg");
// The throughput kernel's workgroup: 4 waves (two workgroups per CU, two waves per SIMD). A
// bit-exact 12-wave form (three waves per SIMD, transposes through half squares to fit the LDS)
// measured 0.469 vs 0.442 ms per C2 launch in round 4 and was removed in round 5.
constexpr int kBW8 = 4;
template <int kPasses>
constexpr int fp8_block_waves() { return kPasses >= 2 ? kBW8 : kBlockWaves; }
static_assert(kBW8 == kBlockWaves, "one workgroup shape");
constexpr int fb_seg(int s) { return s < kFbSegStart[1] ? 0 : s < kFbSegStart[2] ? 1 : s < kFbSegStart[3] ? 2 : 3; }

// Where a pass of 4 frames reads: the clip's samples [(f_first - 1) * 256, (f_first + 4) * 256).
template <typename Smp>
struct PassSrc {
  const Smp* clip;
  int64_t ns;
  int64_t sbase;
  bool aligned;  // clip + sbase is 16-byte aligned
};
// Sample types of the generic kernel: int16 PCM (x / 32768 folded into window_s) or the fp32
// values aubio_source produced (multichannel mean, 24/32-bit, float WAV; tfp_wav_decode_f32).
template <typename Smp>
struct SmpLayout {
  static constexpr int kPer = 16 / (int)sizeof(Smp);          // samples per 16-byte chunk
  static constexpr int kChunks = kPassSamples / kPer;         // chunks per pass
  static constexpr int kRounds = (kChunks + 63) / 64;         // wave-wide chunk rounds
  static constexpr int kHopChunks = kHop / kPer;              // chunks per staged hop
};

// Slow path of one 16-byte chunk: clip edges (zeros outside [0, ns): aubio_source pads the last
// hop, the phase vocoder's first history hop is zeros) and unaligned clips.
__device__ __noinline__ int4 fetch_chunk_checked(const float* clip, int64_t ns, int64_t s) {
  float v[4];
  for (int e = 0; e < 4; e++) v[e] = (s + e >= 0 && s + e < ns) ? clip[s + e] : 0.f;
  return make_int4(__builtin_bit_cast(int, v[0]), __builtin_bit_cast(int, v[1]), __builtin_bit_cast(int, v[2]),
                   __builtin_bit_cast(int, v[3]));
}
__device__ __noinline__ int4 fetch_chunk_checked(const int16_t* clip, int64_t ns, int64_t s) {
  // an aligned chunk wholly inside the clip (most of an edge pass's): one 16-byte load
  if (s >= 0 && s + 8 <= ns && (reinterpret_cast<uintptr_t>(clip + s) & 15) == 0)
    return *reinterpret_cast<const int4*>(clip + s);
  uint32_t w[4];
  for (int e = 0; e < 4; e++) {
    const int64_t a = s + 2 * e;
    const uint32_t lo = (a >= 0 && a < ns) ? (uint16_t)clip[a] : 0u;
    const uint32_t hi = (a + 1 >= 0 && a + 1 < ns) ? (uint16_t)clip[a + 1] : 0u;
    w[e] = lo | (hi << 16);
  }
  return make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]);
}

// The same, inline (the 8 kHz kernel's edge passes): a call makes the caller wait for every
// outstanding load first, and a batch-1 query's PCM is read across PCIe from mapped host memory.
__device__ __forceinline__ int4 fetch_chunk_inline(const int16_t* clip, int64_t ns, int64_t s) {
  uint32_t w[4];
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int64_t a = s + 2 * e;
    const uint32_t lo = (a >= 0 && a < ns) ? (uint16_t)clip[a] : 0u;
    const uint32_t hi = (a + 1 >= 0 && a + 1 < ns) ? (uint16_t)clip[a + 1] : 0u;
    w[e] = lo | (hi << 16);
  }
  return make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]);
}

// 16-byte chunks of a pass into registers, issued one pass ahead of use.
template <typename Smp>
__device__ __forceinline__ void fetch_pass(const PassSrc<Smp>& p, bool valid, int lane,
                                           int4 (&pf)[SmpLayout<Smp>::kRounds]) {
  using Ly = SmpLayout<Smp>;
#pragma unroll
  for (int r = 0; r < Ly::kRounds; r++) {
    const int chunk = lane + 64 * r;
    int4 v = make_int4(0, 0, 0, 0);
    if (valid && chunk < Ly::kChunks) {
      const int64_t s = p.sbase + Ly::kPer * chunk;
      if (p.aligned && s >= 0 && s + Ly::kPer <= p.ns) v = *reinterpret_cast<const int4*>(p.clip + s);
      else v = fetch_chunk_checked(p.clip, p.ns, s);
    }
    pf[r] = v;
  }
}

// All LDS exchanges below stay inside one wave: a wave-level fence + barrier orders them.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float pcm_f(int16_t v) { return (float)v * (1.0f / 32768.0f); }

// Correctly rounded sqrtf (= SSE sqrtss, what glibc's sqrtf is). For inputs in [2^-100, 2^100)
// the raw v_sqrt_f32 (<= 1 ulp) is corrected with two exact fma residuals — the sequence LLVM
// emits for IEEE sqrt minus its denormal scaling and special-value handling, which are only
// needed outside that range; there the full builtin runs.
__device__ __forceinline__ float cr_sqrtf(float x) {
  if (x >= 0x1p-100f && x < 0x1p100f) {
    float y = __builtin_amdgcn_sqrtf(x);
    const float ym = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) - 1u);
    const float yp = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) + 1u);
    const float rm = __builtin_fmaf(-ym, y, x);
    const float rp = __builtin_fmaf(-yp, y, x);
    y = rm <= 0.f ? ym : y;
    y = rp > 0.f ? yp : y;
    return y;
  }
  return __builtin_sqrtf(x);
}

// One lane's 3 filterbank sums (slots A/B/C, lenA >= lenB >= lenC), interleaved in three
// branch-free phases. Each sum runs over its bins in ascending order from 0 (fmat_vecmul); the
// zero-padded tail of a short filter adds exact +0 (N beyond bin 256 is zero-filled).
// W is instantiated per address space (LDS or global) so every load is a ds_read/global_load.
template <class WPtr>
__device__ __forceinline__ void mel3(const float* __restrict__ N, WPtr wA, WPtr wB, WPtr wC, int stA, int stB,
                                     int stC, int lenA, int lenB, int lenC, float& aA, float& aB, float& aC) {
  // lengths and starts are multiples of 4; per 4 bins one 16-byte weight read (the lane's
  // 16-B slot of the 64-float row of bins q..q+3: w + 16 q) and one aligned 16-byte |X| read per slot
#define TFP_MAC4(ACC, NV, WV) \
  ACC = ACC + NV.x * WV.x; ACC = ACC + NV.y * WV.y; ACC = ACC + NV.z * WV.z; ACC = ACC + NV.w * WV.w
  int q = 0;
  for (; q < lenC; q += 4) {
    const float4 a = *reinterpret_cast<const float4*>(wA + 16 * q);
    const float4 b = *reinterpret_cast<const float4*>(wB + 16 * q);
    const float4 c = *reinterpret_cast<const float4*>(wC + 16 * q);
    const float4 na = *reinterpret_cast<const float4*>(N + stA + q);
    const float4 nb = *reinterpret_cast<const float4*>(N + stB + q);
    const float4 nc = *reinterpret_cast<const float4*>(N + stC + q);
    aA = aA + na.x * a.x; aB = aB + nb.x * b.x; aC = aC + nc.x * c.x;
    aA = aA + na.y * a.y; aB = aB + nb.y * b.y; aC = aC + nc.y * c.y;
    aA = aA + na.z * a.z; aB = aB + nb.z * b.z; aC = aC + nc.z * c.z;
    aA = aA + na.w * a.w; aB = aB + nb.w * b.w; aC = aC + nc.w * c.w;
  }
  for (; q < lenB; q += 4) {
    const float4 a = *reinterpret_cast<const float4*>(wA + 16 * q);
    const float4 b = *reinterpret_cast<const float4*>(wB + 16 * q);
    const float4 na = *reinterpret_cast<const float4*>(N + stA + q);
    const float4 nb = *reinterpret_cast<const float4*>(N + stB + q);
    aA = aA + na.x * a.x; aB = aB + nb.x * b.x;
    aA = aA + na.y * a.y; aB = aB + nb.y * b.y;
    aA = aA + na.z * a.z; aB = aB + nb.z * b.z;
    aA = aA + na.w * a.w; aB = aB + nb.w * b.w;
  }
  for (; q < lenA; q += 4) {
    const float4 a = *reinterpret_cast<const float4*>(wA + 16 * q);
    const float4 na = *reinterpret_cast<const float4*>(N + stA + q);
    TFP_MAC4(aA, na, a);
  }
#undef TFP_MAC4
}

// mel3 for a compile-time slot schedule (8 kHz: 36/16/8): fully unrolled, so every weight and
// |X| read of the three slots is issued before the first sum needs it (the runtime-length loop
// waits out one LDS round trip per 4 bins). One dependent chain per slot, each in ascending bin
// order; the products of 4 bins pair into v_pk_mul_f32 without register moves.
template <int LA, int LB, int LC, class WPtr>
__device__ __forceinline__ void mel3_fixed(const float* __restrict__ N, WPtr wA, WPtr wB, WPtr wC, int stA, int stB,
                                           int stC, float& aA, float& aB, float& aC) {
  float4 wa[LA / 4], na[LA / 4], wb[LB / 4], nb[LB / 4], wc[LC / 4], nc[LC / 4];
#pragma unroll
  for (int i = 0; i < LC / 4; i++) {
    wc[i] = *reinterpret_cast<const float4*>(wC + 64 * i);
    nc[i] = *reinterpret_cast<const float4*>(N + stC + 4 * i);
  }
#pragma unroll
  for (int i = 0; i < LB / 4; i++) {
    wb[i] = *reinterpret_cast<const float4*>(wB + 64 * i);
    nb[i] = *reinterpret_cast<const float4*>(N + stB + 4 * i);
  }
#pragma unroll
  for (int i = 0; i < LA / 4; i++) {
    wa[i] = *reinterpret_cast<const float4*>(wA + 64 * i);
    na[i] = *reinterpret_cast<const float4*>(N + stA + 4 * i);
  }
#pragma unroll
  for (int i = 0; i < LC / 4; i++) {
    aC = aC + nc[i].x * wc[i].x; aC = aC + nc[i].y * wc[i].y; aC = aC + nc[i].z * wc[i].z; aC = aC + nc[i].w * wc[i].w;
  }
#pragma unroll
  for (int i = 0; i < LB / 4; i++) {
    aB = aB + nb[i].x * wb[i].x; aB = aB + nb[i].y * wb[i].y; aB = aB + nb[i].z * wb[i].z; aB = aB + nb[i].w * wb[i].w;
  }
#pragma unroll
  for (int i = 0; i < LA / 4; i++) {
    aA = aA + na[i].x * wa[i].x; aA = aA + na[i].y * wa[i].y; aA = aA + na[i].z * wa[i].z; aA = aA + na[i].w * wa[i].w;
  }
}

// |X[k]|^2 of the 512-point real FFT from Z[k] = y and Z[256 - k] = P with w = w512^k:
// E = (a + Px, b - Py), O = (a - Px, b + Py), tr = wx Oi + wy Or, ti = wx Or - wy Oi,
// X = (0.5 (Er + tr), 0.5 (Ei - ti)), |X|^2 = Xr Xr + Xi Xi — each lane of each packed op is
// that scalar operation (-(a - b) and (-a) + b round alike; only a zero's sign may differ in
// Xi, which Xi * Xi erases).
__device__ __forceinline__ float split_power(cf y, cf P, cf w) {
  const cf E = addsub(y, P);                           // (a + Px, b - Py)
  const cf O = subadd(y, P);                           // (a - Px, b + Py)
  const cf T = addsub(O * cf{w.y, w.y}, swap(O) * cf{w.x, w.x});  // (wy Or + wx Oi, wy Oi - wx Or) = (tr, -ti)
  const cf X = cf{0.5f, 0.5f} * (E + T);
  const cf X2 = X * X;
  return X2.x + X2.y;
}

// v_sqrt_f32 (<= 1 ulp) + exact fma-residual correction: the correctly rounded sqrtf for
// x in [2^-100, 2^100) (cr_sqrtf without the range test).
__device__ __forceinline__ float sqrtf_fast_cr(float x) {
  float y = __builtin_amdgcn_sqrtf(x);
  const float ym = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) - 1u);
  const float yp = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) + 1u);
  const float rm = __builtin_fmaf(-ym, y, x);
  const float rp = __builtin_fmaf(-yp, y, x);
  y = rm <= 0.f ? ym : y;
  y = rp > 0.f ? yp : y;
  return y;
}

// Value of lane (16 - L) & 15 of this lane's 16-lane row (L = lane & 15). ds_bpermute: measured
// faster than the two-DPP-mov form (row_mirror + row_ror:1, 0.937 vs 0.911 ms per C2 launch),
// whose chained DPP reads cost wait states, and no slower than one row_mirror with renumbered
// second-stage columns plus selects for the two self-paired columns (round 2: 0.486 vs 0.484 ms).
__device__ __forceinline__ float partner16(float v) { return __shfl(v, (16 - (int)(threadIdx.x & 15)) & 15, 16); }

template <typename Smp>
__global__ __launch_bounds__(kBlockThreads, TFP_FP_WAVES) void fingerprint_kernel(
    const DspTables* __restrict__ T, const Smp* __restrict__ pcm, const int64_t* __restrict__ sbeg,
    const int64_t* __restrict__ send, const int64_t* __restrict__ foff, const int32_t* __restrict__ toff,
    const int32_t* __restrict__ tclip,
    int32_t ntiles, int32_t* __restrict__ micro, double* __restrict__ db, LogFix fx) {
  __shared__ __attribute__((aligned(16))) LdsTables S;
  __shared__ __attribute__((aligned(16))) WaveLds WL[kBlockWaves];
  const int tid = threadIdx.x;
  using Ly = SmpLayout<Smp>;
  constexpr bool kF32 = sizeof(Smp) == 4;
  // int16: hanningz * 2^-15 (aubio's x / 32768 folded in, exact); fp32 samples: hanningz
  for (int i = tid; i < kWin; i += kBlockThreads) S.window[i] = kF32 ? T->window[i] : T->window_s[i];
  for (int i = tid; i < 15 * 16; i += kBlockThreads) {
    const int k1 = 1 + i / 16, L = i % 16;
    S.lane_tw[k1 - 1][L] = cf{T->lane_tw_re[k1][L], T->lane_tw_im[k1][L]};
  }
  for (int i = tid; i < 10; i += kBlockThreads) S.w16[i] = cf{T->tw256_re[16 * i], T->tw256_im[16 * i]};
  for (int i = tid; i < kBins; i += kBlockThreads) S.tw512[i] = cf{T->tw512_re[i], T->tw512_im[i]};
  for (int i = tid; i < kCoefs * kFilters; i += kBlockThreads) (&S.dct[0][0])[i] = (&T->dct[0][0])[i];
  for (int i = tid; i < 48; i += kBlockThreads) {
    (&S.ms_filter[0][0])[i] = (&T->ms_filter[0][0])[i];
    (&S.ms_start[0][0])[i] = (&T->ms_start[0][0])[i];
  }
  if (tid < 3) { S.ms_len[tid] = T->ms_len[tid]; S.ms_woff[tid] = T->ms_woff[tid]; }
  if (tid < 16) S.logf[tid] = logf_table()[tid];
  if (tid == 0) { S.c_defer = T->ms_c_defer; S.c_real[0] = T->ms_c_real[0]; S.c_real[1] = T->ms_c_real[1]; }
  const bool ms_in_lds = T->ms_total <= kMsLds;
  for (int i = tid; i < (ms_in_lds ? T->ms_total : 0); i += kBlockThreads) S.ms_w[i] = T->ms_w[i];
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63, grp = lane >> 4, L = lane & 15;
  WaveLds& M = WL[wave];
  cf* W = M.scratch[grp];
  // |X| at [0, 257) after the FFT; odd frames' rows are shifted by 16 floats so that the |X|
  // stores of frames g and g+1 (one ds_write_b32 lane half) take opposite bank halves
  float* N = reinterpret_cast<float*>(W) + 16 * (grp & 1);
  const int nwaves = gridDim.x * kBlockWaves;
  const int lenA = S.ms_len[0], lenB = S.ms_len[1], lenC = S.ms_len[2];
  const int maxbin = T->ms_maxbin;
  const int fA = S.ms_filter[0][L], fB = S.ms_filter[1][L], fC = S.ms_filter[2][L];
  // Loop-invariant twiddles in registers (2 waves/SIMD leave VGPR room): dft16's W16^e and this
  // lane's inter-stage w256^(L k1), read from LDS once instead of every pass.
  cf w16r[10];
#pragma unroll
  for (int e = 0; e < 10; e++) w16r[e] = S.w16[e];
  cf ltw[15];
#pragma unroll
  for (int k1 = 1; k1 < 16; k1++) ltw[k1 - 1] = S.lane_tw[k1 - 1][L];
  const bool c_defer = S.c_defer != 0;
  const bool c_real = fC >= 0 && (fC == S.c_real[0] || fC == S.c_real[1]);
  {
    // log rows of empty filters (zero sum) never change: the constant log of the clamped 0
    const float lempty = aubio_log10_fast(0.f, S.logf);
    for (int i = lane; i < kWaveFrames * kFilters; i += 64) {
      const int j = i % kFilters;
      if (T->mel_len[j] == 0) M.logs[(i / kFilters) * kLogStride + j] = lempty;
    }
  }

  auto pass_src = [&](int c, int64_t f0, int sub) {
    PassSrc<Smp> p;
    const int64_t s0 = sbeg[c];
    p.clip = pcm + s0;
    p.ns = send[c] - s0;
    p.sbase = (f0 + 4 * sub - 1) * kHop;
    p.aligned = ((reinterpret_cast<uintptr_t>(p.clip) & 15) == 0);
    return p;
  };

  int4 pf[Ly::kRounds];
  int b = blockIdx.x * kBlockWaves + wave;
  int c = b < ntiles ? tclip[b] : 0;
  int64_t f0 = b < ntiles ? (int64_t)(b - toff[c]) * kWaveFrames : 0;
  fetch_pass(pass_src(c, f0, 0), b < ntiles, lane, pf);
  uint32_t dense_rows = 0;  // rows of this tile redone by the dense filterbank (wave-uniform)
  for (; b < ntiles; b += nwaves) {
    const int64_t nf = (send[c] - sbeg[c] + kHop - 1) / kHop;
    const int cur_c = c;
    const int64_t cur_f0 = f0;
    const int bn = b + nwaves;
    const int cn = bn < ntiles ? tclip[bn] : c;
    const int64_t fn0 = bn < ntiles ? (int64_t)(bn - toff[cn]) * kWaveFrames : f0;

    for (int sub = 0; sub < 4; sub++) {
      const int row = sub * 4 + grp;
      // stage this pass's PCM (prefetched; hop h at h * kHopStride) and prefetch the next pass
      wave_sync();  // the previous pass's readers of the scratch are done
      Smp* const stage = reinterpret_cast<Smp*>(kF32 ? (void*)M.pcmf : (void*)M.pcm);
#pragma unroll
      for (int r = 0; r < Ly::kRounds; r++) {
        const int chunk = lane + 64 * r;
        if (chunk < Ly::kChunks)
          *reinterpret_cast<int4*>(stage + (chunk / Ly::kHopChunks) * kHopStride + (chunk % Ly::kHopChunks) * Ly::kPer) =
              pf[r];
      }
      {
        const bool same = sub < 3;
        fetch_pass(pass_src(same ? cur_c : cn, same ? cur_f0 : fn0, same ? sub + 1 : 0), same || bn < ntiles, lane, pf);
      }
      wave_sync();
      // z[m] = x[2m] + i x[2m+1], x = fftshift(hanningz * [hop f-1 | hop f]); lane L holds
      // m = 16 n1 + L: for n1 < 8 the sample pair 32 n1 + 2L of hop f (window half 2), for
      // n1 >= 8 the pair 32 (n1 - 8) + 2L of hop f-1. Frame grp's hops are staged hops grp, grp+1.
      const Smp* hop0 = stage + grp * kHopStride;
      // Opaque zero: keeps the per-lane table reads in LDS instead of letting the compiler hoist
      // ~90 of them into registers for the whole kernel (occupancy).
      int oz = 0;
      asm volatile("" : "+v"(oz));
      const float* __restrict__ win = S.window + oz;  // read per pass (registers: occupancy)
      cf z[16], Y[16];
      {
#pragma unroll
        for (int n1 = 0; n1 < 16; n1++) {
          const int j = (32 * n1 + 2 * L + 256) & 511;
          const int hsel = n1 < 8 ? 1 : 0;
          const cf wj = *reinterpret_cast<const cf*>(win + j);  // j even
          if constexpr (kF32) {
            z[n1] = *reinterpret_cast<const cf*>(hop0 + hsel * kHopStride + (j & 255)) * wj;  // x * hanningz[j]
          } else {
            const int32_t v = *reinterpret_cast<const int32_t*>(hop0 + hsel * kHopStride + (j & 255));
            z[n1] = cf{(float)(int16_t)(v & 0xffff), (float)(int16_t)(v >> 16)} * wj;  // (s / 32768) * hanningz[j]
          }
        }
      }
      {
        dft16(w16r, z, Y);
#pragma unroll
        for (int k1 = 1; k1 < 16; k1++) Y[k1] = cmul(Y[k1], ltw[k1 - 1]);
        wave_sync();  // every lane has read its PCM: the scratch becomes the transpose square
#pragma unroll
        for (int k1 = 0; k1 < 16; k1++) W[L * kSq + k1] = Y[k1];
        wave_sync();
#pragma unroll
        for (int n2 = 0; n2 < 16; n2++) z[n2] = W[n2 * kSq + L];
        dft16(w16r, z, Y);  // Y[k2] = Z[L + 16 k2]
      }
      wave_sync();  // every lane has read its column of the square: W is free for |X|
      // |X[k]| of the 512-point real FFT, k = L + 16 k2, needs Z[256 - k]: for L >= 1 that is
      // Y[15 - k2] of lane 16 - L, for L = 0 it is this lane's own Y[16 - k2] (Z[256] = Z[0]).
      {
        // branch-free: generic split + corrected v_sqrt for every k; lanes whose |X|^2 falls
        // outside [2^-100, 2^100) redo that bin with the full IEEE sqrt below (wave-uniform
        // test, practically never taken); lane 0 then writes the two real bins 0 and 256.
        bool rare = false;
        cf P[16];  // every partner fetched before the first use: the 32 bpermutes overlap
#pragma unroll
        for (int k2 = 0; k2 < 16; k2++) P[k2] = cf{partner16(Y[15 - k2].x), partner16(Y[15 - k2].y)};
#pragma unroll
        for (int k2 = 0; k2 < 16; k2++) {
          const int k = L + 16 * k2;
          const cf own = Y[(16 - k2) & 15];
          const cf Pk = cf{L == 0 ? own.x : P[k2].x, L == 0 ? own.y : P[k2].y};
          const float x = split_power(Y[k2], Pk, S.tw512[k + oz]);
          rare |= !(x >= 0x1p-100f && x < 0x1p100f);
          N[k] = sqrtf_fast_cr(x);
        }
        if (__builtin_expect(__any(rare), 0)) {
          for (int k2 = 0; k2 < 16; k2++) {
            const int k = L + 16 * k2;
            cf Q = cf{partner16(Y[15 - k2].x), partner16(Y[15 - k2].y)};
            if (L == 0) Q = Y[(16 - k2) & 15];
            const float x = split_power(Y[k2], Q, S.tw512[k]);
            if (!(x >= 0x1p-100f && x < 0x1p100f)) N[k] = __builtin_sqrtf(x);
          }
        }
        if (L == 0) {
          N[0] = fabsf(Y[0].x + Y[0].y);
          N[256] = fabsf(Y[0].x - Y[0].y);
        }
      }
      for (int i = 257 + L; i < maxbin; i += 16) N[i] = 0.f;  // bins past 256 read by padded filters
      wave_sync();
      // Filterbank: this lane's 3 filters (slots A, B, C) summed interleaved, each in ascending
      // bin order from 0 (fmat_vecmul); then fvec_log10 of each.
      float* lrow = M.logs + row * kLogStride;
      {
        const int stA = S.ms_start[0][L], stB = S.ms_start[1][L], stC = S.ms_start[2][L];
        float aA = 0.f, aB = 0.f, aC = 0.f;
        const int oA = S.ms_woff[0] + 4 * L, oB = S.ms_woff[1] + 4 * L, oC = S.ms_woff[2] + 4 * L;
        if (ms_in_lds && lenA == 36 && lenB == 16 && lenC == 8)  // the 8 kHz schedule
          mel3_fixed<36, 16, 8>(N, S.ms_w + oA, S.ms_w + oB, S.ms_w + oC, stA, stB, stC, aA, aB, aC);
        else if (ms_in_lds)
          mel3(N, S.ms_w + oA, S.ms_w + oB, S.ms_w + oC, stA, stB, stC, lenA, lenB, lenC, aA, aB, aC);
        else
          mel3(N, T->ms_w + oA, T->ms_w + oB, T->ms_w + oC, stA, stB, stC, lenA, lenB, lenC, aA, aB, aC);
        // three independent log chains, computed unconditionally so they interleave (ILP 3)
        const float lA = aubio_log10_fast(aA, S.logf);  // branch-free: the chains interleave
        const float lB = aubio_log10_fast(aB, S.logf);
        if (fA >= 0) lrow[fA] = lA;
        if (fB >= 0) lrow[fB] = lB;
        if (c_defer) {
          if (c_real) lrow[fC] = aC;  // raw sum: its log is taken in the tile tail
        } else {
          const float lC = aubio_log10_fast(aC, S.logf);
          if (fC >= 0) lrow[fC] = lC;
        }
        // A non-finite |X| bin or band sum (fp32 samples near FLT_MAX, or inf / NaN samples of a
        // float WAV): aubio's dense fmat_vecmul multiplies every bin by every filter's weight, so
        // 0 * inf = NaN reaches bands the sparse slots skip, and fvec_log10 passes NaN and inf
        // through (the fast log assumes finite sums). Such frames are redone densely, in bin
        // order, with the full clamped log (wave-uniform test, never taken for int16 PCM).
        bool bad = !(aA <= 3.40282347e38f) || !(aB <= 3.40282347e38f) || !(aC <= 3.40282347e38f);
        for (int i = L; i < kBins; i += 16) bad |= !(N[i] <= 3.40282347e38f);
        const unsigned long long bm = __ballot(bad);
        if (__builtin_expect(bm != 0, 0)) {
          wave_sync();  // every lane's sparse results are in the row before it is rewritten
          if ((bm >> (16 * grp)) & 0xffffull) {
            for (int j = L; j < kFilters; j += 16) {
              const int st = T->mel_start[j], len = T->mel_len[j], off = T->mel_off[j];
              float acc = 0.f;
              for (int i = 0; i < kBins; i++) {
                const float w = (i >= st && i < st + len) ? T->mel_w[off + i - st] : 0.f;
                acc = acc + N[i] * w;
              }
              lrow[j] = aubio_log10_clamped(acc, S.logf);
            }
          }
#pragma unroll
          for (int g = 0; g < 4; g++)
            if ((bm >> (16 * g)) & 0xffffull) dense_rows |= 1u << (sub * 4 + g);
        }
      }
    }
    wave_sync();
    if (c_defer) {  // the deferred slot-2 logs: lane = (frame row, filter)
      if (lane < 2 * kWaveFrames && !((dense_rows >> (lane >> 1)) & 1u)) {
        const int f = S.c_real[lane & 1];
        if (f >= 0) {
          float* p = M.logs + (lane >> 1) * kLogStride + f;
          *p = aubio_log10_fast(*p, S.logf);
        }
      }
      wave_sync();
    }
    // Tail: lane = (frame row, coef) for the tile's 16 frames: DCT row (fmat_vecmul order),
    // 10*log10|c| (fp_handler.c:651), "%f" micro-units / NULL (db_ctx_handler.c:479-481).
    if (lane < 2 * kWaveFrames) {
      const int row = lane >> 1, cf = lane & 1;
      const int64_t f = cur_f0 + row;
      if (f < nf) {
        const float* lrow = M.logs + row * kLogStride;
        float acc = 0.f;
#pragma unroll 8
        for (int i = 0; i < kFilters; i++) acc = acc + lrow[i] * S.dct[cf][i];
        const double q = db ? db_of_coef(acc, fx) : db_of_coef(acc);  // frame values glibc-exact
        const int64_t g = foff[cur_c] + f;
        micro[2 * g + cf] = micro_of_db(q);
        if (db) db[2 * g + cf] = q;
      }
    }
    wave_sync();  // the log buffer is rewritten by the next tile
    if (__builtin_expect(dense_rows != 0, 0)) {  // dense rows overwrote the empty filters' constant
      const float lempty = aubio_log10_fast(0.f, S.logf);
      for (int i = lane; i < kWaveFrames * kFilters; i += 64) {
        const int r = i / kFilters, j = i % kFilters;
        if (((dense_rows >> r) & 1u) && T->mel_len[j] == 0) M.logs[r * kLogStride + j] = lempty;
      }
      dense_rows = 0;
      wave_sync();
    }
    c = cn;
    f0 = fn0;
  }
}

// ------------------------------------------------------------------------------------
// 8 kHz specialization of fingerprint_kernel (the configs' rate; DspTables::fixed8k()):
// the same arithmetic, with the filterbank slot schedule (36/16/8 bins, slot 2 = 2 real
// filters, deferred logs) fixed at compile time, so the pass has no schedule branches, and:
//   * tile and pass addressing in scalar registers (clip, tile and bounds are wave-uniform):
//     interior passes issue their 16-byte PCM loads unconditionally from an SGPR base;
//   * dft16's multiply by W16^4 = (0, -1) done as a swap (exact up to the sign of a zero,
//     which no magnitude sees);
//   * the real split's 0.5 folded into the filterbank: S = E + T = 2X exactly, the kernel
//     stores N' = sqrt(|S|^2) = 2|X| and sums with half weights w/2, so every product
//     (w/2)(2|X|) and every partial sum equals aubio's w|X| bit for bit (exact power-of-2
//     scalings; proof in DESIGN.md §4); bins with 0 < |S|^2 < 2^-98 (where the scaling or the
//     fast sqrt could round differently) take the spec sequence in a wave-uniform slow path;
//   * filterbank products formed in pairs (v_pk_mul_f32 on the b128 halves), sums sequential.
// dft16 with the W16^4 = (0, -1) multiply of A[2][2] as (y, -x), folded into the dft4 that takes
// it as a2: t0 = a0 + (y, -x) = addsub(a0, swap(A)), t1 = a0 - (y, -x) = subadd(a0, swap(A)),
// the same two roundings (c + (-p) == c - p), with no negation or move.
__device__ __forceinline__ void dft4_rot_a2(cf a0, cf a1, cf A2, cf a3, cf& X0, cf& X1, cf& X2, cf& X3) {
  const cf t0 = addsub(a0, swap(A2)), t1 = subadd(a0, swap(A2)), t2 = a1 + a3, t3 = a1 - a3;
  X0 = t0 + t2;
  X2 = t0 - t2;
  X1 = addsub(t1, swap(t3));
  X3 = subadd(t1, swap(t3));
}
// The two 45-degree twiddles in two ops instead of three. W16^2 = (c, -c) and W16^6 = (d, d)
// (DspTables_fixed8k checks the table halves are equal in magnitude). With p = a c = (a.x c, a.y c):
// the spec's (a.x c - a.y (-c), a.x (-c) + a.y c) is (p.x + p.y, p.y - p.x) bitwise (b (-c) =
// -(b c) exactly, x - (-y) == x + y), and (a.x d - a.y d, a.x d + a.y d) is (p.x - p.y, p.y + p.x).
__device__ __forceinline__ cf cmul_w2(cf a, float c) {
  const cf p = a * cf{c, c};
  return addsub(p, swap(p));
}
__device__ __forceinline__ cf cmul_w6(cf a, float d) {
  const cf p = a * cf{d, d};
  return subadd(p, swap(p));
}
__device__ __forceinline__ void dft16q(const cf (&w16)[10], const cf (&in)[16], cf (&out)[16]) {
  cf A[4][4];
#pragma unroll
  for (int n2 = 0; n2 < 4; n2++) dft4(in[n2], in[4 + n2], in[8 + n2], in[12 + n2], A[n2][0], A[n2][1], A[n2][2], A[n2][3]);
#pragma unroll
  for (int n2 = 1; n2 < 4; n2++)
#pragma unroll
    for (int k1 = 1; k1 < 4; k1++) {
      const int e = n2 * k1;
      if (e == 2) A[n2][k1] = cmul_w2(A[n2][k1], w16[2].x);
      else if (e == 6) A[n2][k1] = cmul_w6(A[n2][k1], w16[6].x);
      else if (e != 4) A[n2][k1] = cmul(A[n2][k1], w16[e]);
    }
#pragma unroll
  for (int k1 = 0; k1 < 4; k1++) {
    if (k1 == 2) dft4_rot_a2(A[0][k1], A[1][k1], A[2][k1], A[3][k1], out[k1], out[k1 + 4], out[k1 + 8], out[k1 + 12]);
    else dft4(A[0][k1], A[1][k1], A[2][k1], A[3][k1], out[k1], out[k1 + 4], out[k1 + 8], out[k1 + 12]);
  }
}

// Filterbank sum over LEN bins (multiple of 4), weights already in registers, products in
// pairs: acc = (((0 + n0 w0) + n1 w1) + n2 w2) + ... in ascending bin order. Every product is
// >= +0 (half weights >= 0, |X| from sqrt of a sum of squares), so 0 + n0 w0 is n0 w0 bitwise.
template <int LEN>
__device__ __forceinline__ float mel_sum_w(const float* __restrict__ N, const float4 (&wv)[LEN / 4], int st) {
  float4 nv[LEN / 4];
#pragma unroll
  for (int i = 0; i < LEN / 4; i++) nv[i] = *reinterpret_cast<const float4*>(N + st + 4 * i);
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < LEN / 4; i++) {
    const cf p01 = cf{nv[i].x, nv[i].y} * cf{wv[i].x, wv[i].y};
    const cf p23 = cf{nv[i].z, nv[i].w} * cf{wv[i].z, wv[i].w};
    acc = i == 0 ? p01.x : acc + p01.x;
    acc = acc + p01.y; acc = acc + p23.x; acc = acc + p23.y;
  }
  return acc;
}
template <int LEN>
__device__ __forceinline__ void load_w(const float* __restrict__ w, float4 (&wv)[LEN / 4]) {
#pragma unroll
  for (int i = 0; i < LEN / 4; i++) wv[i] = *reinterpret_cast<const float4*>(w + 64 * i);
}

// Phase stamps (experiment builds only, -DTFP_STAMPS): per-wave s_memtime deltas at the pass's
// existing wave_syncs (no extra waits), printed by a few waves at exit.
#ifdef TFP_STAMPS
#define TFP_STAMP(i) const uint64_t ts##i = __builtin_amdgcn_s_memtime()
#define TFP_ACC(i, a, b) st[i] += ts##b - ts##a
#else
#define TFP_STAMP(i)
#define TFP_ACC(i, a, b)
#endif

// kPasses = passes of 4 frames per tile: 4 (16-frame tiles, throughput) or 1 (4-frame tiles, for
// small batches: 4x the waves on a short query, a quarter of the per-wave latency).
template <int kPasses>
__global__ __launch_bounds__(64 * fp8_block_waves<kPasses>(), TFP_FP_WAVES) void fingerprint8k_kernel(
    const DspTables* __restrict__ T, const int16_t* __restrict__ pcm, const int64_t* __restrict__ sbeg,
    const int64_t* __restrict__ send, const int64_t* __restrict__ foff, const int32_t* __restrict__ toff,
    const int32_t* __restrict__ tclip, int32_t ntiles, int32_t* __restrict__ micro, double* __restrict__ db,
    float rare_thr, LogFix fx, int64_t single_ns) {
  constexpr int LA = 36, LB = 16, LC = 8;  // DspTables::fixed8k()
  // dB + "%f" in finish_db_kernel for throughput launches (full waves); in the tile tail for small
  // ones (4-frame tiles, batch-1 latency), which saves a launch
  constexpr bool kSplitTail = kPasses >= 2;
#ifdef TFP_STAMPS
  const uint64_t t_entry = __builtin_amdgcn_s_memtime();
#endif
  const uint32_t rare_m1 = __builtin_bit_cast(uint32_t, rare_thr) - 1u;  // 2^-98 (tests may raise it)
  // filterbank weights: the frame-pair schedule (throughput) or the slot schedule (small tiles)
  constexpr bool kPairFb = kPasses >= 2;
  constexpr int kBW = fp8_block_waves<kPasses>();
  using WaveT = WaveLds8;
  __shared__ __attribute__((aligned(16))) LdsTables S;
  __shared__ __attribute__((aligned(16))) WaveT WL[kBW];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, grp = lane >> 4, L = lane & 15;
  // Wave-uniform tile state (scalar registers): clip, first frame, clip sample range.
  struct Tile {
    int c;
    int64_t f0, s0, ns;
    __amdgpu_buffer_rsrc_t rs;  // (throughput launches) the clip's whole 4-byte words, fetchd
    bool odd;                   // ... and whether it starts on an odd sample
  };
  // The clip's bytes as a buffer: its whole 4-byte words (an odd start: from one sample before).
  auto clip_rsrc = [&](int64_t s0, int64_t ns) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(pcm + s0);
    const int16_t* base = reinterpret_cast<const int16_t*>(a & ~(uintptr_t)3);
    const int64_t bytes = (2 * ns + (int64_t)(a & 3) + 3) & ~(int64_t)3;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(base), (short)0, (int)bytes, 0x00020000);
  };
  auto tile_of = [&](int b) {
    Tile t;
    if (single_ns >= 0) {  // one clip at d_pcm[0]: no layout loads
      t.c = 0;
      t.f0 = (int64_t)b * (4 * kPasses);
      t.s0 = 0;
      t.ns = single_ns;
      return t;
    }
    t.c = __builtin_amdgcn_readfirstlane(tclip[b]);
    t.f0 = (int64_t)(b - toff[t.c]) * (4 * kPasses);
    t.s0 = sbeg[t.c];
    t.ns = send[t.c] - t.s0;
    if constexpr (kPairFb) {
      t.rs = clip_rsrc(t.s0, t.ns);
      t.odd = (reinterpret_cast<uintptr_t>(pcm + t.s0) & 3) != 0;
    }
    return t;
  };
  // 16-byte PCM chunks of pass `sub` of tile t (samples [(f0 + 4 sub - 1) 256, + 1280)) into registers.
  auto fetch = [&](const Tile& t, int sub, bool valid, int4 (&pf)[kChunkRounds]) {
    const int16_t* clip = pcm + t.s0;
    const int64_t sb = (t.f0 + 4 * sub - 1) * kHop;
    const bool interior = valid && ((reinterpret_cast<uintptr_t>(clip) & 15) == 0) && sb >= 0 && sb + kPassSamples <= t.ns;
    if (interior) {
      const int4* src = reinterpret_cast<const int4*>(clip + sb);
#pragma unroll
      for (int r = 0; r < kChunkRounds; r++) {
        const int chunk = lane + 64 * r;
        pf[r] = (64 * r + 63 < kPassChunks || chunk < kPassChunks) ? src[chunk] : make_int4(0, 0, 0, 0);
      }
    } else if constexpr (kPasses == 1) {
      // clip edges of a small launch (its PCM may be across PCIe): chunks wholly inside are one
      // 16-byte load, wholly outside zeros, no call (a call waits for every outstanding load).
      // (Throughput launches inline too measured within noise: profiles/r04/edge_fetch_ab_r04m.txt.)
      const bool aligned = (reinterpret_cast<uintptr_t>(clip) & 15) == 0;
#pragma unroll
      for (int r = 0; r < kChunkRounds; r++) {
        const int chunk = lane + 64 * r;
        const int64_t s0 = sb + 8 * chunk;
        int4 v = make_int4(0, 0, 0, 0);
        if (valid && chunk < kPassChunks && s0 + 8 > 0 && s0 < t.ns) {
          if (aligned && s0 >= 0 && s0 + 8 <= t.ns) v = *reinterpret_cast<const int4*>(clip + s0);
          else v = fetch_chunk_inline(clip, t.ns, s0);  // straddling the end, or an unaligned clip
        }
        pf[r] = v;
      }
    } else {  // (throughput launches: 2 edge passes per clip, their latency hidden; less code in the loop)
#pragma unroll
      for (int r = 0; r < kChunkRounds; r++) {
        const int chunk = lane + 64 * r;
        pf[r] = (valid && chunk < kPassChunks) ? fetch_chunk_checked(clip, t.ns, sb + 8 * chunk) : make_int4(0, 0, 0, 0);
      }
    }
  };

  // Direct PCM (throughput launches, round 5): lane (grp, L) loads its own frame's 16 sample
  // pairs straight into registers, one pass ahead: for n1 < 8 the pair 32 n1 + 2L of hop f, for
  // n1 >= 8 the pair 32 (n1 - 8) + 2L of hop f - 1 (z's fftshifted layout), as buffer loads over
  // the clip's bytes, one offset register and immediate offsets. No LDS staging of the pass's PCM
  // (3 16-byte stores and 8 paired reads per lane before). Samples outside the clip (the zero hop
  // before frame 0, the zero-padded tail) are masked where the pass uses them (pcm_pair); the
  // buffer's range only keeps every load inside the clip's 4-byte words (0 beyond). A clip that
  // starts on an odd sample (a stream window after odd-sized ticks) has no 4-byte-aligned pairs:
  // its passes read each pair from two aligned words, synchronously (pcm_pair_odd).
  // (a launch's last tiles fetch their "next" pass from their own clip: loaded, never used)
  auto fetchd = [&](const Tile& t, int sub, uint32_t (&pw)[16]) {
    if (t.odd) return;  // (odd start: read when used)
    const __amdgpu_buffer_rsrc_t rs = t.rs;
    const int32_t fs = (int32_t)((t.f0 + 4 * sub - 1 + grp) * kHop) + 2 * L;  // this frame's first sample + 2L
#pragma unroll
    for (int n1 = 0; n1 < 16; n1++) {
      const int32_t j = n1 < 8 ? 256 + 32 * n1 : 32 * (n1 - 8);
      pw[n1] = __builtin_amdgcn_raw_buffer_load_b32(rs, 2 * (fs + j), 0, 0);
    }
  };

  // The first tile's bounds are known before the tables are staged (a one-clip launch passes
  // them as an argument), and its PCM is requested right after the table loads, so its latency
  // overlaps the staging (most of a small launch's time). The PCM is prefetched one pass ahead
  // (a two-pass distance measured no faster: the pass is bound by instruction issue, not by the
  // PCM loads).
  int4 pf[kChunkRounds];
  uint32_t pw[16];  // (throughput launches: the next pass's sample pairs, fetchd)
  int b = blockIdx.x * kBW + wave;
  Tile cur = tile_of(b < ntiles ? b : 0);
  // window and split twiddles in lane-interleaved pair layouts, [i][L][2] cf: lane L's values for
  // n1 (k2) = 2i, 2i+1 are one conflict-free ds_read_b128 (16 lanes read 256 consecutive bytes)
  cf* winr = reinterpret_cast<cf*>(S.window);
  cf* twr = S.tw512;
  // Table staging: every global load below is issued before any LDS write (indices clamped,
  // writes predicated), so a block waits for one round trip instead of one per table: a small
  // launch is latency-bound.
  // The first 256 threads stage (one entry per thread per table).
  constexpr int kStage = 256;
  const int ts = tid < kStage ? tid : kStage - 1;
  const bool stager = tid < kStage;
  constexpr int kMsW = kPairFb ? kFbSteps * kFbPatterns : 16 * (LA + LB + LC);  // DspTables_fixed8k
  const float* const wsrc = kPairFb ? &T->fb_w[0][0][0] : T->ms_w;
  const int wL = (ts >> 1) & 15, wn1 = 2 * (ts >> 5) + (ts & 1);
  const int wj = (32 * wn1 + 2 * wL + 256) & 511;
  const float win0 = T->window_s[wj], win1 = T->window_s[wj + 1];
  // [k2][L] = (re w512^k, re w512^k', im w512^k, im w512^k'), k = L + 16 k2, k' = 256 - k (k2 < 8;
  // lane 0 at k2 = 0: k = 128): the pair layout of split_pair_sq
  const int tk2 = ts >> 5, tkk = (wL == 0 && tk2 == 0) ? 128 : wL + 16 * tk2;
  const float* tws = (ts & 1) ? T->tw512_im : T->tw512_re;
  const float twk = tws[tkk], twk2 = tws[256 - tkk];
  const int li = ts < 240 ? ts : 239, lk1 = 1 + li / 16, lL = li % 16;
  const float ltre = T->lane_tw_re[lk1][lL], ltim = T->lane_tw_im[lk1][lL];
  const int i10 = ts < 10 ? ts : 9;
  const float w16re = T->tw256_re[16 * i10], w16im = T->tw256_im[16 * i10];
  const int i80 = ts < kCoefs * kFilters ? ts : kCoefs * kFilters - 1;
  const float dctv = (&T->dct[0][0])[i80];
  const int i48 = ts < 48 ? ts : 47;
  const int msf = (&T->ms_filter[0][0])[i48], mss = (&T->ms_start[0][0])[i48];
  const int i3 = ts < 3 ? ts : 2;
  const int msl = T->ms_len[i3], mso = T->ms_woff[i3];
  const LogfEntry lge = logf_table()[ts & 15];
  float mw[(kMsW + kStage - 1) / kStage];
#pragma unroll
  for (int r = 0; r < (kMsW + kStage - 1) / kStage; r++) {
    int idx = ts + kStage * r;
    idx = idx < kMsW ? idx : kMsW - 1;
    if constexpr (kPairFb) {
      // LDS layout [step / 4][pattern][step % 4] (a lane's weights of two step pairs are one
      // ds_read_b128: 4 LDS cycles, where two 8-byte reads took 8) from the table's [step / 2][pattern][step % 2]
      const int q = idx & 3, pat = (idx >> 2) & 15, s4 = idx >> 6;
      idx = ((2 * s4 + (q >> 1)) * kFbPatterns + pat) * 2 + (q & 1);
    }
    mw[r] = wsrc[idx];
  }
  const int mlen = T->mel_len[lane < kFilters ? lane : kFilters - 1];
  // the first pass's PCM after the table loads (loads complete in order, so the tables' waits
  // would otherwise include the PCM's: a batch-1 query's is read across PCIe)
  if constexpr (kPairFb) fetchd(cur, 0, pw);
  else fetch(cur, 0, b < ntiles, pf);
  if (stager) {
    winr[tid] = cf{win0, win1};
    twr[tid] = cf{twk, twk2};
  if (tid < 240) S.lane_tw[lk1 - 1][lL] = cf{ltre, ltim};
  if (tid < 10) S.w16[tid] = cf{w16re, w16im};
  if (tid < kCoefs * kFilters) (&S.dct[0][0])[tid] = dctv;
  if (tid < 48) {
    (&S.ms_filter[0][0])[tid] = msf;
    (&S.ms_start[0][0])[tid] = mss;
  }
  if (tid < 3) { S.ms_len[tid] = msl; S.ms_woff[tid] = mso; }
  if (tid < 16) S.logf[tid] = lge;
  if (kPairFb && tid < kLogf2Entries) S.logf2[tid] = logf2_entry(tid, logf_table());
  if (tid == 0) { S.c_defer = T->ms_c_defer; S.c_real[0] = T->ms_c_real[0]; S.c_real[1] = T->ms_c_real[1]; }
#pragma unroll
    for (int r = 0; r < (kMsW + kStage - 1) / kStage; r++) {
      const int idx = tid + kStage * r;
      if (idx < kMsW) S.ms_w[idx] = 0.5f * mw[r];  // exact: w/2
    }
  }
  const unsigned long long empty_filters = __ballot(lane < kFilters && mlen == 0);  // (log of 0 + 2e-42)
  __syncthreads();
#ifdef TFP_STAMPS
  const uint64_t t_staged = __builtin_amdgcn_s_memtime();
#endif

  WaveT& M = WL[wave];
  cf* W = M.scratch[grp];
  float* N = reinterpret_cast<float*>(W) + 48 * (grp & 1);  // |X| row (WaveLds8)
  const int nwaves = gridDim.x * kBW;
  const int maxbin = T->ms_maxbin;
  const int fA = S.ms_filter[0][L], fB = S.ms_filter[1][L], fC = S.ms_filter[2][L];
  const bool c_real = fC >= 0 && (fC == S.c_real[0] || fC == S.c_real[1]);
  // dft16's twiddles W16^e (e = 1, 2, 3, 6, 9 used) are wave-uniform: scalar loads, held in SGPRs
  // for the kernel (no LDS read per pass)
  cf w16r[10];
#pragma unroll
  for (int e = 0; e < 10; e++)
    w16r[e] = cf{T->tw256_re[16 * e], T->tw256_im[16 * e]};
  // inter-stage lane twiddles w256^(L k1) held in registers (30 VGPRs) instead of read per pass
  cf ltw[15];
#pragma unroll
  for (int k1 = 1; k1 < 16; k1++) ltw[k1 - 1] = S.lane_tw[k1 - 1][L];
  const float lempty = aubio_log10_fast(0.f, S.logf);  // log of an empty filter's clamped 0
  if constexpr (!kPairFb) {
    for (int i = lane; i < 4 * kPasses * kFilters; i += 64) {
      const int j = i % kFilters;
      if ((empty_filters >> j) & 1) M.logs[(i / kFilters) * kLogStride + j] = lempty;
    }
  }
  // Frame-pair filterbank (kPairFb): lane = pair grp x pattern L. Pair grp's rows: the even
  // pass's pairs 0, 1 in xeven, the odd pass's in the scratch. Per segment k: the read base (step
  // s reads the bins at fbb[k] + 2 s), where the job's raw sums go (frames 2 grp, 2 grp + 1 of
  // double pass 0: rows 4 grp, 4 grp + 2; double pass 1 one row on), and 0 where the segment
  // starts a job (acc = fma(acc, 0, p) = p; 1: acc + p).
  const float* fbb[kFbSegs];
  float* fbc[kFbSegs];
  float fbk[kFbSegs];
  cf dctl, dct9;  // the DCT weights (rows 0, 1) of this lane's filter in the tail's log rounds
  const float* const fbrow = (grp < 2 ? M.xeven : reinterpret_cast<const float*>(M.scratch)) + (grp & 1) * kFbRow;
  float* const fblog = M.logs + 4 * grp * kFbNf;
  if constexpr (kPairFb) {
    const int lf = lane < kFbNf ? lane : lane - kFbNf, l9 = kFbNf - 4 + (lane & 3);
    dctl = cf{S.dct[0][lf], S.dct[1][lf]};
    dct9 = cf{S.dct[0][l9], S.dct[1][l9]};
#pragma unroll
    for (int k = 0; k < kFbSegs; k++) {
      fbb[k] = fbrow + 2 * (T->fb_bin[L][k] - kFbSegStart[k]);
      fbc[k] = fblog + T->fb_filter[L][k];
      fbk[k] = T->fb_new[L][k] ? 0.f : 1.f;
    }
  }

#ifdef TFP_STAMPS
  uint64_t st[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t tprev = __builtin_amdgcn_s_memtime();
  const uint64_t tstart = tprev;
  int npass = 0;
#endif
  for (; b < ntiles; b += nwaves) {
    const int64_t nf = (cur.ns + kHop - 1) / kHop;
    const int bn = b + nwaves;
    const Tile nxt = bn < ntiles ? tile_of(bn) : cur;

    for (int sub = 0; sub < kPasses; sub++) {
      const int row = sub * 4 + grp;
      // Opaque zero: keeps the per-lane table reads in LDS instead of letting the compiler hoist
      // them into registers for the whole kernel (occupancy).
      int oz = 0;
      asm volatile("" : "+v"(oz));
      wave_sync();  // the previous pass's readers of the scratch are done
      TFP_STAMP(0);
      // the pass's window values (a table no one writes) requested with the PCM staging, so the
      // staging's sync waits for both at once
      cf wreg[16];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const float4 w4 = *reinterpret_cast<const float4*>(winr + (i * 16 + L) * 2 + oz);
        wreg[2 * i] = cf{w4.x, w4.y};
        wreg[2 * i + 1] = cf{w4.z, w4.w};
      }
      if constexpr (!kPairFb) {
#pragma unroll
        for (int r = 0; r < kChunkRounds; r++) {
          const int chunk = lane + 64 * r;
          if (chunk < kPassChunks) *reinterpret_cast<int4*>(M.pcm + (chunk >> 5) * kHopStride + (chunk & 31) * 8) = pf[r];
        }
        if (sub < kPasses - 1) fetch(cur, sub + 1, true, pf);
        else fetch(nxt, 0, bn < ntiles, pf);
      }
      wave_sync();
      TFP_STAMP(1);
      const int16_t* hop0 = M.pcm + grp * kHopStride;
      // z[m] = x[2m] + i x[2m+1], x = fftshift(hanningz * [hop f-1 | hop f]); lane L holds
      // m = 16 n1 + L: for n1 < 8 the sample pair 32 n1 + 2L of hop f (window half 2), for
      // n1 >= 8 the pair 32 (n1 - 8) + 2L of hop f-1. Frame grp's hops are staged hops grp, grp+1.
      cf z[16], Y[16];
      if constexpr (kPairFb) {
        const int64_t pb = (cur.f0 + 4 * sub - 1) * kHop;  // the pass's first sample
        const int32_t fs = (int32_t)(pb + grp * kHop) + 2 * L;
        if (cur.odd) {  // odd start: two aligned words per pair
          const __amdgpu_buffer_rsrc_t rs = cur.rs;
#pragma unroll
          for (int n1 = 0; n1 < 16; n1++) {
            const int32_t j = n1 < 8 ? 256 + 32 * n1 : 32 * (n1 - 8);
            const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs, 2 * (fs + j), 0, 0);  // (samples s - 1, s)
            const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs, 2 * (fs + j) + 4, 0, 0);
            pw[n1] = (lo >> 16) | (hi << 16);
          }
        }
        if (pb < 0 || pb + kPassSamples > cur.ns) {  // an edge pass: samples outside [0, ns) are 0 (aubio's padding)
#pragma unroll
          for (int n1 = 0; n1 < 16; n1++) {
            const int32_t s0 = fs + (n1 < 8 ? 256 + 32 * n1 : 32 * (n1 - 8));
            const uint32_t lo = (s0 >= 0 && s0 < cur.ns) ? 0xffffu : 0u;
            const uint32_t hi = (s0 + 1 >= 0 && s0 + 1 < cur.ns) ? 0xffff0000u : 0u;
            pw[n1] &= lo | hi;
          }
        }
      }
#pragma unroll
      for (int n1 = 0; n1 < 16; n1++) {
        int32_t v;
        if constexpr (kPairFb) {
          v = (int32_t)pw[n1];
        } else {
          const int j = (32 * n1 + 2 * L + 256) & 511;
          const int hsel = n1 < 8 ? 1 : 0;
          v = *reinterpret_cast<const int32_t*>(hop0 + hsel * kHopStride + (j & 255));
        }
        z[n1] = cf{(float)(int16_t)(v & 0xffff), (float)(int16_t)(v >> 16)} * wreg[n1];
      }
      if constexpr (kPairFb) {  // the next pass's samples, into the registers just read
        if (sub < kPasses - 1) fetchd(cur, sub + 1, pw);
        else fetchd(nxt, 0, pw);
      }
      dft16q(w16r, z, Y);
#pragma unroll
      for (int k1 = 1; k1 < 16; k1++) Y[k1] = cmul(Y[k1], ltw[k1 - 1]);
      wave_sync();  // every lane has read its PCM: the scratch becomes the transpose square
      TFP_STAMP(2);
      // the split's twiddles (a table no one writes) requested with the square's writes, so the
      // square's sync waits for both at once
      const float4* tw4 = reinterpret_cast<const float4*>(twr + 2 * L + oz);  // + 16 k2: one base, immediate offsets
      float4 t4s[8];
#pragma unroll
      for (int k2 = 0; k2 < 8; k2++) t4s[k2] = tw4[16 * k2];
#pragma unroll
      for (int k1 = 0; k1 < 16; k1++) W[k1 * kSq8 + L] = Y[k1];
      wave_sync();
#pragma unroll
      for (int n2 = 0; n2 < 16; n2 += 2) {
        const float4 v = *reinterpret_cast<const float4*>(W + L * kSq8 + n2);
        z[n2] = cf{v.x, v.y};
        z[n2 + 1] = cf{v.z, v.w};
      }
      dft16q(w16r, z, Y);  // Y[k2] = Z[L + 16 k2]
      wave_sync();         // every lane has read its column of the square: W is free for |X|
      TFP_STAMP(3);
      // Real split per conjugate pair on one lane: lane L (k2 < 8) owns bins k = L + 16 k2 and
      // 256 - k, whose Z values are its Y[k2] and Y[15 - k2] of lane 16 - L (8 ds_bpermute pairs).
      // Column 0 pairs inside lane 0: (16 k2, 256 - 16 k2) for k2 = 1..7 and (128, 128) at k2 = 0;
      // bins 0 and 256 come from Z[0] below. The spec's partner-side operands are exact sign
      // flips of this side's: E' = (E.re, -E.im), O' = (-O.re, O.im) (a - b = -(b - a),
      // a + b = b + a in IEEE), so E and O are formed once per pair; each bin then takes its
      // own table twiddle (w512^k, w512^(256-k)) through the spec's T and S = E + T = 2X.
      cf Pq[8];
#pragma unroll
      for (int k2 = 0; k2 < 8; k2++) Pq[k2] = cf{partner16(Y[15 - k2].x), partner16(Y[15 - k2].y)};
      // bins 0 and 256 (lane 0) from Z[0], taken now so Y[0] is not kept alive
      const float n0 = 2.f * fabsf(Y[0].x + Y[0].y), n256 = 2.f * fabsf(Y[0].x - Y[0].y);
      // min over bins of bits(|S|^2) - 1: exact zeros wrap to the top. (On |S|^2 itself, not on its
      // v_sqrt_f32: that returns 0 for denormal inputs; tests/native/check_fast_sqrt.hip.)
      uint32_t umin = 0xffffffffu;
      float nk[8], nk2[8];
#pragma unroll
      for (int k2 = 0; k2 < 8; k2++) {
        const cf own = Y[k2 == 0 ? 8 : 16 - k2];
        cf y = Y[k2];
        if (k2 == 0) y = cf{L == 0 ? own.x : y.x, L == 0 ? own.y : y.y};
        const cf p = cf{L == 0 ? own.x : Pq[k2].x, L == 0 ? own.y : Pq[k2].y};
        const float4 t4 = t4s[k2];
        const cf sq = split_pair_sq(y, p, cf{t4.x, t4.y}, cf{t4.z, t4.w});
        sqrt_pair_cr(sq, nk[k2], nk2[k2]);
        umin = min(umin, rare_key_pair(sq));
      }
      // |X| rows, addressed as bins L + 16 k2 and 256 - that for every lane (paired ds_write2_b32);
      // lane 0's k2 = 0 pair is bin 128 twice (the partner-side value stands, below): its writes to
      // bins 0 and 256 are overwritten by n0 and n256. Bin b of this frame is NX[kXs * b]: its own
      // row (slot schedule) or its lane of the pair's interleaved row (frame-pair schedule).
      constexpr int kXs = kPairFb ? 2 : 1;
      float* const NX = kPairFb ? ((sub & 1) ? reinterpret_cast<float*>(M.scratch) : M.xeven) + (grp >> 1) * kFbRow + (grp & 1)
                                : N;
#pragma unroll
      for (int k2 = 0; k2 < 8; k2++) NX[kXs * (L + 16 * k2)] = nk[k2];
      float* const nrev = NX + kXs * (144 - L);  // bin 256 - L - 16 k2 = nrev[16 (7 - k2)]: one base, immediate offsets
#pragma unroll
      for (int k2 = 0; k2 < 8; k2++) nrev[kXs * 16 * (7 - k2)] = nk2[k2];
      if (L == 0) NX[kXs * 128] = nk2[0];  // before the slow path below, which may redo bin 128
      // 0 < |S|^2 < rare_thr (bits - 1 wraps exact zeros to the top): the spec's order below
      if (__builtin_expect(__any(umin < rare_m1), 0)) {  // redo the affected bins in the spec's order
#pragma unroll
        for (int k2 = 0; k2 < 8; k2++) {
          const cf own = Y[k2 == 0 ? 8 : 16 - k2];
          cf y = Y[k2];
          if (k2 == 0 && L == 0) y = own;
          const cf p = L == 0 ? own : Pq[k2];
          const float4 t4 = *reinterpret_cast<const float4*>(twr + (k2 * 16 + L) * 2);
          const cf sq = split_pair_sq(y, p, cf{t4.x, t4.y}, cf{t4.z, t4.w});
          const cf w = cf{t4.x, t4.z}, w2 = cf{t4.y, t4.w};
          const int k = (k2 == 0 && L == 0) ? 128 : L + 16 * k2;
          if (sq.x > 0.f && sq.x < rare_thr) NX[kXs * k] = 2.f * __builtin_sqrtf(split_power(y, p, w));
          if (sq.y > 0.f && sq.y < rare_thr) NX[kXs * (256 - k)] = 2.f * __builtin_sqrtf(split_power(p, y, w2));
        }
      }
      if (L == 0) {
        NX[0] = n0;
        NX[kXs * 256] = n256;
        if constexpr (kPairFb) NX[kXs * 257] = 0.f;  // the zero pad a pattern's last pair of bins may read
      }
      if constexpr (!kPairFb)
        for (int i = 257 + L; i < maxbin; i += 16) N[i] = 0.f;
      wave_sync();
      TFP_STAMP(4);
      if constexpr (!kPairFb) {
        // Filterbank: this lane's 3 filters (slots A, B, C) from the half weights, then the logs
        const float* wbase = S.ms_w + 4 * L + oz;
        float* lrow = M.logs + row * kLogStride;
        const int stA = S.ms_start[0][L], stB = S.ms_start[1][L], stC = S.ms_start[2][L];
        float4 wA[LA / 4], wB[LB / 4], wC[LC / 4];
        load_w<LC>(wbase + S.ms_woff[2], wC);
        load_w<LB>(wbase + S.ms_woff[1], wB);
        load_w<LA>(wbase + S.ms_woff[0], wA);
        const float aC = mel_sum_w<LC>(N, wC, stC);
        const float aB = mel_sum_w<LB>(N, wB, stB);
        const float aA = mel_sum_w<LA>(N, wA, stA);
        lrow[fA] = aubio_log10_fast(aA, S.logf);
        lrow[fB] = aubio_log10_fast(aB, S.logf);
        if (c_real) lrow[fC] = aC;  // raw sum: its log is taken in the tile tail
      } else if (sub & 1) {
        // Frame-pair filterbank over this double pass's 8 frames: each step multiplies a pair of
        // bins' (frame, frame) |X| by the pattern's half weight and adds both frames' products to
        // their sums in one packed op (sums sequential in ascending bins from the job's first
        // bin, as above); a job's raw sums go to the log rows at each of its segments' ends (the
        // last write stands), their logs are taken in the tile tail. One copy per double pass,
        // so the row offset of its sums is an immediate.
        auto pair_fb = [&](auto dp) {
          constexpr int doff = decltype(dp)::value * kFbNf;
          cf acc;
          const float* jb[kFbSegs];
          float* jc[kFbSegs];
          float jk[kFbSegs];
#pragma unroll
          for (int k = 0; k < kFbSegs; k++) {
            jb[k] = fbb[k];
            jc[k] = fbc[k];
            jk[k] = fbk[k];
          }
          // a step pair's weights: one ds_read_b64 each, whose halves the packed multiplies
          // broadcast with op_sel (a b128 of 4 steps made the compiler move the halves apart).
          // The segments' sums are stored after the last step: a store to the log rows between
          // them kept the compiler from hoisting the later reads above it (it cannot tell the two
          // LDS arrays apart), so the phase waited out the LDS latency once per segment.
          const f4v* const wfb = reinterpret_cast<const f4v*>(S.fbw) + L + oz;
          // Each segment's reads are issued one segment ahead of its sums (all of them at once
          // needed 108 VGPRs and spilled); the compiler barriers keep them in those groups.
          // (the weights of step pairs 2g, 2g + 1 are one read, with pair 2g's segment's)
          cf seg[kFbSegs];
          f4v wv4[kFbSteps / 4];
          f4v nv[kFbSteps / 2];
          static_assert(kFbSteps % 4 == 0, "weights in groups of 4 steps");
          auto load_seg = [&](auto kk) {
            constexpr int k = decltype(kk)::value;
#pragma unroll
            for (int st = kFbSegStart[k]; st < kFbSegStart[k + 1]; st += 2) {
              if ((st & 3) == 0) wv4[st >> 2] = wfb[(st >> 2) * kFbPatterns];
              nv[st >> 1] = *reinterpret_cast<const f4v*>(jb[k] + 2 * st);
            }
          };
          auto sum_seg = [&](auto kk) {
            constexpr int k = decltype(kk)::value;
#pragma unroll
            for (int st = kFbSegStart[k]; st < kFbSegStart[k + 1]; st += 2) {
              const int i = st >> 1;
              const f4v w = wv4[st >> 2];
              const float w0 = (st & 3) ? w.z : w.x, w1 = (st & 3) ? w.w : w.y;
              const cf p0 = cf{nv[i].x, nv[i].y} * cf{w0, w0};
              const cf p1 = cf{nv[i].z, nv[i].w} * cf{w1, w1};
              if (st == 0) acc = p0;
              else if (st == kFbSegStart[k]) acc = __builtin_elementwise_fma(acc, cf{jk[k], jk[k]}, p0);
              else acc = acc + p0;
              acc = acc + p1;
            }
            seg[k] = acc;
          };
          using I0 = std::integral_constant<int, 0>;
          using I1 = std::integral_constant<int, 1>;
          using I2 = std::integral_constant<int, 2>;
          using I3 = std::integral_constant<int, 3>;
          static_assert(kFbSegs == 4, "four segments");
          load_seg(I0{});
          load_seg(I1{});
          asm volatile("" ::: "memory");
          sum_seg(I0{});
          load_seg(I2{});
          asm volatile("" ::: "memory");
          sum_seg(I1{});
          load_seg(I3{});
          asm volatile("" ::: "memory");
          sum_seg(I2{});
          sum_seg(I3{});
#pragma unroll
          for (int k = 0; k < kFbSegs; k++) {
            jc[k][doff] = seg[k].x;
            jc[k][doff + 2 * kFbNf] = seg[k].y;
          }
        };
        if (sub == 1) pair_fb(std::integral_constant<int, 0>{});
        else pair_fb(std::integral_constant<int, 1>{});
      }
#ifdef TFP_STAMPS
      const uint64_t ts5 = __builtin_amdgcn_s_memtime();
      st[0] += ts0 - tprev;  // previous pass's end (or the tail) to this pass's first wave_sync
      TFP_ACC(1, 0, 1);      // PCM staging (prefetched registers -> LDS), next pass's loads issued
      TFP_ACC(2, 1, 2);      // PCM reads, window, DFT16, lane twiddles
      TFP_ACC(3, 2, 3);      // transpose square write + read, DFT16
      TFP_ACC(4, 3, 4);      // partner exchange, real split, sqrt, |X| writes, rare test
      TFP_ACC(5, 4, 5);      // filterbank + logs
      tprev = ts5;
      npass++;
#endif
    }
    wave_sync();
    if constexpr (kPairFb) {
      // The tile's 16 x kFbNf band logs, each times its two DCT weights (the DCT rows' products,
      // formed here once per log instead of per row term): round r < 8, lane l takes log row pair
      // (2r, 2r + 1) = frames r, r + 8 at filter l (l < 34) or l - 34, one filter per lane in
      // every round; the 32 left (filters 30..33 of frames 8..15) go to round 8. Products to the
      // free scratch as (c0, c1) pairs at the raw sum's index. All table reads issued up front.
      constexpr int kFull = 8;
      static_assert(kWaveFrames * kFbNf == kFull * 2 * kFbNf && 2 * kFbNf - 64 == 4, "log rounds");
      cf* const prod = reinterpret_cast<cf*>(M.scratch);
      LogArg g[kFull];
      LogfEntry en[kFull];
#pragma unroll
      for (int r = 0; r < kFull; r++) g[r] = log_reduce(M.logs[2 * kFbNf * r + lane]);
#pragma unroll
      for (int r = 0; r < kFull; r++) en[r] = S.logf2[g[r].idx];
#pragma unroll
      for (int r = 0; r < kFull; r++) {
        const float l = log_finish(g[r], en[r]);
        prod[2 * kFbNf * r + lane] = cf{l, l} * dctl;
      }
      if (lane < kWaveFrames * 2) {
        const int i = 2 * kFbNf * (lane >> 2) + 64 + (lane & 3);
        const float l = aubio_log10_frexp(M.logs[i], S.logf2);
        prod[i] = cf{l, l} * dct9;
      }
    } else if (lane < 2 * 4 * kPasses) {  // the deferred slot-2 logs: lane = (frame row, filter)
      const int f = S.c_real[lane & 1];
      if (f >= 0) {
        float* p = M.logs + (lane >> 1) * kLogStride + f;
        *p = aubio_log10_fast(*p, S.logf);
      }
    }
    wave_sync();
    if (lane < 2 * 4 * kPasses) {  // DCT row, 10*log10|c|, "%f" micro-units / NULL
      const int row = lane >> 1, cfi = lane & 1;
      const int64_t f = cur.f0 + row;
      if (f < nf) {
        float acc = 0.f;
        if constexpr (kPairFb) {
          const float* prow = reinterpret_cast<const float*>(M.scratch) + 2 * (2 * (row & 7) + (row >> 3)) * kFbNf + cfi;
#pragma unroll
          for (int i = 0; i < kFbNf; i++) acc = acc + prow[2 * i];
#pragma unroll
          for (int i = kFbNf; i < kFilters; i++) acc = acc + lempty * S.dct[cfi][i];
        } else {
          const float* lrow = M.logs + row * kLogStride;
#pragma unroll 8
          for (int i = 0; i < kFilters; i++) acc = acc + lrow[i] * S.dct[cfi][i];
        }
        const int64_t g = (single_ns >= 0 ? 0 : foff[cur.c]) + f;
        if constexpr (kSplitTail) {
          micro[2 * g + cfi] = __builtin_bit_cast(int32_t, acc);  // finish_db_kernel: dB + "%f" on full waves
        } else {
          const double q = db ? db_of_coef(acc, fx) : db_of_coef(acc);  // frame values glibc-exact
          micro[2 * g + cfi] = micro_of_db(q);
          if (db) db[2 * g + cfi] = q;
        }
      }
    }
    wave_sync();
    cur = nxt;
  }
#ifdef TFP_STAMPS
  const uint64_t t_end = __builtin_amdgcn_s_memtime();
  if (lane == 0 && (blockIdx.x & 63) == 0)
    printf("stamps<%d> block %d wave %d passes %d | entry->staged %lu staged->loop %lu loop %lu after-last-pass %lu | "
           "lead %lu stage %lu fft1 %lu fft2 %lu split %lu mel %lu\n",
           kPasses, (int)blockIdx.x, wave, npass, (unsigned long)(t_staged - t_entry), (unsigned long)(tstart - t_staged),
           (unsigned long)(tprev - tstart), (unsigned long)(t_end - tprev), (unsigned long)st[0], (unsigned long)st[1],
           (unsigned long)st[2], (unsigned long)st[3], (unsigned long)st[4], (unsigned long)st[5]);
#endif
}

// 10*log10|c| (fp_handler.c:651) and "%f" micro-units / NULL (db_ctx_handler.c:479-481) of every
// coefficient fingerprint8k_kernel stored (as float bits) in micro[], in place, on full waves: the
// kernel's tile tail would run this double-precision work on 32 of 64 lanes.
__global__ void finish_db_kernel(int32_t* __restrict__ micro, double* __restrict__ db, int64_t nvals, LogFix fx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvals; i += (int64_t)gridDim.x * blockDim.x) {
    const float c = __builtin_bit_cast(float, micro[i]);
    const double q = db ? db_of_coef(c, fx) : db_of_coef(c);  // frame values glibc-exact
    micro[i] = micro_of_db(q);
    if (db) db[i] = q;
  }
}

bool DspTables_fixed8k(const DspTables& t) {
  return t.ms_len[0] == 36 && t.ms_len[1] == 16 && t.ms_len[2] == 8 && t.ms_total == 16 * (36 + 16 + 8) &&
         t.ms_total <= kMsLds && t.ms_c_defer == 1 && t.ms_maxbin <= 2 * kFrameStride8 - 48 &&
         t.ms_filter[0][15] >= 0 && t.ms_filter[1][15] >= 0 && t.fb_ok == 1 && t.fb_nfilters == kFbNf &&
         t.tw256_im[32] == -t.tw256_re[32] && t.tw256_im[96] == t.tw256_re[96];  // dft16q's cmul_w2 / cmul_w6
}

// Resident 256-thread blocks per CU of kernel k: the occupancy query, capped by what the
// kernel's VGPRs and LDS admit on gfx950 (512 VGPRs per SIMD lane in granules of 8, one wave of
// a block per SIMD; 160 KiB of LDS per CU). The query alone over-counted once the LDS shrank
// below a third of the CU while the VGPRs still admitted two waves: a grid of 3 blocks per CU
// ran its last third as a tail (0.71 vs 0.54 ms per C2 launch).
static int resident_blocks(const void* k, int waves = kBlockWaves) {
  int per = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 64 * waves, 0);
  hipFuncAttributes a;
  if (hipFuncGetAttributes(&a, k) == hipSuccess) {
    const int vg = ((a.numRegs > 0 ? a.numRegs : 1) + 7) / 8 * 8;
    int by_vgpr = 512 / vg;  // waves per SIMD
    if (by_vgpr > 8) by_vgpr = 8;
    by_vgpr = by_vgpr * 4 / waves;  // workgroups per CU (a workgroup's waves spread over the 4 SIMDs)
    const int by_lds = a.sharedSizeBytes ? (int)((160 * 1024) / a.sharedSizeBytes) : 8;
    const int own = by_vgpr < by_lds ? by_vgpr : by_lds;
    if (per <= 0 || own < per) per = own;
  }
  return per > 0 ? per : 1;
}

hipError_t fp_launch_config(int device, FpLaunchCfg* cfg) {
  int cus = 0;
  hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) return e;
  auto cap = [&](const void* k, int waves = kBlockWaves) { return cus * resident_blocks(k, waves); };
  cfg->grid_cap_8k = cap(reinterpret_cast<const void*>(fingerprint8k_kernel<kTile8k / 4>), kBW8);
  cfg->grid_cap_8k_small = cap(reinterpret_cast<const void*>(fingerprint8k_kernel<1>));
  cfg->grid_cap_generic = cap(reinterpret_cast<const void*>(fingerprint_kernel<int16_t>));
  cfg->grid_cap_f32 = cap(reinterpret_cast<const void*>(fingerprint_kernel<float>));
  if (knob("TFP_DEBUG_OCC")) {
    int per = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(fingerprint8k_kernel<kTile8k / 4>),
                                                       64 * kBW8, 0);
    fprintf(stderr, "[tfp] fingerprint8k_kernel<%d>: %d blocks/CU (occupancy query %d), grid cap %d\n", kTile8k / 4,
            cfg->grid_cap_8k / cus, per, cfg->grid_cap_8k);
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(fingerprint8k_kernel<kTile8k / 4>)) == hipSuccess)
      fprintf(stderr, "[tfp]   %d threads/block (max %d), %d VGPRs, %zu B LDS, %zu B scratch\n", 64 * kBW8,
              fa.maxThreadsPerBlock, fa.numRegs, fa.sharedSizeBytes, fa.localSizeBytes);
    int smem = 0, smem_optin = 0;
    (void)hipDeviceGetAttribute(&smem, hipDeviceAttributeMaxSharedMemoryPerBlock, device);
    (void)hipDeviceGetAttribute(&smem_optin, hipDeviceAttributeSharedMemPerBlockOptin, device);
    fprintf(stderr, "[tfp]   device: %d B LDS per block (opt-in %d)\n", smem, smem_optin);
  }
  // TFP_FP_BLOCKS_PER_CU (experiments): fewer resident workgroups per CU for the 8 kHz throughput
  // kernel (1 = one wave per SIMD), to measure how its time scales with the waves per SIMD
  if (const char* b = knob("TFP_FP_BLOCKS_PER_CU")) {
    const int n = atoi(b);
    if (n > 0 && cus * n < cfg->grid_cap_8k) cfg->grid_cap_8k = cus * n;
  }
  const char* g = knob("TFP_GENERIC");
  cfg->force_generic = g && atoi(g);
  const char* rt = knob("TFP_RARE_THR_LOG2");
  int rl = rt ? atoi(rt) : -98;
  rl = rl < -98 ? -98 : (rl > 100 ? 100 : rl);  // any threshold >= 2^-98 gives the same, exact, result
  cfg->rare_thr = ldexpf(1.f, rl);
  return hipSuccess;
}

hipError_t launch_fingerprint(const FpLaunchCfg& cfg, const DspTables* d_tables, bool fixed8k, int32_t tile_frames,
                              const int16_t* d_pcm, const int64_t* d_sbeg, const int64_t* d_send, const int64_t* d_foff,
                              const int32_t* d_toff, const int32_t* d_tclip, int32_t ntiles, int64_t nframes,
                              int32_t* d_micro, double* d_db, hipStream_t s, const LogFix& fx, int64_t single_ns) {
  const bool v8 = fixed8k && (tile_frames == 4 || !cfg.force_generic);
  if (v8 ? !(tile_frames == 4 || tile_frames == kTile8k) : tile_frames != kFramesPerBlock) return hipErrorInvalidValue;
  if (ntiles <= 0) return hipSuccess;
  const int cap = v8 ? (tile_frames == 4 ? cfg.grid_cap_8k_small : cfg.grid_cap_8k) : cfg.grid_cap_generic;
  if (cap <= 0) return hipErrorInvalidValue;
  const int bw = (v8 && tile_frames != 4) ? kBW8 : kBlockWaves;
  const int want = (ntiles + bw - 1) / bw;  // one tile per wave per step
  const int grid = want < cap ? want : cap;
  if (v8) {
    if (tile_frames == 4) {  // fingerprint8k_kernel<1> finishes its own tail
      hipLaunchKernelGGL(fingerprint8k_kernel<1>, dim3(grid), dim3(kBlockThreads), 0, s, d_tables, d_pcm, d_sbeg, d_send,
                         d_foff, d_toff, d_tclip, ntiles, d_micro, d_db, cfg.rare_thr, fx, single_ns);
    } else {
      hipLaunchKernelGGL(fingerprint8k_kernel<kTile8k / 4>, dim3(grid), dim3(64 * kBW8), 0, s, d_tables, d_pcm, d_sbeg,
                         d_send, d_foff, d_toff, d_tclip, ntiles, d_micro, d_db, cfg.rare_thr, fx, single_ns);
      // (each HIP call overwrites the last error: a failed launch must be caught before the next one)
      if (const hipError_t le = hipGetLastError(); le != hipSuccess) return le;
      const int64_t nv = 2 * nframes;
      int64_t g = (nv + 255) / 256;
      if (g > 8192) g = 8192;
      if (nv > 0) hipLaunchKernelGGL(finish_db_kernel, dim3((unsigned)g), dim3(256), 0, s, d_micro, d_db, nv, fx);
    }
    return hipGetLastError();
  }
  hipLaunchKernelGGL(fingerprint_kernel<int16_t>, dim3(grid), dim3(kBlockThreads), 0, s, d_tables, d_pcm, d_sbeg, d_send,
                     d_foff, d_toff, d_tclip, ntiles, d_micro, d_db, fx);
  return hipGetLastError();
}

hipError_t launch_fingerprint_f32(const FpLaunchCfg& cfg, const DspTables* d_tables, const float* d_x,
                                  const int64_t* d_sbeg, const int64_t* d_send, const int64_t* d_foff,
                                  const int32_t* d_toff, const int32_t* d_tclip, int32_t ntiles, int32_t* d_micro,
                                  double* d_db, hipStream_t s, const LogFix& fx) {
  if (ntiles <= 0) return hipSuccess;
  if (cfg.grid_cap_f32 <= 0) return hipErrorInvalidValue;
  const int want = (ntiles + kBlockWaves - 1) / kBlockWaves;
  const int grid = want < cfg.grid_cap_f32 ? want : cfg.grid_cap_f32;
  hipLaunchKernelGGL(fingerprint_kernel<float>, dim3(grid), dim3(kBlockThreads), 0, s, d_tables, d_x, d_sbeg, d_send,
                     d_foff, d_toff, d_tclip, ntiles, d_micro, d_db, fx);
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
__global__ void prep_boxes_kernel(const double* __restrict__ q, int64_t n, SearchConsts sc, FrameBox* __restrict__ boxes,
                                  uint32_t* __restrict__ zero_words, int32_t nzero) {
  // the vote path's key mask, max count and per-query best keys start at 0 (read by later kernels)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nzero; i += (int64_t)gridDim.x * blockDim.x)
    zero_words[i] = 0u;
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

hipError_t launch_prep_boxes(const double* d_q, int64_t nframes, SearchConsts sc, FrameBox* boxes, uint32_t* zero_words,
                             int32_t nzero, hipStream_t s) {
  if (nframes <= 0 && nzero <= 0) return hipSuccess;
  int64_t g = ((nframes > nzero ? nframes : nzero) + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(prep_boxes_kernel, dim3((unsigned)g), dim3(256), 0, s, d_q, nframes, sc, boxes, zero_words, nzero);
  return hipGetLastError();
}

constexpr int kVoteColsPerBlock = 1024;  // clips per vote_gemm block (a power of 2)
constexpr int kClassKuMax = 10;  // pattern-class vote path: at most 2^10 - 1 patterns
constexpr float kVoteScale = 1024.f;      // Bt's box entries: acc = 1024 * score + column-in-chunk

// ---- coefs = 1: vote matrix. score[q][clip] = sum_k N[q][k] * B[k][clip], where N counts the
// query's non-ignored frames with trunc key k and B[k][clip] = 1 iff the clip has a row in
// [fmt6(k - tol), fmt6(k + tol)] — exactly the per-frame "group by audio_uuid" hit count.
// The trunc key of a query frame and whether its SQL runs (prep_boxes' flags & 1, restated for
// the vote path, which needs nothing else of the box).
__device__ __forceinline__ bool frame_key(const double* __restrict__ q, int64_t i, const SearchConsts& sc, int32_t& k) {
  const double q1 = q[2 * i];
  const double v1 = __builtin_isfinite(q1) ? q1 : 0.0;  // ast_json_real_get(NULL) = 0.0
  k = (v1 > -2147483649.0 && v1 < 2147483648.0) ? (int32_t)v1 : INT32_MIN;  // (int) truncation, :290
  const double freq = (double)k;
  if (sc.has_low && freq < sc.thr_low) return false;   // :293-306
  if (sc.has_high && freq > sc.thr_high) return false;
  return __builtin_isfinite(freq - sc.tole) && __builtin_isfinite(freq + sc.tole);
}

// The batch's used-key mask over all frames at once (every frame's key is independent of its
// query): bits set in a 32-word LDS mask per block, ORed into the global mask; a key outside the
// vote range is reported through maxc as INT32_MAX (the batch then goes to the scan path).
__global__ __launch_bounds__(256) void key_mask_kernel(const double* __restrict__ qv, SearchConsts sc, int64_t nf,
                                                       uint32_t* __restrict__ mask, int32_t* __restrict__ maxc,
                                                       VoteMeta* __restrict__ meta) {
  if (blockIdx.x == 0 && threadIdx.x == 0) meta->ok = 1;  // build_A only ever clears it
  // one byte per key, set by plain stores (keys concentrate on a few values, so LDS atomics on a
  // few mask words would serialise), then folded to mask words by ballots
  __shared__ uint8_t used[kKeyRange];
  for (int i = threadIdx.x; i < kKeyRange; i += blockDim.x) used[i] = 0;
  __syncthreads();
  bool out_of_range = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nf; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t k;
    if (!frame_key(qv, i, sc, k)) continue;
    const int64_t idx = (int64_t)k + kKeyOffset;
    if (idx < 0 || idx >= kKeyRange) {
      out_of_range = true;
      continue;
    }
    used[idx] = 1;
  }
  if (out_of_range) atomicMax(maxc, INT32_MAX);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  for (int base = threadIdx.x & ~63; base < kKeyRange; base += blockDim.x) {
    const unsigned long long bits = __ballot(used[base + lane] != 0);
    if (lane == 0) {
      if ((uint32_t)bits) atomicOr(&mask[base >> 5], (uint32_t)bits);
      if ((uint32_t)(bits >> 32)) atomicOr(&mask[(base >> 5) + 1], (uint32_t)(bits >> 32));
    }
  }
}

hipError_t launch_key_mask(const double* d_q, SearchConsts sc, int64_t nf, uint32_t* d_mask, int32_t* d_maxc,
                           VoteMeta* d_meta, hipStream_t s) {
  // few blocks: each ORs its words into the same few global mask words, and same-address atomics
  // serialise in L2 (4096 blocks cost ~50 us); at least one (it sets meta->ok)
  int64_t g = (nf + 255) / 256;
  if (g > 256) g = 256;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(key_mask_kernel, dim3((unsigned)g), dim3(256), 0, s, d_q, sc, nf, d_mask, d_maxc, d_meta);
  return hipGetLastError();
}

// Row range [lo, hi) in the m1-sorted index of every key's "%f" box at tolerance tole (all 1024
// keys: cached by the engine per index version and tolerance).
__global__ void key_ranges_all_kernel(const int32_t* __restrict__ m1s, int64_t R, double tole, int64_t* __restrict__ rng) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kKeyRange) return;
  const double freq = (double)(t - kKeyOffset);
  rng[2 * t] = lower_bound_i32(m1s, R, fmt6_bound(freq - tole));
  rng[2 * t + 1] = upper_bound_i32(m1s, R, fmt6_bound(freq + tole));
}

hipError_t launch_key_ranges_all(const int32_t* m1s, int64_t R, double tole, int64_t* d_rng_all, hipStream_t s) {
  hipLaunchKernelGGL(key_ranges_all_kernel, dim3(kKeyRange / 64), dim3(64), 0, s, m1s, R, tole, d_rng_all);
  return hipGetLastError();
}

// Used-key compaction on the GPU (no host round trip), in every build_A block: the batch's key mask
// -> column kc of each used key (ascending key order) by a prefix popcount of the 32 mask words;
// block 0 writes meta = (Ku, Kp = padded Ku + 1, cls). (A separate one-block compaction launch
// cost ~5 us per batch.)
//
// One wave per query row of A: the query's frames counted per used key in LDS, then the row
// written as fp16 (A[q][Ku] = 1 picks up Bt's column-position entry for vote_gemm's packed argmax;
// rows q >= nq up to Qp are zero). A count above 2048 (not exact in fp16) clears meta->ok, before
// vote_gemm reads it, and the host redoes the batch on the scan path.
__global__ __launch_bounds__(256) void build_A_kernel(const double* __restrict__ qv, SearchConsts sc,
                                                      const int64_t* __restrict__ qoff, int32_t nq, int32_t Qp,
                                                      const uint32_t* __restrict__ mask, const int32_t* __restrict__ maxc,
                                                      VoteMeta* __restrict__ meta, int32_t class_ku_max,
                                                      _Float16* __restrict__ A, _Float16* __restrict__ Bt, int32_t Cp) {
  __shared__ int32_t hist[4][kVoteKpMax];
  __shared__ uint32_t mw[kKeyRange / 32];
  __shared__ int32_t pre[kKeyRange / 32 + 1];  // used keys below mask word w; pre[32] = Ku
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // used-key compaction (ascending key = column), derived by every block from the 32 mask words
  if (threadIdx.x < 64) {
    const uint32_t m = threadIdx.x < kKeyRange / 32 ? mask[threadIdx.x] : 0u;
    const int c = __popc(m);
    int incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off, 64);
      if (lane >= off) incl += v;
    }
    if (threadIdx.x < kKeyRange / 32) {
      mw[threadIdx.x] = m;
      pre[threadIdx.x] = incl - c;
    }
    if (threadIdx.x == kKeyRange / 32 - 1) pre[kKeyRange / 32] = incl;
  }
  __syncthreads();
  const int32_t Ku = pre[kKeyRange / 32], Kp = ((Ku + 1 + 15) / 16) * 16;
  const int32_t cls = Ku <= class_ku_max && Ku <= kClassKuMax ? 1 : 0;
  // the region of Bt build_B marks, cleared over the whole grid (each block knows the path: a
  // separate clearing launch cost ~5 us per batch)
  {
    const int64_t n16 = cls ? (1 << kClassKuMax) / 4 : 0;  // 16-byte units: the pattern maxima
                                                             // (build_B writes all of the GEMM's Bt)
    uint4* p = reinterpret_cast<uint4*>(Bt);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
      p[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the vote's metadata
    meta->ku = Ku;
    meta->kp = Kp;
    meta->cls = cls;
    if (*maxc > 2048) meta->ok = 0;  // a key outside the vote range (key_mask)
  }
  const int q = blockIdx.x * 4 + wave;
  if (q >= Qp) return;
  int32_t* h = hist[wave];
  for (int c = lane; c < Kp; c += 64) h[c] = 0;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (q < nq) {
    for (int64_t i = qoff[q] + lane; i < qoff[q + 1]; i += 64) {
      int32_t k;
      if (!frame_key(qv, i, sc, k)) continue;
      const int64_t idx = (int64_t)k + kKeyOffset;
      if (idx < 0 || idx >= kKeyRange) continue;  // already flagged by key_mask (meta->ok = 0)
      const uint32_t m = mw[idx >> 5];
      atomicAdd(&h[pre[idx >> 5] + __popc(m & ((1u << (idx & 31)) - 1u))], 1);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  bool big = false;
  _Float16* row = A + (int64_t)q * Kp;
  for (int c = lane; c < Kp; c += 64) {
    int32_t v = q < nq ? h[c] : 0;
    if (q < nq && c == Ku) v = 1;
    big |= v > 2048;
    row[c] = (_Float16)(float)v;  // exact for v <= 2048
  }
  if (big) meta->ok = 0;
}

hipError_t launch_build_A(const double* d_q, SearchConsts sc, const int64_t* d_qoff, int32_t nq, int32_t Qp,
                          const uint32_t* d_mask, const int32_t* d_maxc,
                          VoteMeta* d_meta, int32_t class_ku_max, _Float16* d_A, _Float16* d_Bt, int32_t Cp,
                          hipStream_t s) {
  hipLaunchKernelGGL(build_A_kernel, dim3((unsigned)((Qp + 3) / 4)), dim3(256), 0, s, d_q, sc, d_qoff, nq, Qp, d_mask,
                     d_maxc, d_meta, class_ku_max, d_A, d_Bt, Cp);
  return hipGetLastError();
}

// Bt[clip][kc] = kVoteScale when the clip has a row in the kc-th used key's box, Bt[clip][Ku] =
// clip mod 1024 (the clip's position in its vote_gemm chunk), 0 elsewhere: build_B writes the
// [Cp][Kp] region the GEMM reads from the cached key bitsets.
//
// Few used keys (meta->cls: Ku <= kClassKuMax) take the pattern-class path instead, in the same
// buffer: a clip's score for query q is the sum of q's counts over the keys whose boxes hold a row
// of the clip, so it depends only on that key set (the clip's pattern, Ku bits). Per pattern only
// the greatest column matters (a tie goes to the greatest uuid), so the vote is an argmax over at
// most 2^Ku - 1 classes per query instead of over every clip. Layout: cls[2^kClassKuMax] int32
// (greatest column + 1 per pattern, 0 = none); a clip's pattern comes from the cached key-presence
// bitsets (launch_key_bits), one bit per used key.
// GEMM path: every row of Bt written whole from the cached key bitsets (one thread per clip,
// 16-byte stores), so nothing needs clearing first and the work does not grow with the boxes'
// rows. Against clearing plus marking the boxes' rows (scattered 2-byte stores): 42 -> 33 us at
// 81 used keys and 280 -> 199 us at 601 (scripts/vote_bench.py under rocprofv3, C3 size).
typedef _Float16 bt8 __attribute__((ext_vector_type(8)));
__global__ __launch_bounds__(256) void build_B_kernel(const uint32_t* __restrict__ mask, const uint32_t* __restrict__ bits,
                                                      int32_t C, const VoteMeta* __restrict__ meta, int32_t Cp,
                                                      _Float16* __restrict__ Bt) {
  if (meta->cls) return;  // the class path reads the cached key bitsets itself
  const int32_t Ku = meta->ku, Kp = meta->kp;
  __shared__ int16_t kk[kKeyRange];  // used keys, ascending (= columns kc)
  __shared__ int32_t pre[kKeyRange / 32];
  if (threadIdx.x < 64) {  // exclusive prefix of the mask words' popcounts
    const int lane = threadIdx.x;
    const int c = lane < kKeyRange / 32 ? __popc(mask[lane]) : 0;
    int incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off, 64);
      if (lane >= off) incl += v;
    }
    if (lane < kKeyRange / 32) pre[lane] = incl - c;
  }
  __syncthreads();
  if (threadIdx.x < kKeyRange / 32) {
    int kc = pre[threadIdx.x];
    for (uint32_t m = mask[threadIdx.x]; m; m &= m - 1u) kk[kc++] = (int16_t)(32 * threadIdx.x + __builtin_ctz(m));
  }
  __syncthreads();
  const int32_t W = key_bits_words(C);
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < Cp; c += (int64_t)gridDim.x * blockDim.x) {
    bt8* row = reinterpret_cast<bt8*>(Bt + c * Kp);
    const uint32_t* col = bits + (c >> 5);
    const int sh = (int)(c & 31);
    for (int k0 = 0; k0 < Kp; k0 += 8) {
      bt8 v;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const int kc = k0 + j;
        float x = 0.f;
        if (kc < Ku) x = ((col[(int64_t)kk[kc] * W] >> sh) & 1u) ? kVoteScale : 0.f;
        else if (kc == Ku) x = (float)(c & (kVoteColsPerBlock - 1));
        v[j] = (_Float16)x;
      }
      row[k0 / 8] = v;
    }
  }
}

// Pattern-class path: every clip's pattern from its flags, the greatest tie key per pattern (the
// columns need not be in uuid order: an index delta's clips sit in columns after the main index's)
// reduced in LDS per block first (many clips share a pattern; same-address global atomics
// serialise, so only the first kClassMaxBlocks blocks take part), then merged with one global
// atomicMax per pattern present in the block. Run by vote_gemm_regs_kernel's blocks when
// meta->cls (its GEMM is not needed then): a launch of its own cost ~4.5 us per batch.
constexpr int kClassMaxBlocks = 64;
__device__ void class_max_block(int blk, int nblk, int32_t Ku, const uint32_t* __restrict__ mask,
                                const uint32_t* __restrict__ bits, int32_t C, const int32_t* __restrict__ tiekey,
                                _Float16* __restrict__ Bt, int32_t* best, int32_t* kk) {
  for (int i = threadIdx.x; i < (1 << kClassKuMax); i += blockDim.x) best[i] = 0;
  if (threadIdx.x == 0) {  // the used keys, ascending (= columns kc)
    int n = 0;
    for (int w = 0; w < kKeyRange / 32 && n < Ku; w++)
      for (uint32_t m = mask[w]; m && n < Ku; m &= m - 1u) kk[n++] = 32 * w + __builtin_ctz(m);
  }
  __syncthreads();
  int32_t* cls = reinterpret_cast<int32_t*>(Bt);
  const int32_t W = key_bits_words(C);
  for (int64_t c = (int64_t)blk * blockDim.x + threadIdx.x; c < C; c += (int64_t)nblk * blockDim.x) {
    uint32_t pat = 0;
    for (int k = 0; k < Ku; k++) pat |= ((bits[(int64_t)kk[k] * W + (c >> 5)] >> (c & 31)) & 1u) << k;
    if (pat) atomicMax(&best[pat], tiekey[c] + 1);  // the pattern's greatest tie key (uuid order), + 1
  }
  __syncthreads();
  for (int i = threadIdx.x; i < (1 << kClassKuMax); i += blockDim.x)
    if (best[i]) atomicMax(&cls[i], best[i]);
}

hipError_t launch_build_B(const uint32_t* d_mask, const uint32_t* d_bits, int32_t C, const VoteMeta* d_meta, int32_t Cp,
                          _Float16* d_Bt, hipStream_t s) {
  hipLaunchKernelGGL(build_B_kernel, dim3(1024), dim3(256), 0, s, d_mask, d_bits, C, d_meta, Cp, d_Bt);
  return hipGetLastError();
}

// Pattern-class path: one wave per query, lanes over the patterns present; score = the query's
// counts (A, exact in fp16) summed over the pattern's keys; key = score << 32 | the pattern's
// greatest tie key, max over patterns with a non-zero score.
// The vote's last step, one wave per query: the pattern-class vote (meta->cls), or for the GEMM
// path the max of the query's per-chunk keys (one launch for both: the path is known only on the
// device).
__global__ __launch_bounds__(256) void class_vote_kernel(const _Float16* __restrict__ A, int32_t Qp,
                                                         const VoteMeta* __restrict__ meta,
                                                         const _Float16* __restrict__ Bt,
                                                         const int32_t* __restrict__ tiekey,
                                                         const unsigned long long* __restrict__ part, int32_t nchunks,
                                                         unsigned long long* __restrict__ best) {
  const int32_t Ku = meta->ku, Kp = meta->kp;
  if (!meta->ok) return;
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= Qp) return;
  if (!meta->cls) {  // GEMM path: max over the chunks' partial keys (score << 32 | tiekey)
    unsigned long long b = 0;
    for (int c = lane; c < nchunks; c += 64) {
      const unsigned long long v = part[(int64_t)c * Qp + q];
      b = v > b ? v : b;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const unsigned long long o = __shfl_xor(b, off, 64);
      b = o > b ? o : b;
    }
    if (lane == 0) best[q] = b;
    return;
  }
  const int32_t* cls = reinterpret_cast<const int32_t*>(Bt);
  int32_t cnt[kClassKuMax];
#pragma unroll
  for (int k = 0; k < kClassKuMax; k++) cnt[k] = k < Ku ? (int32_t)(float)A[(int64_t)q * Kp + k] : 0;
  unsigned long long mine = 0;
  for (int P = lane + 1; P < (1 << Ku); P += 64) {
    const int32_t c1 = cls[P];
    if (!c1) continue;
    uint32_t score = 0;
#pragma unroll
    for (int k = 0; k < kClassKuMax; k++) score += (P >> k) & 1 ? (uint32_t)cnt[k] : 0u;
    if (!score) continue;
    const unsigned long long key = ((unsigned long long)score << 32) | (unsigned)(c1 - 1);  // (c1 = tie key + 1)
    mine = key > mine ? key : mine;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const unsigned long long o = __shfl_xor(mine, off, 64);
    mine = o > mine ? o : mine;
  }
  if (lane == 0 && mine) atomicMax(&best[q], mine);
}

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// Packed argmax: the K dimension carries one extra column, A = 1 against Bt = the clip's position
// in its 1024-clip chunk, and the box entries are 1024, so each accumulator is exactly
// 1024 * score + position (< 2^24 for scores < 16384 frames, exact in fp32): one v_max per score
// keeps the best (score, latest column) — columns are the clips in ascending uuid order, so a
// later column wins a tie, as SQLite returns the greatest audio_uuid. Result key =
// score << 32 | tiekey[column], merged across chunks with atomicMax.
#ifndef TFP_VOTE_CHUNK
#define TFP_VOTE_CHUNK 1024
#endif
constexpr int kVoteChunk = TFP_VOTE_CHUNK;  // clips per block (a divisor of kVoteColsPerBlock)

// m holds the bit patterns of the running maxima. Every accumulator is a non-negative float
// (non-negative operands), and non-negative floats order as their bit patterns, so the max is an
// integer v_max_u32 (fmaxf would canonicalise both operands first: 3 VALU per element).
typedef uint32_t uintx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void vote_max_into(uintx16& m, const floatx16& acc) {
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = max(m[i], __float_as_uint(acc[i]));
}

// The wave's 32 rows of its chunk's partial results (part = this chunk's row of [nchunks][Qp]):
// plain stores, merged by class_vote_kernel (GEMM branch). Device-scope atomics on shared addresses go past the
// per-XCD L2s and serialise: 400 k of them cost ~50 us.
__device__ __forceinline__ void vote_reduce_rows(const uintx16& m, int q0, int h, int r, int base,
                                                 const int32_t* __restrict__ tiekey,
                                                 unsigned long long* __restrict__ part) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint32_t v = m[i];
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
    const uint32_t packed = (uint32_t)__uint_as_float(v);
    const uint32_t score = packed / (uint32_t)kVoteScale;
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    if (r == 0) {
      const int col = base + (int)(packed % (uint32_t)kVoteScale);
      part[q0 + row] = score > 0 ? ((unsigned long long)score << 32) | (unsigned)tiekey[col] : 0ull;
    }
  }
}

// Kp = 16 * KS <= 128: the wave's two 32-query A tiles stay in registers for the whole chunk and
// each B fragment (32 clips x 16 keys) feeds two MFMAs. B is loaded G 32-clip steps at a time,
// double-buffered: the next group's loads are in flight while the current group is multiplied
// (with few keys a step is only a few MFMAs, so one step of prefetch cannot cover the latency).
template <int KS, int G>
__device__ __forceinline__ void vote_tile_regs(const _Float16* __restrict__ A, const _Float16* __restrict__ Bt, int q0,
                                               int cbeg, int cend, const int32_t* __restrict__ tiekey,
                                               unsigned long long* __restrict__ best) {
  constexpr int Kp = 16 * KS;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const uint32_t voff = (uint32_t)((r * Kp + 8 * h) * sizeof(_Float16));  // lane's byte offset in a step
  half8 a0[KS], a1[KS], b[G][KS];
#pragma unroll
  for (int s = 0; s < KS; s++) {
    a0[s] = *reinterpret_cast<const half8*>(A + (int64_t)(q0 + r) * Kp + 16 * s + 8 * h);
    a1[s] = *reinterpret_cast<const half8*>(A + (int64_t)(q0 + 32 + r) * Kp + 16 * s + 8 * h);
  }
  auto load_group = [&](int c, half8 (&dst)[G][KS]) {
#pragma unroll
    for (int g = 0; g < G; g++) {
      const int cc = min(c + 32 * g, cend - 32);  // past the chunk: a duplicate, not used
      const char* sb = reinterpret_cast<const char*>(Bt + (int64_t)cc * Kp);  // wave-uniform base
#pragma unroll
      for (int s = 0; s < KS; s++) dst[g][s] = *reinterpret_cast<const half8*>(sb + voff + 32 * s);
    }
  };
  load_group(cbeg, b);
  uintx16 m0, m1;
#pragma unroll
  for (int i = 0; i < 16; i++) m0[i] = m1[i] = 0u;
  for (int c = cbeg; c < cend; c += 32 * G) {
    half8 bn[G][KS];
    load_group(c + 32 * G < cend ? c + 32 * G : c, bn);
#pragma unroll
    for (int g = 0; g < G; g++) {
      if (G > 1 && c + 32 * g >= cend) break;
      floatx16 acc0, acc1;
#pragma unroll
      for (int i = 0; i < 16; i++) acc0[i] = acc1[i] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; s++) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[s], b[g][s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[s], b[g][s], acc1, 0, 0, 0);
      }
      vote_max_into(m0, acc0);
      vote_max_into(m1, acc1);
    }
#pragma unroll
    for (int g = 0; g < G; g++)
#pragma unroll
      for (int s = 0; s < KS; s++) b[g][s] = bn[g][s];
  }
  const int base = cbeg & ~(kVoteColsPerBlock - 1);
  vote_reduce_rows(m0, q0, h, r, base, tiekey, best);
  vote_reduce_rows(m1, q0 + 32, h, r, base, tiekey, best);
}

// Kp = 16 * KS in (32, 128]: B shared by the block's 4 waves through LDS. Each B fragment feeds
// two MFMAs per wave, so per-wave loads of B (6 KB per 32 clips at Kp = 96) ran the kernel at the
// L1 bandwidth with waves parked on s_waitcnt 72 % of their cycles; staged once per block, B
// costs a quarter of that. Groups of 4 steps (128 clips) are loaded into registers while the
// previous group is multiplied from the other LDS buffer; rows are padded by 16 B (an odd number
// of 16-byte units) so the 8 lanes of each ds_read_b128 phase hit distinct bank groups. All four
// waves take part in the loads and barriers; a wave whose rows are past Qp only skips the math.
constexpr int kVoteGroupClips = 128;
constexpr int kVoteLdsRow = 2 * 128 + 16;  // bytes per clip row at the largest Kp of this path

template <int KS>
__device__ __forceinline__ void vote_tile_lds(const _Float16* __restrict__ A, const _Float16* __restrict__ Bt,
                                              int q0, bool rows_valid, int cbeg, int cend,
                                              const int32_t* __restrict__ tiekey, unsigned long long* __restrict__ part,
                                              char* __restrict__ lds /*[2][kVoteGroupClips * kVoteLdsRow]*/) {
  constexpr int Kp = 16 * KS;
  constexpr int kRow = 2 * Kp + 16;                      // padded LDS row (bytes)
  constexpr int kBuf = kVoteGroupClips * kRow;
  constexpr int kChunksPerClip = 2 * KS;                 // 16-byte units per clip row
  constexpr int kLoads = kVoteGroupClips * kChunksPerClip / 256;  // per thread (= KS)
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, h = lane >> 5;
  half8 a0[KS], a1[KS];
  if (rows_valid) {
#pragma unroll
    for (int s = 0; s < KS; s++) {
      a0[s] = *reinterpret_cast<const half8*>(A + (int64_t)(q0 + r) * Kp + 16 * s + 8 * h);
      a1[s] = *reinterpret_cast<const half8*>(A + (int64_t)(q0 + 32 + r) * Kp + 16 * s + 8 * h);
    }
  }
  int4 pre[kLoads];
  auto load_regs = [&](int g0) {
#pragma unroll
    for (int i = 0; i < kLoads; i++) {
      const int id = t + 256 * i, clip = id / kChunksPerClip, j = id % kChunksPerClip;
      pre[i] = g0 + clip < cend ? *reinterpret_cast<const int4*>(Bt + (int64_t)(g0 + clip) * Kp + 8 * j)
                                : make_int4(0, 0, 0, 0);
    }
  };
  auto store_lds = [&](int buf) {
#pragma unroll
    for (int i = 0; i < kLoads; i++) {
      const int id = t + 256 * i, clip = id / kChunksPerClip, j = id % kChunksPerClip;
      *reinterpret_cast<int4*>(lds + buf * kBuf + clip * kRow + 16 * j) = pre[i];
    }
  };
  uintx16 m0, m1;
#pragma unroll
  for (int i = 0; i < 16; i++) m0[i] = m1[i] = 0u;
  const int ngroups = (cend - cbeg + kVoteGroupClips - 1) / kVoteGroupClips;
  load_regs(cbeg);
  store_lds(0);
  __syncthreads();
  for (int g = 0; g < ngroups; g++) {
    const int g0 = cbeg + g * kVoteGroupClips;
    if (g + 1 < ngroups) load_regs(g0 + kVoteGroupClips);
    if (rows_valid) {
      const char* buf = lds + (g & 1) * kBuf + r * kRow + 16 * h;
#pragma unroll
      for (int st = 0; st < kVoteGroupClips / 32; st++) {
        if (g0 + 32 * st >= cend) break;
        floatx16 acc0, acc1;
#pragma unroll
        for (int i = 0; i < 16; i++) acc0[i] = acc1[i] = 0.f;
#pragma unroll
        for (int s = 0; s < KS; s++) {
          const half8 b = *reinterpret_cast<const half8*>(buf + st * 32 * kRow + 32 * s);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[s], b, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[s], b, acc1, 0, 0, 0);
        }
        vote_max_into(m0, acc0);
        vote_max_into(m1, acc1);
      }
    }
    if (g + 1 < ngroups) store_lds((g + 1) & 1);
    __syncthreads();
  }
  if (rows_valid) {
    const int base = cbeg & ~(kVoteColsPerBlock - 1);
    vote_reduce_rows(m0, q0, h, r, base, tiekey, part);
    vote_reduce_rows(m1, q0 + 32, h, r, base, tiekey, part);
  }
}

// Any Kp (up to kVoteKpMax): A and B fragments streamed from memory per 16-key step.
__device__ __forceinline__ void vote_tile_stream(const _Float16* __restrict__ A, const _Float16* __restrict__ Bt,
                                                 int32_t Kp, int q0, int cbeg, int cend,
                                                 const int32_t* __restrict__ tiekey,
                                                 unsigned long long* __restrict__ best) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  uintx16 m;
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = 0u;
  const _Float16* arow = A + (int64_t)(q0 + r) * Kp + 8 * h;
  constexpr int kSub = 4;  // 32-clip sub-tiles per step: their B fragments are loaded together
  for (int c0 = cbeg; c0 < cend; c0 += 32 * kSub) {
    floatx16 acc[kSub];
#pragma unroll
    for (int j = 0; j < kSub; j++)
#pragma unroll
      for (int i = 0; i < 16; i++) acc[j][i] = 0.f;
    for (int kb = 0; kb < Kp; kb += 16) {
      const half8 a = *reinterpret_cast<const half8*>(arow + kb);
      half8 bv[kSub];
#pragma unroll
      for (int j = 0; j < kSub; j++) {
        const int c = min(c0 + 32 * j, cend - 32);  // (a clamped duplicate sub-tile is not used below)
        bv[j] = *reinterpret_cast<const half8*>(Bt + (int64_t)(c + r) * Kp + 8 * h + kb);
      }
#pragma unroll
      for (int j = 0; j < kSub; j++) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bv[j], acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kSub; j++)
      if (c0 + 32 * j < cend) vote_max_into(m, acc[j]);
  }
  vote_reduce_rows(m, q0, h, r, cbeg & ~(kVoteColsPerBlock - 1), tiekey, best);
}

// Block = 4 waves x 64 queries against one kVoteChunk-clip chunk (Qp is a multiple of 128, Cp of
// 32, so every wave's 64 rows and every 32-clip step are in range). Two kernels, both launched,
// each returning at once unless Kp is its own (the host does not wait for Kp): Kp <= 32 (A and B
// in registers, more waves per SIMD) and Kp > 128 (fragments streamed) in the kernel without
// LDS, 32 < Kp <= 128 in the LDS-staged one.
__global__ __launch_bounds__(256) void vote_gemm_regs_kernel(const _Float16* __restrict__ A,
                                                              _Float16* __restrict__ Bt, int32_t Qp, int32_t Cp,
                                                              const VoteMeta* __restrict__ meta,
                                                              const int32_t* __restrict__ tiekey,
                                                              unsigned long long* __restrict__ part,
                                                              const uint32_t* __restrict__ mask,
                                                              const uint32_t* __restrict__ bits, int32_t C) {
  const int32_t Kp = meta->kp;
  if (meta->cls) {  // the pattern-class path's per-pattern maxima instead of a GEMM
    __shared__ int32_t cbest[1 << kClassKuMax];
    __shared__ int32_t ckk[kClassKuMax];
    const int blk = blockIdx.y * gridDim.x + blockIdx.x;
    const int nblk = min((int)(gridDim.x * gridDim.y), min(kClassMaxBlocks, (C + 255) / 256));
    if (blk < nblk) class_max_block(blk, nblk, meta->ku, mask, bits, C, tiekey, Bt, cbest, ckk);
    return;
  }
  if (!meta->ok || (Kp > 32 && Kp <= 128)) return;
  const int q0 = (blockIdx.y * 4 + (threadIdx.x >> 6)) * 64;
  if (q0 >= Qp) return;
  unsigned long long* __restrict__ best = part + (int64_t)blockIdx.x * Qp;
  const int cbeg = blockIdx.x * kVoteChunk;
  const int cend = min(cbeg + kVoteChunk, Cp);
  if (Kp == 16) {
    vote_tile_regs<1, 4>(A, Bt, q0, cbeg, cend, tiekey, best);
  } else if (Kp == 32) {
    vote_tile_regs<2, 4>(A, Bt, q0, cbeg, cend, tiekey, best);
  } else {
    vote_tile_stream(A, Bt, Kp, q0, cbeg, cend, tiekey, best);
    vote_tile_stream(A, Bt, Kp, q0 + 32, cbeg, cend, tiekey, best);
  }
}

__global__ __launch_bounds__(256) void vote_gemm_lds_kernel(const _Float16* __restrict__ A, const _Float16* __restrict__ Bt,
                                                        int32_t Qp, int32_t Cp, const VoteMeta* __restrict__ meta,
                                                        const int32_t* __restrict__ tiekey,
                                                        unsigned long long* __restrict__ part) {
  if (!meta->ok || meta->cls || meta->kp <= 32 || meta->kp > 128) return;  // redo / class / regs kernel
  __shared__ __attribute__((aligned(16))) char lds[2 * kVoteGroupClips * kVoteLdsRow];
  const int32_t Kp = meta->kp;
  const int wave = threadIdx.x >> 6;
  const int q0 = (blockIdx.y * 4 + wave) * 64;
  const bool rows_valid = q0 < Qp;
  unsigned long long* __restrict__ best = part + (int64_t)blockIdx.x * Qp;
  const int cbeg = blockIdx.x * kVoteChunk;
  const int cend = min(cbeg + kVoteChunk, Cp);
  switch (Kp >> 4) {  // uniform over the block: every wave reaches the same barriers
    case 3: vote_tile_lds<3>(A, Bt, q0, rows_valid, cbeg, cend, tiekey, best, lds); break;
    case 4: vote_tile_lds<4>(A, Bt, q0, rows_valid, cbeg, cend, tiekey, best, lds); break;
    case 5: vote_tile_lds<5>(A, Bt, q0, rows_valid, cbeg, cend, tiekey, best, lds); break;
    case 6: vote_tile_lds<6>(A, Bt, q0, rows_valid, cbeg, cend, tiekey, best, lds); break;
    case 7: vote_tile_lds<7>(A, Bt, q0, rows_valid, cbeg, cend, tiekey, best, lds); break;
    case 8: vote_tile_lds<8>(A, Bt, q0, rows_valid, cbeg, cend, tiekey, best, lds); break;
  }
}

// best[q] = max over the chunks' partial keys: 64 queries per block, 16 threads per query over
// the chunks (one thread per query left the loads latency-bound: 24 us for 98 chunks).
int32_t vote_chunks(int32_t Cp) { return (Cp + kVoteChunk - 1) / kVoteChunk; }

hipError_t launch_vote_gemm(const _Float16* d_A, _Float16* d_Bt, int32_t Qp, int32_t Cp, const VoteMeta* d_meta,
                            const int32_t* d_tiekey, unsigned long long* d_part, unsigned long long* d_best,
                            const uint32_t* d_mask, const uint32_t* d_bits, int32_t C, hipStream_t s) {
  if (Qp <= 0 || Cp <= 0) return hipSuccess;
  if (Qp % 128 || Cp % 32) return hipErrorInvalidValue;  // the tiles assume these paddings
  const int32_t nchunks = vote_chunks(Cp);
  dim3 grid(nchunks, (Qp / 64 + 3) / 4);
  hipLaunchKernelGGL(vote_gemm_regs_kernel, grid, dim3(256), 0, s, d_A, d_Bt, Qp, Cp, d_meta, d_tiekey, d_part, d_mask,
                     d_bits, C);
  hipLaunchKernelGGL(vote_gemm_lds_kernel, grid, dim3(256), 0, s, d_A, d_Bt, Qp, Cp, d_meta, d_tiekey, d_part);
  hipLaunchKernelGGL(class_vote_kernel, dim3((unsigned)(Qp / 4)), dim3(256), 0, s, d_A, Qp, d_meta, d_Bt, d_tiekey, d_part,
                     nchunks, d_best);
  return hipGetLastError();
}

// ---- small-batch path (see tfp_kernels.hpp). Same sets and counts as key_hist + build_A/B +
// vote_gemm: a query frame with trunc key k votes once for every clip with a row in k's box.
// The batch's used keys (ascending key order = column order kc), derived by each block from the
// query frames with frame_key's filter; bad = a key outside the vote range.
struct SmallKeySet {
  uint8_t used[kKeyRange];
  uint32_t mask[kKeyRange / 32];
  int32_t pre[kKeyRange / 32];  // used keys below mask word w
  int32_t ku, bad;
};
__device__ void small_keys(const double* __restrict__ q, int64_t nf, const SearchConsts& sc, SmallKeySet& K) {
  const int t = threadIdx.x;
  for (int i = t; i < kKeyRange; i += blockDim.x) K.used[i] = 0;
  if (t == 0) K.bad = 0;
  __syncthreads();
  for (int64_t i = t; i < nf; i += blockDim.x) {
    int32_t k;
    if (!frame_key(q, i, sc, k)) continue;
    const int64_t idx = (int64_t)k + kKeyOffset;
    if (idx < 0 || idx >= kKeyRange) K.bad = 1;
    else K.used[idx] = 1;  // plain byte stores: keys concentrate on a few values
  }
  __syncthreads();
  const int lane = t & 63;
  for (int base = t & ~63; base < kKeyRange; base += blockDim.x) {
    const unsigned long long bits = __ballot(K.used[base + lane] != 0);
    if (lane == 0) {
      K.mask[base >> 5] = (uint32_t)bits;
      K.mask[(base >> 5) + 1] = (uint32_t)(bits >> 32);
    }
  }
  __syncthreads();
  if (t < 32) {  // exclusive prefix of the words' popcounts
    const int c = __popc(K.mask[t]);
    int incl = c;
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) {
      const int v = __shfl_up(incl, off, 32);
      if (t >= off) incl += v;
    }
    K.pre[t] = incl - c;
    if (t == 31) K.ku = incl;
  }
  __syncthreads();
}
__device__ __forceinline__ int small_kc(const SmallKeySet& K, int key) {
  const int w = key >> 5;
  return K.pre[w] + __popc(K.mask[w] & ((1u << (key & 31)) - 1u));
}

// Key-presence bitsets without a global atomic per box row (round 5; the round-2 kernel's
// atomicOr per row serialised in L2 on the few dense keys: 42-50 ms at tolerance 0.45 on 100k
// clips, where one key's box holds ~84 M rows). A key's box rows are a contiguous range of the
// m1-sorted index, so the grid walks the concatenation of all keys' ranges in chunks of kKbChunk
// rows (every block scans the 1,024 range sizes into an LDS prefix first). Per piece of a key in its
// chunk, the block sets the piece's bits in an LDS copy of the key's row (one LDS OR per row) and
// then ORs its nonzero words into the row in memory (one atomic per word: the key's other chunks
// share the row). Pieces under `direct` rows (small boxes) set their bits with global atomics
// directly. A row wider than the LDS window (win words) is done window by window.
constexpr int kKbChunk = 1 << 16;
constexpr int kKbThreads = 256;
__global__ __launch_bounds__(kKbThreads) void key_bits_kernel(const int64_t* __restrict__ rng_all, const int32_t* __restrict__ cols,
                                                              int32_t W, int32_t win, int64_t direct, uint32_t* __restrict__ bits) {
  extern __shared__ uint32_t lrow[];  // win words
  __shared__ int64_t pre[kKeyRange + 1];
  __shared__ int64_t part[kKbThreads];
  const int t = threadIdx.x;
  constexpr int kPer = kKeyRange / kKbThreads;
  int64_t sz[kPer], sum = 0;
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const int k = t * kPer + j;
    sz[j] = max((int64_t)0, rng_all[2 * k + 1] - rng_all[2 * k]);
    sum += sz[j];
  }
  part[t] = sum;
  __syncthreads();
  for (int o = 1; o < kKbThreads; o <<= 1) {  // inclusive scan of the per-thread sums
    const int64_t y = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += y;
    __syncthreads();
  }
  int64_t run = part[t] - sum;
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    pre[t * kPer + j] = run;
    run += sz[j];
  }
  if (t == kKbThreads - 1) pre[kKeyRange] = part[t];
  __syncthreads();
  const int64_t total = pre[kKeyRange];
  for (int64_t v0 = (int64_t)blockIdx.x * kKbChunk; v0 < total; v0 += (int64_t)gridDim.x * kKbChunk) {
    const int64_t v1 = min(total, v0 + kKbChunk);
    int k = 0, hi = kKeyRange;  // the key whose range holds v0: the last k with pre[k] <= v0
    while (hi - k > 1) {
      const int mid = (k + hi) >> 1;
      if (pre[mid] <= v0) k = mid; else hi = mid;
    }
    for (; k < kKeyRange && pre[k] < v1; k++) {
      const int64_t a = max(v0, pre[k]), b = min(v1, pre[k + 1]);
      if (a >= b) continue;
      const int32_t* c = cols + rng_all[2 * k] + (a - pre[k]);
      const int64_t n = b - a;
      uint32_t* row = bits + (int64_t)k * W;
      if (n < direct) {  // (block-uniform)
        for (int64_t i = t; i < n; i += kKbThreads) atomicOr(&row[c[i] >> 5], 1u << (c[i] & 31));
        continue;
      }
      for (int32_t w0 = 0; w0 < W; w0 += win) {
        const int32_t wn = min(win, W - w0);
        const int32_t c0 = 32 * w0, c1 = 32 * (w0 + wn);
        for (int32_t j = t; j < wn; j += kKbThreads) lrow[j] = 0u;
        __syncthreads();
        for (int64_t i = t; i < n; i += kKbThreads) {
          const int32_t x = c[i];
          if (x >= c0 && x < c1) atomicOr(&lrow[(x - c0) >> 5], 1u << (x & 31));
        }
        __syncthreads();
        for (int32_t j = t; j < wn; j += kKbThreads)
          if (lrow[j]) atomicOr(&row[w0 + j], lrow[j]);
        __syncthreads();
      }
    }
  }
}

hipError_t launch_key_bits(const int64_t* d_rng_all, const int32_t* cols, int32_t C, int64_t rows_bound, int32_t win,
                           int64_t direct, uint32_t* d_bits, hipStream_t s) {
  const int32_t W = key_bits_words(C);
  hipError_t e = hipMemsetAsync(d_bits, 0, sizeof(uint32_t) * (size_t)kKeyRange * W, s);
  if (e) return e;
  // LDS window: the whole row up to 16 K words (64 KB: 524,288 columns), else windows of it
  win = win > 0 ? std::min(win, W) : std::min<int32_t>(W, 16384);
  win = std::max(win, 1);
  if (direct < 0) direct = std::max<int64_t>(2048, W / 2);  // a piece below a few row-clears of work
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(4096, (rows_bound + kKbChunk - 1) / kKbChunk));
  hipLaunchKernelGGL(key_bits_kernel, dim3(grid), dim3(kKbThreads), sizeof(uint32_t) * (size_t)win, s, d_rng_all, cols, W,
                     win, direct, d_bits);
  return hipGetLastError();
}

// Every block: the batch's used keys and per-(query, used key) frame counts from the query frames
// (per 64 frames of a wave: one ballot per distinct (query, key) among them and one LDS add per
// ballot, since keys concentrate on a few values), then clip-parallel scores of every query (4
// clips per thread: one bitset word per used key) and the per-query max of score << 32 | tie key
// (a later uuid wins a tie, as SQLite's ORDER BY count(*) DESC returns it), reduced per block and
// written to the caller's host-mapped result as this block's part; block 0 also writes (ku, bad).
// (The clips used to be stamped per call by a separate marking launch over the used keys' boxes;
// publishing the final max from the device cost a one-wave kernel of ~4 us per call, or a done
// counter and fences in every block.)
__global__ __launch_bounds__(256) void small_vote_kernel(const double* __restrict__ q, SmallQueries sq, SearchConsts sc,
                                                         const uint32_t* __restrict__ bits, int32_t C,
                                                         const int32_t* __restrict__ tiekey,
                                                         SmallResult* __restrict__ out) {
  static_assert(4 * 256 == kSmallVoteClips, "4 clips per thread");
  __shared__ SmallKeySet K;
  __shared__ int32_t A[kSmallQ][kKeyRange];
  __shared__ int16_t kkey[kKeyRange];  // kc -> key index (row of bits)
  __shared__ unsigned long long bmax[kSmallQ][4];
  const int nq = sq.nq;
  const int64_t nf = sq.qoff[nq];
  small_keys(q, nf, sc, K);
  const int ku = K.ku, bad = K.bad;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (!bad && ku > 0) {  // else every frame was ignored (NOTFOUND: best stays 0) or the caller redoes it
    for (int i = threadIdx.x; i < nq * ku; i += blockDim.x) A[i / ku][i % ku] = 0;
    if (threadIdx.x < kKeyRange / 32) {  // used keys in ascending order
      int kc = K.pre[threadIdx.x];
      for (uint32_t m = K.mask[threadIdx.x]; m; m &= m - 1u) kkey[kc++] = (int16_t)(32 * threadIdx.x + __builtin_ctz(m));
    }
    __syncthreads();
    for (int64_t base = threadIdx.x & ~63; base < nf; base += blockDim.x) {
      const int64_t i = base + lane;
      int32_t k = 0;
      int slot = -1;  // qi * kKeyRange + kc of this frame, -1 if ignored
      if (i < nf && frame_key(q, i, sc, k)) {
        int qi = 0;
        while (qi + 1 < nq && sq.qoff[qi + 1] <= i) qi++;
        slot = qi * kKeyRange + small_kc(K, k + kKeyOffset);
      }
      unsigned long long todo = __ballot(slot >= 0);
      while (todo) {
        const int lead = __builtin_ctzll(todo);
        const int ls = __shfl(slot, lead, 64);
        const unsigned long long same = __ballot(slot == ls);
        if (lane == lead) atomicAdd(&A[0][0] + ls, (int)__popcll(same));
        todo &= ~same;
      }
    }
    __syncthreads();
    const int c4 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);  // first of this thread's 4 clips
    const int W = key_bits_words(C);
    int32_t sc4[kSmallQ][4];
#pragma unroll
    for (int qi = 0; qi < kSmallQ; qi++)
#pragma unroll
      for (int j = 0; j < 4; j++) sc4[qi][j] = 0;
    if (c4 < C) {
      const uint32_t* col = bits + (c4 >> 5);
      const int sh = c4 & 31;
      int kc = 0;
      for (; kc + 4 <= ku; kc += 4) {  // 4 independent bitset loads in flight
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = col[(int64_t)kkey[kc + u] * W] >> sh;
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
          for (int j = 0; j < 4; j++)
            if ((v[u] >> j) & 1u)
#pragma unroll
              for (int qi = 0; qi < kSmallQ; qi++) sc4[qi][j] += qi < nq ? A[qi][kc + u] : 0;
      }
      for (; kc < ku; kc++) {
        const uint32_t x = col[(int64_t)kkey[kc] * W] >> sh;
#pragma unroll
        for (int j = 0; j < 4; j++)
          if ((x >> j) & 1u)
#pragma unroll
            for (int qi = 0; qi < kSmallQ; qi++) sc4[qi][j] += qi < nq ? A[qi][kc] : 0;
      }
    }
    for (int qi = 0; qi < nq; qi++) {
      unsigned long long key = 0ull;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int c = c4 + j;
        if (c < C && sc4[qi][j] > 0) {
          const unsigned long long k = ((unsigned long long)(unsigned)sc4[qi][j] << 32) | (unsigned)tiekey[c];
          key = k > key ? k : key;
        }
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off, 64);
        key = o > key ? o : key;
      }
      if (lane == 0) bmax[qi][wv] = key;
    }
    __syncthreads();
    if (threadIdx.x < nq) {
      unsigned long long key = bmax[threadIdx.x][0];
      for (int i = 1; i < 4; i++) key = bmax[threadIdx.x][i] > key ? bmax[threadIdx.x][i] : key;
      small_result_parts(out)[(int64_t)blockIdx.x * kSmallQ + threadIdx.x] = key;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out->ku = ku;
    out->bad = bad;
  }
}

hipError_t launch_search_small(const double* d_q, const SmallQueries& sq, SearchConsts sc, const uint32_t* d_bits,
                               int32_t C, const int32_t* d_tiekey, SmallResult* h_out, hipStream_t s) {
  if (sq.nq <= 0 || sq.nq > kSmallQ || C <= 0 || !h_out) return hipErrorInvalidValue;
  hipLaunchKernelGGL(small_vote_kernel, dim3(small_vote_blocks(C)), dim3(256), 0, s, d_q, sq, sc, d_bits, C, d_tiekey,
                     h_out);
  return hipGetLastError();
}

// ---- general path (any coefs / tolerance): one wave per query, frames in order; per frame the
// rows with max1 in [L1, U1] (binary search on the sorted index) filtered by the max2 box; each
// clip counts once per frame (stamp), i.e. the per-frame GROUP BY audio_uuid of :353.
}  // namespace tfp

