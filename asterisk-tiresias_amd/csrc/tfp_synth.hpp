// tfp_synth.hpp — deterministic synthetic 8 kHz PCM (benchmark / test data).
//
// Counter-based and integer-only, so sample s of clip c is the same value on the host and on
// the GPU and can be generated in any order: 2-5 tones (100-3800 Hz) with a slow AM envelope,
// uniform noise and 0-20 % silent 2048-sample gaps (these exercise the silent-frame
// max2 rounding-residue case), peak around -6 dBFS.
#pragma once
#include <stdint.h>

#ifndef TFP_HD
#if defined(__HIPCC__) || defined(__HIP__)
#define TFP_HD __host__ __device__ inline
#else
#define TFP_HD static inline
#endif
#endif

namespace tfp {

TFP_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Parabolic sine, Q15, one period per 2^32 of phase.
TFP_HD int32_t isin_q15(uint32_t phase) {
  const uint32_t p = phase >> 17;
  const int32_t half = (int32_t)(p & 16383u);
  int32_t y = (half * (16384 - half)) >> 11;
  if (y > 32767) y = 32767;
  return (p & 16384u) ? -y : y;
}

struct SynthClip {
  int32_t ntones;
  uint32_t inc[5], ph0[5];
  int32_t amp[5];
  uint32_t am_inc;
  int32_t am_depth;  // Q15
  int32_t noise_amp;
  int32_t gap_pct;
  uint64_t key;
};

TFP_HD SynthClip synth_clip(uint64_t seed, int64_t clip) {
  SynthClip p;
  uint64_t h = splitmix64(seed ^ splitmix64((uint64_t)clip * 0x2545F4914F6CDD1Dull));
  p.key = h;
  p.ntones = 2 + (int32_t)(h % 4u);
  int32_t budget = 15000;
  for (int i = 0; i < 5; i++) {
    h = splitmix64(h);
    // 100 .. 3800 Hz at 8 kHz: inc = f / 8000 * 2^32
    p.inc[i] = 53687091u + (uint32_t)(h % 1986422374u);
    p.ph0[i] = (uint32_t)(h >> 32);
    const int32_t a = budget / (p.ntones - (i < p.ntones ? i : 0) + 1) + (int32_t)((h >> 20) % 2000u);
    p.amp[i] = i < p.ntones ? a : 0;
    if (i < p.ntones) budget -= a / 2;
  }
  h = splitmix64(h);
  p.am_inc = 53687u + (uint32_t)(h % 2147483u);  // 0.1 .. 4 Hz
  p.am_depth = (int32_t)((h >> 24) % 24000u);
  p.noise_amp = 64 + (int32_t)((h >> 40) % 1500u);
  p.gap_pct = (int32_t)((h >> 52) % 21u);
  return p;
}

TFP_HD int16_t synth_sample(const SynthClip& p, int64_t s) {
  if (s < 0) return 0;
  const uint64_t blk = (uint64_t)s >> 11;
  if ((int32_t)(splitmix64(p.key ^ (blk * 0x9E3779B97F4A7C15ull)) % 100u) < p.gap_pct) return 0;
  int32_t acc = 0;
  for (int i = 0; i < 5; i++) {
    if (i >= p.ntones) break;
    const uint32_t ph = p.inc[i] * (uint32_t)s + p.ph0[i];
    acc += (p.amp[i] * isin_q15(ph)) >> 15;
  }
  const int32_t env = 32768 - ((p.am_depth * (isin_q15(p.am_inc * (uint32_t)s) + 32767)) >> 16);
  acc = (int32_t)(((int64_t)acc * env) >> 15);
  const uint64_t n = splitmix64(p.key + (uint64_t)s * 0xD1B54A32D192ED03ull);
  acc += (((int32_t)(n >> 52) - 2048) * p.noise_amp) >> 11;
  if (acc > 32767) acc = 32767;
  if (acc < -32768) acc = -32768;
  return (int16_t)acc;
}

}  // namespace tfp
