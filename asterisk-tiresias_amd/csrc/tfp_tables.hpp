// tfp_tables.hpp — per-sample-rate DSP constants, built on the host, uploaded once.
//
// The expressions follow libaubio 0.4.5 exactly in float (smpl_t) arithmetic, because the
// reference computes them that way when create_audio_fingerprints() calls
// new_aubio_pvoc(512, 256) and new_aubio_mfcc(512, 40, 2, samplerate)
// (/root/reference/src/fp_handler.c:613-615):
//   window  fvec_set_window("hanningz")                       phasevoc.c / mathutils.c
//   mel     aubio_filterbank_set_mel_coeffs_slaney +
//           aubio_filterbank_set_triangle_bands               filterbank_mel.c
//   dct     new_aubio_mfcc DCT rows j = 0, 1                  mfcc.c
// Twiddles are this project's canonical FFT (the reference's FFT backend is unpinned).
#pragma once
#include <stdint.h>

namespace tfp {

constexpr int kHop = 256, kWin = 512, kBins = 257, kFilters = 40, kCoefs = 2;

// Device-resident table block (one per sample rate). Mel filters are stored sparse:
// filter j covers bins [mel_start[j], mel_start[j] + mel_len[j]) with weights at mel_w[mel_off[j] ...].
struct DspTables {
  float window[kWin];
  float tw256_re[256], tw256_im[256];
  float tw512_re[kBins], tw512_im[kBins];
  float dct[kCoefs][kFilters];
  int32_t mel_start[kFilters], mel_len[kFilters], mel_off[kFilters];
  int32_t mel_total;
  int32_t sample_rate;
  float mel_w[kFilters * kBins];
};

// Dense filterbank as aubio lays it out (40 x 257), for tests.
void build_mel_dense(int sample_rate, float (*mel)[kBins]);
bool build_tables(int sample_rate, DspTables* t);

}  // namespace tfp
