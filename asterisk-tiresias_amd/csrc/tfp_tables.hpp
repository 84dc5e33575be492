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

// Frame-pair filterbank schedule of the 8 kHz throughput kernel (fingerprint8k_kernel<4>): 16
// patterns of kFbSteps steps in kFbSegs fixed segments [kFbSegStart[k], kFbSegStart[k + 1]).
constexpr int kFbSteps = 36, kFbSegs = 4, kFbPatterns = 16;
constexpr int kFbSegStart[kFbSegs + 1] = {0, 10, 20, 26, 36};
constexpr int kFbRowBins = 258;  // bins a pattern step may read: 0..257 (257 reads the zero pad)

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
  // Kernel schedule of the filterbank: filters sorted by the span they read are dealt to 3
  // slots x 16 lanes (slot 0 = the 16 longest); a lane computes one sum per slot. Each span
  // starts at the filter's first bin rounded down to a multiple of 4 and is zero-padded to the
  // slot's longest span rounded up to 4 (zero weights add exact +0 before the first and after
  // the last bin, so every sum is still aubio's sequential ascending-bin sum).
  int32_t ms_len[3];         // padded slot length (multiple of 4)
  int32_t ms_filter[3][16];  // filter id or -1
  int32_t ms_start[3][16];   // first bin read, a multiple of 4 (leading weights are zero)
  int32_t ms_woff[3];        // offset of slot s in ms_w
  int32_t ms_total;          // floats used in ms_w
  int32_t ms_maxbin;         // 1 + the highest bin a padded slot reads (bins > 256 read zeros)
  alignas(16) float ms_w[3 * (kBins + 8) * 16];  // [slot][q / 4][lane][q % 4], slot at ms_woff
  // hanningz window pre-scaled by 2^-15 (exact): x = (float)sample * window_s[j] equals aubio's
  // ((float)sample / 32768) * window[j] bit for bit.
  float window_s[kWin];
  // Inter-stage FFT twiddles per lane: lane_tw[k1][L] = w256^(L*k1) (re, im), conflict-free reads.
  float lane_tw_re[16][16], lane_tw_im[16][16];
  // Slot 2 with at most 2 non-empty filters (8 kHz: 2 real + 6 empty): the kernel writes those
  // 2 raw sums and takes their logs once per 16-frame tile on 32 lanes, instead of a third
  // log per lane per pass; empty filters' log rows hold the constant log of the clamped 0.
  int32_t ms_c_defer;       // 1 when slot 2 qualifies
  int32_t ms_c_real[2];     // its non-empty filter ids (-1: none)
  // The frame-pair schedule (kFbSteps above). A lane sums one pattern for two frames at once
  // (packed), reading their interleaved |X| rows: step s of segment k reads bin
  // fb_bin[j][k] + s - kFbSegStart[k]. Every segment belongs to a job: one filter's sequential
  // sum over one or more consecutive segments, restarted where fb_new is set. Weights outside the
  // filter's bins are zero (exact +0 terms, as for the slots). fb_ok = 0: no such schedule
  // (more than 16 patterns needed, or a segment left uncovered).
  int32_t fb_ok;
  int32_t fb_nfilters;                          // non-empty filters, all below every empty one
  int32_t fb_bin[kFbPatterns][kFbSegs];
  int32_t fb_new[kFbPatterns][kFbSegs];
  int32_t fb_filter[kFbPatterns][kFbSegs];
  alignas(16) float fb_w[kFbSteps / 2][kFbPatterns][2];  // [step / 2][pattern][step % 2]
};

// Dense filterbank as aubio lays it out (40 x 257), for tests.
void build_mel_dense(int sample_rate, float (*mel)[kBins]);
bool build_tables(int sample_rate, DspTables* t);
// The reduced arguments where log_acc differs from this host's glibc log, with glibc's value
// (tfp_math.hpp LogFix), ascending keys; computed once per process (~0.3 s).
void log_fix_table(const uint32_t** keys, const double** vals, int32_t* n);
// The same entries as an open-addressing hash of 2^kLogFixHashBits slots (tfp_math.hpp
// log_fix_slot: multiplicative hash, linear probing, empty slots keyed kLogFixEmpty): the device
// lookup is one or two loads from a 512 KiB key array instead of a 16-step binary search.
void log_fix_hash(const uint32_t** keys, const double** vals, int32_t* n);

}  // namespace tfp
