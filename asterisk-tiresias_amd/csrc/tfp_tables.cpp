// tfp_tables.cpp — host construction of DspTables (see tfp_tables.hpp for provenance).
// Compiled with -ffp-contract=off -fno-builtin so every float expression rounds where the
// C source of libaubio rounds and cosf/powf are glibc's run-time functions.
#include <mutex>
#include <vector>
#include "tfp_tables.hpp"
#include "tfp_math.hpp"

#include <math.h>
#include <string.h>

namespace tfp {

namespace {
const double kPi = 3.14159265358979323846;  // aubio_priv.h PI
const double kTwoPi = kPi * 2.;             // aubio_priv.h TWO_PI

void hanningz(float* w, unsigned size) {
  for (unsigned i = 0; i < size; i++) {
    const float c = cosf((float)(kTwoPi * i / size));
    w[i] = (float)(0.5 * (1.0 - (double)c));
  }
}

// (cos t, -sin t), t = 2 pi j / N; exact at quarter turns.
void twiddles(int N, int count, float* re, float* im) {
  for (int j = 0; j < count; j++) {
    const int q = N / 4;
    if (j % q == 0) {
      switch ((j / q) & 3) {
        case 0: re[j] = 1.f; im[j] = 0.f; break;
        case 1: re[j] = 0.f; im[j] = -1.f; break;
        case 2: re[j] = -1.f; im[j] = 0.f; break;
        default: re[j] = 0.f; im[j] = 1.f; break;
      }
      continue;
    }
    const double t = (2.0 * kPi * (double)j) / (double)N;
    re[j] = (float)cos(t);
    im[j] = (float)(-sin(t));
  }
}
// Filterbank lane order with few LDS bank conflicts. The kernels read |X| for 4 bins per lane
// with ds_read_b128 from per-frame rows that start at 16-B slot 136 g + 4 (g & 1) (frame g of a
// wave: fingerprint_kernel / fingerprint8k_kernel's |X| row). Such a read is served in four
// 16-lane groups; two lanes of a group collide when they read different slots that are equal
// mod 16. Which lane computes which filter of a slot is free (each sum goes to its filter's log
// row), so this permutes the slot's lanes to minimise the modelled extra cycles: deterministic
// random restarts + pairwise swaps.
int bank_cost(const int32_t* filt, const int32_t* start, const int* perm, int len) {
  static const int G[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                               {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                               {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                               {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  int extra = 0;
  for (int i = 0; i < len / 4; i++)
    for (int g = 0; g < 4; g++) {
      int slot_of_bank[16], cnt[16];
      for (int b = 0; b < 16; b++) { slot_of_bank[b] = -1; cnt[b] = 0; }
      int worst = 0;
      for (int k = 0; k < 16; k++) {
        const int l = G[g][k], fr = l >> 4, L = l & 15;
        if (filt[perm[L]] < 0) continue;
        const int sl = 136 * fr + 4 * (fr & 1) + start[perm[L]] / 4 + i;
        const int b = sl & 15;
        // distinct slots on one bank group cost a cycle each (same slot broadcasts); lanes of one
        // frame never share a slot, lanes of two frames do only by coincidence: count distinct
        if (slot_of_bank[b] != sl) { cnt[b]++; slot_of_bank[b] = sl; }
        if (cnt[b] > worst) worst = cnt[b];
      }
      extra += worst > 0 ? worst - 1 : 0;
    }
  return extra;
}

void lane_order_for_banks(int32_t* filt, int32_t* start, int len) {
  int best[16], perm[16];
  for (int L = 0; L < 16; L++) best[L] = L;
  int best_cost = bank_cost(filt, start, best, len);
  uint32_t rng = 0x9e3779b9u;
  for (int rs = 0; rs < 64 && best_cost > 0; rs++) {
    for (int L = 0; L < 16; L++) perm[L] = L;
    for (int L = 15; L > 0; L--) {  // Fisher-Yates with an LCG: deterministic
      rng = rng * 1664525u + 1013904223u;
      const int r = (int)((rng >> 8) % (uint32_t)(L + 1));
      const int x = perm[L]; perm[L] = perm[r]; perm[r] = x;
    }
    int c = bank_cost(filt, start, perm, len);
    for (bool improved = true; improved;) {
      improved = false;
      for (int a = 0; a < 16; a++)
        for (int b = a + 1; b < 16; b++) {
          int x = perm[a]; perm[a] = perm[b]; perm[b] = x;
          const int c2 = bank_cost(filt, start, perm, len);
          if (c2 < c) { c = c2; improved = true; }
          else { x = perm[a]; perm[a] = perm[b]; perm[b] = x; }
        }
    }
    if (c < best_cost) { best_cost = c; for (int L = 0; L < 16; L++) best[L] = perm[L]; }
  }
  int32_t f2[16], s2[16];
  for (int L = 0; L < 16; L++) { f2[L] = filt[best[L]]; s2[L] = start[best[L]]; }
  for (int L = 0; L < 16; L++) { filt[L] = f2[L]; start[L] = s2[L]; }
}
}  // namespace

void build_mel_dense(int sample_rate, float (*mel)[kBins]) {
  // aubio_filterbank_set_mel_coeffs_slaney: Malcolm Slaney's auditory-toolbox constants.
  const float lowest = 133.3333f;
  const float lin_spacing = 66.66666666f;
  const float log_spacing = 1.0711703f;
  const unsigned n_lin = 13, n_log = 27, n_filters = kFilters;
  float freqs[n_lin + n_log + 2];
  for (unsigned fn = 0; fn < n_lin; fn++) {
    const float step = (float)fn * lin_spacing;
    freqs[fn] = lowest + step;
  }
  const float last_lin = freqs[n_lin - 1];
  for (unsigned fn = 0; fn < n_log + 2; fn++)
    freqs[n_lin + fn] = last_lin * powf(log_spacing, (float)(fn + 1));

  // aubio_filterbank_set_triangle_bands
  const float sr = (float)sample_rate;
  const unsigned nb = kBins;
  float fft_freqs[kBins];
  const float bin_hz = sr / (float)((nb - 1) * 2);  // aubio_bintofreq
  for (unsigned b = 0; b < nb; b++) fft_freqs[b] = bin_hz * (float)b;
  memset(mel, 0, sizeof(float) * kFilters * kBins);
  for (unsigned fn = 0; fn < n_filters; fn++) {
    const float lo = freqs[fn], ce = freqs[fn + 1], up = freqs[fn + 2];
    const float height = (float)(2. / (double)(up - lo));  // unit-area triangles
    unsigned b = 0;
    for (; b < nb - 1; b++) {                                // skip first elements
      if (fft_freqs[b] <= lo && fft_freqs[b + 1] > lo) { b++; break; }
    }
    const float rise = height / (ce - lo);
    for (; b < nb - 1; b++) {
      mel[fn][b] = (fft_freqs[b] - lo) * rise;
      if (fft_freqs[b + 1] >= ce) { b++; break; }
    }
    const float down = height / (up - ce);
    for (; b < nb - 1; b++) {
      mel[fn][b] += (up - fft_freqs[b]) * down;
      if (mel[fn][b] < 0.f) mel[fn][b] = 0.f;
      if (fft_freqs[b + 1] >= up) break;
    }
  }
}

// Pattern-to-lane order of the frame-pair schedule with few LDS bank conflicts. Lane 16 p + j
// reads its pattern's bins (b, b + 1) of pair p's interleaved row as one 16-B slot b / 2, the odd
// pairs' rows 8 slots further round the banks (kFbRow); a ds_read_b128 is served in the four
// 16-lane groups of bank_cost, each mixing 8 lanes of an even pair with 8 of an odd one. Same
// search as lane_order_for_banks over which pattern each j runs.
static int fb_bank_cost(const DspTables* t, const int* perm) {
  static const int G[2][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                               {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31}};  // (groups 2, 3 alike)
  int extra = 0;
  for (int s = 0; s < kFbSteps; s += 2) {
    int k = 0;
    while (s >= kFbSegStart[k + 1]) k++;
    for (const auto& g : G) {
      int slot_of_bank[16], cnt[16], worst = 0;
      for (int b = 0; b < 16; b++) { slot_of_bank[b] = -1; cnt[b] = 0; }
      for (int l : g) {
        const int p = l >> 4, pat = perm[l & 15];
        const int sl = (t->fb_bin[pat][k] + s - kFbSegStart[k]) / 2 + 8 * (p & 1);
        const int b = sl & 15;
        if (slot_of_bank[b] != sl) { cnt[b]++; slot_of_bank[b] = sl; }  // a rough count, as bank_cost
        if (cnt[b] > worst) worst = cnt[b];
      }
      extra += worst - 1;
    }
  }
  return extra;
}

static void fb_order_for_banks(DspTables* t) {
  int best[kFbPatterns], perm[kFbPatterns];
  for (int j = 0; j < kFbPatterns; j++) best[j] = j;
  int best_cost = fb_bank_cost(t, best);
  uint32_t rng = 0x9e3779b9u;
  for (int rs = 0; rs < 64 && best_cost > 0; rs++) {
    for (int j = 0; j < kFbPatterns; j++) perm[j] = j;
    for (int j = kFbPatterns - 1; j > 0; j--) {  // Fisher-Yates with an LCG: deterministic
      rng = rng * 1664525u + 1013904223u;
      const int r = (int)((rng >> 8) % (uint32_t)(j + 1));
      const int x = perm[j]; perm[j] = perm[r]; perm[r] = x;
    }
    int c = fb_bank_cost(t, perm);
    for (bool improved = true; improved;) {
      improved = false;
      for (int a = 0; a < kFbPatterns; a++)
        for (int b = a + 1; b < kFbPatterns; b++) {
          int x = perm[a]; perm[a] = perm[b]; perm[b] = x;
          const int c2 = fb_bank_cost(t, perm);
          if (c2 < c) { c = c2; improved = true; }
          else { x = perm[a]; perm[a] = perm[b]; perm[b] = x; }
        }
    }
    if (c < best_cost) { best_cost = c; for (int j = 0; j < kFbPatterns; j++) best[j] = perm[j]; }
  }
  int bin[kFbPatterns][kFbSegs], nw[kFbPatterns][kFbSegs], fil[kFbPatterns][kFbSegs];
  float w[kFbSteps / 2][kFbPatterns][2];
  memcpy(bin, t->fb_bin, sizeof bin);
  memcpy(nw, t->fb_new, sizeof nw);
  memcpy(fil, t->fb_filter, sizeof fil);
  memcpy(w, t->fb_w, sizeof w);
  for (int j = 0; j < kFbPatterns; j++) {
    for (int k = 0; k < kFbSegs; k++) {
      t->fb_bin[j][k] = bin[best[j]][k];
      t->fb_new[j][k] = nw[best[j]][k];
      t->fb_filter[j][k] = fil[best[j]][k];
    }
    for (int q = 0; q < kFbSteps / 2; q++)
      for (int i = 0; i < 2; i++) t->fb_w[q][j][i] = w[q][best[j]][i];
  }
}

// The frame-pair schedule (DspTables::fb_*): best-fit decreasing. Filters, longest span first
// (span = the filter's bins from its start rounded down to even, rounded up to even), each take
// the run of consecutive free segments of an open pattern that fits them with the least slack,
// or open a new pattern (up to 16) at the least-slack run. A job's window of bins starts at the
// filter's even-rounded start, moved down when the window would pass bin 257, so every read is a
// bin of the |X| row or its zero pad.
static void build_fb_schedule(DspTables* t) {
  t->fb_ok = 0;
  int nf = 0;
  while (nf < kFilters && t->mel_len[nf] > 0) nf++;
  for (int f = nf; f < kFilters; f++)
    if (t->mel_len[f] > 0) return;  // the kernel keeps the logs of filters [0, nf) only
  t->fb_nfilters = nf;
  int order[kFilters], span[kFilters];
  for (int f = 0; f < nf; f++) {
    span[f] = (t->mel_start[f] & 1) + t->mel_len[f];
    span[f] += span[f] & 1;
    order[f] = f;
  }
  for (int a = 0; a < nf; a++)  // stable selection sort, longest span first
    for (int b = a + 1; b < nf; b++)
      if (span[order[b]] > span[order[a]]) { const int x = order[a]; order[a] = order[b]; order[b] = x; }
  int owner[kFbPatterns][kFbSegs];
  for (auto& o : owner)
    for (int& v : o) v = -1;
  int npat = 0;
  memset(t->fb_w, 0, sizeof t->fb_w);
  for (int q = 0; q < nf; q++) {
    const int f = order[q], need = span[f];
    int bp = -1, bk0 = 0, bk1 = 0, bw = 1 << 30;
    auto scan = [&](int p) {
      for (int k0 = 0; k0 < kFbSegs; k0++)
        for (int k1 = k0; k1 < kFbSegs && owner[p][k1] < 0; k1++) {
          const int cap = kFbSegStart[k1 + 1] - kFbSegStart[k0];
          if (cap >= need && cap - need < bw) { bw = cap - need; bp = p; bk0 = k0; bk1 = k1; }
        }
    };
    for (int p = 0; p < npat; p++) scan(p);
    if (bp < 0) {
      if (npat == kFbPatterns) return;
      scan(npat++);
      if (bp < 0) return;  // longer than a whole pattern
    }
    const int cap = kFbSegStart[bk1 + 1] - kFbSegStart[bk0];
    const int start = t->mel_start[f], len = t->mel_len[f];
    int b0 = start & ~1;
    if (b0 + cap > kFbRowBins) b0 = (kFbRowBins - cap) & ~1;
    if (b0 < 0 || b0 > start || b0 + cap < start + len) return;
    for (int k = bk0; k <= bk1; k++) {
      owner[bp][k] = f;
      t->fb_bin[bp][k] = b0 + kFbSegStart[k] - kFbSegStart[bk0];
      t->fb_new[bp][k] = k == bk0;
      t->fb_filter[bp][k] = f;
    }
    for (int s = kFbSegStart[bk0]; s < kFbSegStart[bk1 + 1]; s++) {
      const int b = b0 + s - kFbSegStart[bk0];
      t->fb_w[s / 2][bp][s % 2] = (b >= start && b < start + len) ? t->mel_w[t->mel_off[f] + b - start] : 0.f;
    }
  }
  for (int p = 0; p < kFbPatterns; p++)
    for (int k = 0; k < kFbSegs; k++)
      if (owner[p][k] < 0) return;  // the kernel has no idle lanes
  fb_order_for_banks(t);
  t->fb_ok = 1;
}

bool build_tables(int sample_rate, DspTables* t) {
  if (sample_rate <= 0 || !t) return false;
  memset(t, 0, sizeof *t);
  t->sample_rate = sample_rate;
  hanningz(t->window, kWin);
  twiddles(256, 256, t->tw256_re, t->tw256_im);
  twiddles(512, kBins, t->tw512_re, t->tw512_im);

  // new_aubio_mfcc (0.4.5): scaling = 1/SQRT(n/2); row j: scaling*COS(j(i+.5)PI/n); row 0 *= SQRT(2)/2
  const unsigned n = kFilters;
  const float scaling = (float)(1. / (double)sqrtf((float)(n / 2.)));
  const double row0 = (double)sqrtf(2.f) / 2.;
  for (unsigned i = 0; i < n; i++) {
    for (unsigned j = 0; j < (unsigned)kCoefs; j++)
      t->dct[j][i] = scaling * cosf((float)(j * (i + 0.5) * kPi / n));
    t->dct[0][i] = (float)((double)t->dct[0][i] * row0);
  }

  // (per call, not static: engines of a device group build their tables in parallel threads)
  std::vector<float> mel_buf((size_t)kFilters * kBins);
  float (*mel)[kBins] = reinterpret_cast<float (*)[kBins]>(mel_buf.data());
  build_mel_dense(sample_rate, mel);
  int off = 0;
  for (int j = 0; j < kFilters; j++) {
    int first = -1, last = -1;
    for (int b = 0; b < kBins; b++)
      if (mel[j][b] != 0.f) { if (first < 0) first = b; last = b; }
    t->mel_off[j] = off;
    if (first < 0) { t->mel_start[j] = 0; t->mel_len[j] = 0; continue; }
    t->mel_start[j] = first;
    t->mel_len[j] = last - first + 1;
    for (int b = first; b <= last; b++) t->mel_w[off++] = mel[j][b];
  }
  t->mel_total = off;

  // filterbank slot schedule: each filter's bins are read from its start rounded down to a
  // multiple of 4, so the kernel reads |X| with aligned 16-byte loads; the lead-in weights are
  // zero and add exact +0 to the +0 sum (fmat_vecmul sums every bin from 0 anyway)
  int order[kFilters], lead[kFilters];
  for (int j = 0; j < kFilters; j++) lead[j] = t->mel_len[j] ? (t->mel_start[j] & 3) : 0;
  for (int j = 0; j < kFilters; j++) order[j] = j;
  auto span = [&](int j) { return t->mel_len[j] ? lead[j] + t->mel_len[j] : 0; };
  for (int a = 0; a < kFilters; a++)  // stable selection sort by span read, longest first
    for (int b = a + 1; b < kFilters; b++)
      if (span(order[b]) > span(order[a])) { const int x = order[a]; order[a] = order[b]; order[b] = x; }
  int woff = 0;
  for (int sl = 0; sl < 3; sl++) {
    int len = 0;
    for (int L = 0; L < 16; L++) {
      const int idx = sl * 16 + L;
      const int j = idx < kFilters ? order[idx] : -1;
      t->ms_filter[sl][L] = j;
      t->ms_start[sl][L] = j >= 0 ? t->mel_start[j] - lead[j] : 0;
      if (j >= 0 && t->mel_len[j] && lead[j] + t->mel_len[j] > len) len = lead[j] + t->mel_len[j];
    }
    len = (len + 3) & ~3;
    lane_order_for_banks(t->ms_filter[sl], t->ms_start[sl], len);
    t->ms_len[sl] = len;
    t->ms_woff[sl] = woff;
    for (int L = 0; L < 16; L++)
      for (int q = 0; q < len; q++) {
        const int j = t->ms_filter[sl][L];
        const int r = j >= 0 ? q - lead[j] : -1;
        // [slot][q / 4][lane][q % 4]: a 16-lane ds_read_b128 group reads 16 consecutive 16-B slots
        t->ms_w[woff + (q >> 2) * 64 + L * 4 + (q & 3)] =
            (j >= 0 && r >= 0 && r < t->mel_len[j]) ? t->mel_w[t->mel_off[j] + r] : 0.f;
      }
    woff += len * 16;
  }
  t->ms_total = woff;
  t->ms_c_real[0] = t->ms_c_real[1] = -1;
  int nreal = 0;
  for (int L = 0; L < 16; L++) {
    const int j = t->ms_filter[2][L];
    if (j >= 0 && t->mel_len[j] > 0) {
      if (nreal < 2) t->ms_c_real[nreal] = j;
      nreal++;
    }
  }
  t->ms_c_defer = nreal <= 2 ? 1 : 0;
  t->ms_maxbin = kBins;
  for (int sl = 0; sl < 3; sl++)
    for (int L = 0; L < 16; L++)
      if (t->ms_start[sl][L] + t->ms_len[sl] > t->ms_maxbin) t->ms_maxbin = t->ms_start[sl][L] + t->ms_len[sl];
  if (t->ms_maxbin > 500) return false;  // the kernel's per-frame |X| row holds 528 floats
  build_fb_schedule(t);
  for (int i = 0; i < kWin; i++) t->window_s[i] = t->window[i] * 0x1p-15f;
  for (int k1 = 0; k1 < 16; k1++)
    for (int L = 0; L < 16; L++) {
      t->lane_tw_re[k1][L] = t->tw256_re[(L * k1) & 255];
      t->lane_tw_im[k1][L] = t->tw256_im[(L * k1) & 255];
    }
  return true;
}

void log_fix_table(const uint32_t** keys, const double** vals, int32_t* n) {
  static std::vector<uint32_t> K;
  static std::vector<double> V;
  static std::once_flag once;
  std::call_once(once, [] {
    for (uint32_t i = 0; i < 2; i++)
      for (uint32_t m = 0; m < (1u << 23); m++) {
        const double x = u2d(((uint64_t)(0x3ff - i) << 52) | ((uint64_t)m << 29));
        const double want = log(x);  // glibc (built with -fno-builtin: no compile-time folding)
        if (d2u(log_acc(x)) != d2u(want)) {
          K.push_back((i << 23) | m);
          V.push_back(want);
        }
      }
  });
  *keys = K.data();
  *vals = V.data();
  *n = (int32_t)K.size();
}

void log_fix_hash(const uint32_t** keys, const double** vals, int32_t* n) {
  static std::vector<uint32_t> K;
  static std::vector<double> V;
  static int32_t N = 0;
  static std::once_flag once;
  std::call_once(once, [] {
    const uint32_t* k;
    const double* v;
    log_fix_table(&k, &v, &N);
    const uint32_t mask = (1u << kLogFixHashBits) - 1;
    K.assign(mask + 1, kLogFixEmpty);
    V.assign(mask + 1, 0.0);
    for (int32_t j = 0; j < N; j++) {
      uint32_t h = log_fix_slot(k[j]);
      while (K[h] != kLogFixEmpty) h = (h + 1) & mask;
      K[h] = k[j];
      V[h] = v[j];
    }
  });
  *keys = K.data();
  *vals = V.data();
  *n = N;
}

}  // namespace tfp
