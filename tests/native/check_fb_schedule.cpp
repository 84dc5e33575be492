// The 8 kHz throughput kernel's frame-pair filterbank schedule (tfp_tables.cpp build_fb_schedule)
// against the dense filterbank: every non-empty filter is exactly one job (consecutive segments
// of one pattern, restarted at its first segment only), the job's weights over its bins equal the
// filter's dense row bit for bit with zeros elsewhere, every bin read is in [0, 257] and
// step pairs read 16-byte aligned pairs of bins. Prints "OK" or the first violation.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tfp_tables.hpp"

using namespace tfp;

static DspTables T;
static float mel[kFilters][kBins];

int main(int argc, char** argv) {
  const int sr = argc > 1 ? atoi(argv[1]) : 8000;
  if (!build_tables(sr, &T)) { printf("build_tables failed\n"); return 2; }
  if (!T.fb_ok) { printf("no frame-pair schedule at %d Hz\n", sr); return 3; }
  build_mel_dense(sr, mel);
  int jobs_of[kFilters];
  memset(jobs_of, 0, sizeof jobs_of);
  for (int p = 0; p < kFbPatterns; p++) {
    for (int k = 0; k < kFbSegs; k++) {
      const int f = T.fb_filter[p][k];
      if (f < 0 || f >= T.fb_nfilters) { printf("pattern %d segment %d: filter %d\n", p, k, f); return 1; }
      if ((T.fb_bin[p][k] & 1) != 0) { printf("pattern %d segment %d: odd first bin\n", p, k); return 1; }
      if (k > 0 && !T.fb_new[p][k]) {  // continuation: same filter, bins continue
        if (T.fb_filter[p][k - 1] != f || T.fb_bin[p][k] != T.fb_bin[p][k - 1] + kFbSegStart[k] - kFbSegStart[k - 1]) {
          printf("pattern %d segment %d: broken continuation\n", p, k);
          return 1;
        }
      }
      if (k == 0 && !T.fb_new[p][k]) { printf("pattern %d: segment 0 continues\n", p); return 1; }
      if (!T.fb_new[p][k]) continue;
      jobs_of[f]++;
      int k1 = k;  // the job's last segment
      while (k1 + 1 < kFbSegs && !T.fb_new[p][k1 + 1]) k1++;
      float dense[kBins + 2];
      memset(dense, 0, sizeof dense);
      for (int s = kFbSegStart[k]; s < kFbSegStart[k1 + 1]; s++) {
        const int b = T.fb_bin[p][k] + s - kFbSegStart[k];
        if (b < 0 || b >= kFbRowBins) { printf("pattern %d step %d: bin %d\n", p, s, b); return 1; }
        const float w = T.fb_w[s / 2][p][s % 2];
        if (b >= kBins) {
          if (w != 0.f) { printf("pattern %d: weight on the pad bin\n", p); return 1; }
          continue;
        }
        dense[b] = w;
      }
      if (memcmp(dense, mel[f], sizeof(float) * kBins) != 0) { printf("filter %d: weights differ\n", f); return 1; }
    }
  }
  for (int f = 0; f < kFilters; f++) {
    bool nonempty = false;
    for (int b = 0; b < kBins; b++) nonempty |= mel[f][b] != 0.f;
    if (jobs_of[f] != (nonempty ? 1 : 0)) { printf("filter %d: %d jobs\n", f, jobs_of[f]); return 1; }
  }
  printf("OK: %d filters in %d patterns x %d steps\n", T.fb_nfilters, kFbPatterns, kFbSteps);
  return 0;
}
