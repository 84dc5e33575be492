/* Batch-1 search latency measured from C, the way the Asterisk shim's channel threads call the
 * engine (fp_search_fingerprint_info -> tfp_search_pcm_batch). Benchmark
 * harness only (bench.py loads it next to libtiresias_fp.so); not part of the C-ABI.
 *
 * For i < iters: query q = i % nqueries (n samples each, contiguous in pcm), one
 * tfp_search_pcm_batch call, wall time in ms -> out_ms[i]; found[i] = the result's found flag.
 * The queries are first copied (untimed) into one tfp_host_alloc buffer, as the shim reads its
 * WAV files into one: the engine then reads each query's samples where they lie. */
#define _POSIX_C_SOURCE 199309L
#include <string.h>
#include <time.h>

#include "tiresias_fp.h"

static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e3 + (double)t.tv_nsec * 1e-6;
}

int tfp_latency_search_pcm(tfp_engine* eng, const int16_t* pcm, int64_t n, int32_t nqueries, int32_t sample_rate,
                           const tfp_search_params* params, int32_t iters, double* out_ms, int32_t* found) {
  int32_t i;
  int rc = TFP_OK;
  int16_t* hq = NULL;
  if (!eng || !pcm || n <= 0 || nqueries <= 0 || iters < 0 || !params || (iters && (!out_ms || !found)))
    return TFP_E_ARG;
  if (tfp_host_alloc(sizeof(int16_t) * (size_t)n * (size_t)nqueries, (void**)&hq) != TFP_OK) return TFP_E_NOMEM;
  memcpy(hq, pcm, sizeof(int16_t) * (size_t)n * (size_t)nqueries);
  for (i = 0; i < iters && rc == TFP_OK; i++) {
    const int64_t off[2] = {0, n};
    tfp_result r;
    double t0 = now_ms(), t1;
    rc = tfp_search_pcm_batch(eng, hq + (int64_t)(i % nqueries) * n, off, 1, sample_rate, params, &r);
    t1 = now_ms();
    out_ms[i] = t1 - t0;
    found[i] = r.found;
  }
  tfp_host_free(hq);
  return rc;
}
