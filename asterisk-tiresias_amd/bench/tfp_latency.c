/* Batch-1 search latency measured from C, the way the Asterisk shim's channel threads call the
 * engine (fp_search_fingerprint_info -> tfp_search_pcm_batch). Benchmark
 * harness only (bench.py loads it next to libtiresias_fp.so); not part of the C-ABI.
 *
 * For i < iters: query q = i % nqueries (n samples each, contiguous in pcm), one
 * tfp_search_pcm_batch call, wall time in ms -> out_ms[i]; found[i] = the result's found flag.
 * The queries are first copied (untimed) into one tfp_host_alloc buffer, as the shim reads its
 * WAV files into one: the engine then reads each query's samples where they lie. */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
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

/* Stream ticks from C, as the shim's channel threads would push them: ticks
 * t < nticks of pcm (int16 [nchannels][total] row-major, tick samples each, starting at sample
 * first), one tfp_stream_push per tick with results into one caller array; wall time per tick in
 * ms -> out_ms[t]; *found_last = the channels found on the last tick. */
int tfp_latency_stream(tfp_stream* st, const int16_t* pcm, int32_t nchannels, int64_t total, int64_t first,
                       int32_t tick, int32_t nticks, const tfp_search_params* params, double* out_ms,
                       int32_t* found_last) {
  int32_t t, c;
  int rc = TFP_OK;
  int16_t* blk;
  tfp_result* res;
  if (!st || !pcm || nchannels <= 0 || tick <= 0 || nticks < 0 || !params || !out_ms || !found_last ||
      first < 0 || first + (int64_t)tick * nticks > total)
    return TFP_E_ARG;
  if (tfp_host_alloc(sizeof(int16_t) * (size_t)nchannels * (size_t)tick, (void**)&blk) != TFP_OK) return TFP_E_NOMEM;
  if (tfp_host_alloc(sizeof(tfp_result) * (size_t)nchannels, (void**)&res) != TFP_OK) {
    tfp_host_free(blk);
    return TFP_E_NOMEM;
  }
  *found_last = 0;
  for (t = 0; t < nticks && rc == TFP_OK; t++) {
    double t0, t1;
    for (c = 0; c < nchannels; c++)  /* the tick's samples arrive: untimed, as the channel audio */
      memcpy(blk + (int64_t)c * tick, pcm + (int64_t)c * total + first + (int64_t)t * tick, sizeof(int16_t) * (size_t)tick);
    t0 = now_ms();
    rc = tfp_stream_push(st, blk, tick, params, res);
    t1 = now_ms();
    out_ms[t] = t1 - t0;
  }
  for (c = 0; c < nchannels; c++) *found_last += res[c].found;
  tfp_host_free(res);
  tfp_host_free(blk);
  return rc;
}

/* Searches per second from nthreads concurrent callers, as the module's channel threads make them
 * (application_handler.c:66, :180): each thread runs reps batch-1 tfp_search_pcm_batch calls, thread
 * t's r-th on query (t * 7 + r) % nqueries, every query in its own tfp_host_alloc buffer (the shim's
 * per-call WAV read). Wall time from the threads' common start to the last return -> *seconds;
 * found per call -> found[t * reps + r] (may be NULL). */
typedef struct {
  tfp_engine* eng;
  int16_t** q;
  int64_t n;
  int32_t nq, sr, t, reps;
  const tfp_search_params* p;
  int32_t* found;
  pthread_barrier_t* go;
  int rc;
} lat_thread;

static void* lat_thread_main(void* v) {
  lat_thread* a = (lat_thread*)v;
  int32_t r;
  pthread_barrier_wait(a->go);
  for (r = 0; r < a->reps && a->rc == TFP_OK; r++) {
    const int64_t off[2] = {0, a->n};
    tfp_result res;
    a->rc = tfp_search_pcm_batch(a->eng, a->q[(a->t * 7 + r) % a->nq], off, 1, a->sr, a->p, &res);
    if (a->found) a->found[(int64_t)a->t * a->reps + r] = res.found;
  }
  return NULL;
}

int tfp_latency_threads(tfp_engine* eng, const int16_t* pcm, int64_t n, int32_t nqueries, int32_t sample_rate,
                        const tfp_search_params* params, int32_t nthreads, int32_t reps, double* seconds,
                        int32_t* found) {
  pthread_t* th;
  lat_thread* args;
  int16_t** q;
  pthread_barrier_t go;
  int32_t i;
  int rc = TFP_OK;
  double t0;
  if (!eng || !pcm || n <= 0 || nqueries <= 0 || nthreads <= 0 || reps < 0 || !params || !seconds) return TFP_E_ARG;
  q = (int16_t**)calloc((size_t)nqueries, sizeof *q);
  th = (pthread_t*)calloc((size_t)nthreads, sizeof *th);
  args = (lat_thread*)calloc((size_t)nthreads, sizeof *args);
  for (i = 0; i < nqueries && rc == TFP_OK; i++) {
    rc = tfp_host_alloc(sizeof(int16_t) * (size_t)n, (void**)&q[i]);
    if (rc == TFP_OK) memcpy(q[i], pcm + (int64_t)i * n, sizeof(int16_t) * (size_t)n);
  }
  if (rc == TFP_OK) {
    pthread_barrier_init(&go, NULL, (unsigned)nthreads + 1);
    for (i = 0; i < nthreads; i++) {
      lat_thread a = {eng, q, n, nqueries, sample_rate, i, reps, params, found, &go, TFP_OK};
      args[i] = a;
      pthread_create(&th[i], NULL, lat_thread_main, &args[i]);
    }
    t0 = now_ms();
    pthread_barrier_wait(&go);
    for (i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    *seconds = (now_ms() - t0) * 1e-3;
    pthread_barrier_destroy(&go);
    for (i = 0; i < nthreads; i++)
      if (args[i].rc != TFP_OK) rc = args[i].rc;
  }
  for (i = 0; i < nqueries; i++) tfp_host_free(q[i]);
  free(q);
  free(th);
  free(args);
  return rc;
}

/* The same two loops through a device group (tfp_group_*: the shim's handle, one engine per GPU of
 * the node): batch-1 host-PCM searches, and stream ticks of a group stream. */
int tfp_latency_group_search_pcm(tfp_group* g, const int16_t* pcm, int64_t n, int32_t nqueries, int32_t sample_rate,
                                 const tfp_search_params* params, int32_t iters, double* out_ms, int32_t* found) {
  int32_t i;
  int rc = TFP_OK;
  int16_t* hq = NULL;
  if (!g || !pcm || n <= 0 || nqueries <= 0 || iters < 0 || !params || (iters && (!out_ms || !found)))
    return TFP_E_ARG;
  if (tfp_host_alloc(sizeof(int16_t) * (size_t)n * (size_t)nqueries, (void**)&hq) != TFP_OK) return TFP_E_NOMEM;
  memcpy(hq, pcm, sizeof(int16_t) * (size_t)n * (size_t)nqueries);
  for (i = 0; i < iters && rc == TFP_OK; i++) {
    const int64_t off[2] = {0, n};
    tfp_result r;
    double t0 = now_ms(), t1;
    rc = tfp_group_search_pcm_batch(g, hq + (int64_t)(i % nqueries) * n, off, 1, sample_rate, params, &r);
    t1 = now_ms();
    out_ms[i] = t1 - t0;
    found[i] = r.found;
  }
  tfp_host_free(hq);
  return rc;
}

int tfp_latency_group_stream(tfp_group_stream* st, const int16_t* pcm, int32_t nchannels, int64_t total, int64_t first,
                             int32_t tick, int32_t nticks, const tfp_search_params* params, double* out_ms,
                             int32_t* found_last) {
  int32_t t, c;
  int rc = TFP_OK;
  int16_t* blk;
  tfp_result* res;
  if (!st || !pcm || nchannels <= 0 || tick <= 0 || nticks < 0 || !params || !out_ms || !found_last ||
      first < 0 || first + (int64_t)tick * nticks > total)
    return TFP_E_ARG;
  if (tfp_host_alloc(sizeof(int16_t) * (size_t)nchannels * (size_t)tick, (void**)&blk) != TFP_OK) return TFP_E_NOMEM;
  if (tfp_host_alloc(sizeof(tfp_result) * (size_t)nchannels, (void**)&res) != TFP_OK) {
    tfp_host_free(blk);
    return TFP_E_NOMEM;
  }
  *found_last = 0;
  for (t = 0; t < nticks && rc == TFP_OK; t++) {
    double t0, t1;
    for (c = 0; c < nchannels; c++)
      memcpy(blk + (int64_t)c * tick, pcm + (int64_t)c * total + first + (int64_t)t * tick, sizeof(int16_t) * (size_t)tick);
    t0 = now_ms();
    rc = tfp_group_stream_push(st, blk, tick, params, res);
    t1 = now_ms();
    out_ms[t] = t1 - t0;
  }
  for (c = 0; c < nchannels; c++) *found_last += res[c].found;
  tfp_host_free(res);
  tfp_host_free(blk);
  return rc;
}
