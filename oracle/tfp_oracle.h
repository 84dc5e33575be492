/* tfp_oracle.h — CPU ORACLE (test infrastructure only; never linked into the product).
 *
 * A plain-C restatement of the reference hot path, used by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg as the checker:
 *   - create_audio_fingerprints()        /root/reference/src/fp_handler.c:577-671
 *     with libaubio 0.4.5 source/pvoc/mfcc semantics (un-vendored; restated, see oracle.c)
 *   - the "%f" storage rule              /root/reference/src/db_ctx_handler.c:479-481
 *   - fp_search_fingerprint_info() SQL   /root/reference/src/fp_handler.c:247-374
 *
 * Parity status: the search semantics are pinned against the reference's own SQL strings
 * executed by SQLite (tests/golden/, oracle/sql_oracle.py). The DSP arithmetic is pinned
 * for log10f/log10/%f against this image's glibc (exhaustive), but the FFT backend of the
 * reference build (fftw3f) cannot be reproduced: the FFT below is this project's canonical
 * 16x16 Cooley-Tukey restatement, so DSP parity to a real libaubio build is UNPINNED.
 */
#ifndef TFP_ORACLE_H
#define TFP_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#define TFO_HOP 256
#define TFO_WIN 512
#define TFO_BINS 257
#define TFO_FILTERS 40
#define TFO_COEFS 2
#define TFO_NULL INT32_MIN

typedef struct {
  int sample_rate;
  float window[TFO_WIN];
  float tw256_re[256], tw256_im[256];  /* exp(-2*pi*i*j/256) */
  float tw512_re[257], tw512_im[257];  /* exp(-2*pi*i*k/512) */
  float mel[TFO_FILTERS][TFO_BINS];    /* dense filterbank, aubio layout */
  float dct[TFO_COEFS][TFO_FILTERS];
} tfo_tables;

int tfo_build_tables(int sample_rate, tfo_tables* t);

/* Frames produced for n samples: ceil(n / 256) (aubio_source_do loop, fp_handler.c:632-636). */
size_t tfo_frame_count(size_t nsamples);

/* One clip. Per frame f: coef[2f..2f+1] = MFCC c0,c1 (float); db[2f..] = 10*log10|c| (glibc);
 * micro[2f..] = "%f" micro-units or TFO_NULL. Any output pointer may be NULL. Returns frames. */
size_t tfo_fingerprint(const tfo_tables* t, const int16_t* pcm, size_t n, float* coef, double* db,
                       int32_t* micro);
/* The same from fp32 hop values x (aubio's source output for multichannel / 24-32-bit / float
 * audio) instead of int16 PCM: x[s] replaces pcm[s] / 32768.f. */
size_t tfo_fingerprint_f32(const tfo_tables* t, const float* x, size_t n, float* coef, double* db,
                           int32_t* micro);

/* Batch of clips over `nthreads` POSIX threads (cpu_baseline). offsets has nclips+1 entries
 * (sample offsets); frame outputs are concatenated in clip order. Returns total frames. */
size_t tfo_fingerprint_batch(const tfo_tables* t, const int16_t* pcm, const int64_t* offsets,
                             int nclips, int32_t* micro, double* db, int nthreads);

/* The same with another valid fp32 FFT order in place of the canonical one (0), to measure how
 * much the unpinned FFT backend can move the stored values: 1 = radix-2 256-point complex FFT +
 * the canonical real split, 2 = radix-2 512-point complex FFT of the real input. */
/* variant bits (sensitivity study, scripts/fft_sensitivity.py): (variant & 3) = 1 radix-2 256-point
 * complex FFT + canonical split, 2 = radix-2 512-point complex FFT of the real input; FB_BLOCKED and
 * DCT_BLOCKED sum the filterbank / DCT rows in a vectorised-sgemv order instead of fmat_vecmul's */
#define TFO_VARIANT_FB_BLOCKED 4
#define TFO_VARIANT_DCT_BLOCKED 8
size_t tfo_fingerprint_batch_variant(const tfo_tables* t, const int16_t* pcm, const int64_t* offsets,
                                     int nclips, int32_t* micro, double* db, int nthreads, int variant);

/* fp_search_fingerprint_info over an in-memory audio_fingerprint table.
 *   rows:    m1/m2 micro-units (TFO_NULL = SQL NULL), row_clip = clip index
 *   uuids:   clip index -> audio_uuid string (tie-break: greatest string wins)
 *   query:   q1/q2 = the unrounded doubles create_audio_fingerprints produced for the query
 *            (+-inf/NaN when the JSON key was absent; read back as 0.0, fp_handler.c:290,321)
 * Returns 1 and sets winner and match_count on a hit, 0 for NOTFOUND (incl. bad coefs / SQL
 * error cases the reference maps to NULL), and *frame_count = nqframes. */
int tfo_search(const int32_t* m1, const int32_t* m2, const int32_t* row_clip, int64_t nrows,
               const char* const* uuids, int32_t nclips, const double* q1, const double* q2,
               int32_t nqframes, int coefs, double tolerance, int freq_ignore_low,
               int freq_ignore_high, int32_t* winner, int32_t* match_count, int32_t* frame_count);

/* Large tables (configs[2] size): the same search semantics over rows sorted by max1.
 * tfo_sort_rows orders (m1, m2, clip) by m1 (stable LSD radix sort; returns n or -1).
 * tfo_search_sorted_batch runs nq queries (frames qoff[q]..qoff[q+1]) over the sorted rows with
 * a binary search per frame box, on nthreads threads; tiekey[clip] orders clips like their uuid
 * strings (the greatest wins a tie). winner[q] = clip or -1 (NOTFOUND), match_count[q]. */
int64_t tfo_sort_rows(const int32_t* m1, const int32_t* m2, const int32_t* clip, int64_t n, int32_t* om1,
                      int32_t* om2, int32_t* oclip);
int tfo_search_sorted_batch(const int32_t* m1s, const int32_t* m2s, const int32_t* row_clip, int64_t nrows,
                            const int32_t* tiekey, int32_t nclips, const double* q1, const double* q2,
                            const int64_t* qoff, int32_t nq, int coefs, double tolerance, int low, int high,
                            int32_t* winner, int32_t* match_count, int nthreads);

/* The same search, organised per distinct max1 box (oracle_boxes.c): for wide coefs = 2 windows at
 * configs[2] size, where one row scan per frame box would read tens of millions of rows per frame.
 * Same arguments and results as tfo_search_sorted_batch (rows sorted by max1); mode 0 picks the
 * cheaper form per (query, box), 1 forces the max2-ordered runs, 2 the per-clip merges (tests). */
int tfo_search_boxes_batch(const int32_t* m1s, const int32_t* m2s, const int32_t* row_clip, int64_t nrows,
                           const int32_t* tiekey, int32_t nclips, const double* q1, const double* q2,
                           const int64_t* qoff, int32_t nq, int coefs, double tolerance, int low, int high,
                           int32_t* winner, int32_t* match_count, int nthreads, int mode);

/* One query frame's WHERE clause (fp_handler.c:287-351): 0 = the frame runs no SQL; else [L1, U1]
 * on max1 and, when *has2, [L2, U2] on max2, in micro-units. */
int tfo_frame_box(double q1v, double q2v, int coefs, double tole, int low, int high, int64_t* L1, int64_t* U1,
                  int* has2, int64_t* L2, int64_t* U2);

/* printf("%f") micro-units of x, parsed from the printed string. */
int64_t tfo_fmt6(double x);

#endif
