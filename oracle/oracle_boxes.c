/* oracle_boxes.c — CPU ORACLE (test infrastructure only; never linked into the product).
 *
 * fp_search_fingerprint_info's per-frame SQL (/root/reference/src/fp_handler.c:308-359) and its
 * scoring (:367-374) over an audio_fingerprint table sorted by max1, organised per distinct max1
 * box. Same semantics as tfo_search_sorted_batch (oracle.c), which scans every row of a frame's
 * max1 box once per distinct frame clause: at configs[2] size a coefs = 2 batch at a wide
 * tolerance gives every frame its own clause over a box of tens of millions of rows, too slow to
 * check a full-size batch with. Here each distinct box (L1, U1) of the batch is gathered once:
 *   - the clips with any row in it (a frame without a max2 condition adds 1 to each),
 *   - its rows with a non-NULL max2 sorted by max2 (a narrow max2 window is a short run of them),
 *   - the same rows grouped per clip, each group's max2 values ascending (a wide window: per clip,
 *     the frames sorted by their window start meet the clip's sorted values in one merge).
 * Per (query, box) the cheaper of the two is taken; both count, per frame, 1 for every clip with
 * a row inside the frame's box (GROUP BY audio_uuid, :353) and nothing for NULL max2 rows under a
 * max2 condition (NULL compares false). tests/test_oracle.py checks this against the brute-force
 * tfo_search and the SQLite goldens.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "tfp_oracle.h"

typedef struct {
  int64_t L1, U1;
  int32_t nclip;        /* clips with any row in the box */
  int32_t* clip;
  int64_t npts;         /* rows with non-NULL max2 */
  int32_t* bym2_v;      /* their max2, ascending */
  int32_t* bym2_c;      /* ... and clip */
  int32_t ngroup;       /* clips with a non-NULL max2 row */
  int32_t* gclip;
  int64_t* gbeg;        /* [ngroup + 1] into pts */
  int32_t* pts;         /* max2 per clip, ascending */
} obox;

static int64_t lb32(const int32_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = lo + ((hi - lo) >> 1);
    if ((int64_t)a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

/* stable LSD radix sort of (v, c) pairs by v (signed) */
static int sort_pairs(int32_t* v, int32_t* c, int64_t n) {
  uint32_t* ka = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n ? n : 1));
  uint32_t* kb = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n ? n : 1));
  int32_t* ca = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  int32_t* cb = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  int64_t* cnt = (int64_t*)malloc(sizeof(int64_t) * 65537);
  int64_t i;
  int pass;
  if (!ka || !kb || !ca || !cb || !cnt) { free(ka); free(kb); free(ca); free(cb); free(cnt); return -1; }
  for (i = 0; i < n; i++) { ka[i] = (uint32_t)v[i] ^ 0x80000000u; ca[i] = c[i]; }
  for (pass = 0; pass < 2; pass++) {
    int sh = 16 * pass, d;
    uint32_t* tk;
    int32_t* tc;
    memset(cnt, 0, sizeof(int64_t) * 65537);
    for (i = 0; i < n; i++) cnt[((ka[i] >> sh) & 65535) + 1]++;
    for (d = 0; d < 65536; d++) cnt[d + 1] += cnt[d];
    for (i = 0; i < n; i++) {
      int64_t o = cnt[(ka[i] >> sh) & 65535]++;
      kb[o] = ka[i];
      cb[o] = ca[i];
    }
    tk = ka; ka = kb; kb = tk;
    tc = ca; ca = cb; cb = tc;
  }
  for (i = 0; i < n; i++) { v[i] = (int32_t)(ka[i] ^ 0x80000000u); c[i] = ca[i]; }
  free(ka); free(kb); free(ca); free(cb); free(cnt);
  return 0;
}

typedef struct {
  const int32_t *m1s, *m2s, *clip;
  int64_t nrows;
  int32_t nclips;
  obox* boxes;
  int32_t nbox, tid, nthreads, status;
} build_arg;

static int build_box(const build_arg* a, obox* b) {
  const int64_t lo = lb32(a->m1s, a->nrows, b->L1), hi = lb32(a->m1s, a->nrows, b->U1 + 1);
  uint8_t* seen = (uint8_t*)calloc((size_t)(a->nclips > 0 ? a->nclips : 1), 1);
  int64_t* cnt = (int64_t*)calloc((size_t)a->nclips + 1, sizeof(int64_t));
  int64_t r, n = 0;
  int32_t c;
  if (!seen || !cnt) { free(seen); free(cnt); return -1; }
  b->bym2_v = (int32_t*)malloc(sizeof(int32_t) * (size_t)(hi - lo + 1));
  b->bym2_c = (int32_t*)malloc(sizeof(int32_t) * (size_t)(hi - lo + 1));
  if (!b->bym2_v || !b->bym2_c) { free(seen); free(cnt); return -1; }
  b->nclip = 0;
  for (r = lo; r < hi; r++) {
    if (a->m1s[r] == TFO_NULL) continue; /* NULL compares false */
    c = a->clip[r];
    seen[c] = 1;
    if (a->m2s[r] == TFO_NULL) continue;
    b->bym2_v[n] = a->m2s[r];
    b->bym2_c[n] = c;
    n++;
  }
  b->npts = n;
  for (c = 0; c < a->nclips; c++) b->nclip += seen[c];
  b->clip = (int32_t*)malloc(sizeof(int32_t) * (size_t)(b->nclip + 1));
  if (!b->clip) { free(seen); free(cnt); return -1; }
  b->nclip = 0;
  for (c = 0; c < a->nclips; c++)
    if (seen[c]) b->clip[b->nclip++] = c;
  if (sort_pairs(b->bym2_v, b->bym2_c, n)) { free(seen); free(cnt); return -1; }
  /* stable counting sort by clip: groups of ascending max2 */
  for (r = 0; r < n; r++) cnt[b->bym2_c[r] + 1]++;
  b->ngroup = 0;
  for (c = 0; c < a->nclips; c++) b->ngroup += cnt[c + 1] > 0;
  b->gclip = (int32_t*)malloc(sizeof(int32_t) * (size_t)(b->ngroup + 1));
  b->gbeg = (int64_t*)malloc(sizeof(int64_t) * (size_t)(b->ngroup + 1));
  b->pts = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
  if (!b->gclip || !b->gbeg || !b->pts) { free(seen); free(cnt); return -1; }
  {
    int32_t g = 0;
    int64_t at = 0;
    for (c = 0; c < a->nclips; c++) {
      const int64_t k = cnt[c + 1];
      cnt[c + 1] = at; /* cnt[c + 1] := the clip's first slot */
      if (k) { b->gclip[g] = c; b->gbeg[g] = at; g++; }
      at += k;
    }
    b->gbeg[g] = at;
  }
  for (r = 0; r < n; r++) b->pts[cnt[b->bym2_c[r] + 1]++] = b->bym2_v[r];
  free(seen);
  free(cnt);
  return 0;
}

static void* build_worker(void* p) {
  build_arg* a = (build_arg*)p;
  int32_t i;
  for (i = a->tid; i < a->nbox; i += a->nthreads)
    if (build_box(a, &a->boxes[i])) a->status = -1;
  return NULL;
}

typedef struct {
  int64_t L1, U1, L2, U2;
  int has2;
  int32_t box;
} fbox;

static int fbox_cmp(const void* x, const void* y) {
  const fbox *a = (const fbox*)x, *b = (const fbox*)y;
  if (a->box != b->box) return a->box < b->box ? -1 : 1;
  if (a->has2 != b->has2) return a->has2 < b->has2 ? -1 : 1;
  if (a->L2 != b->L2) return a->L2 < b->L2 ? -1 : 1;
  if (a->U2 != b->U2) return a->U2 < b->U2 ? -1 : 1;
  return 0;
}

typedef struct {
  const obox* boxes;
  int32_t nbox, nclips;
  const int32_t* tiekey;
  const double *q1, *q2;
  const int64_t* qoff;
  int32_t nq, coefs, low, high, tid, nthreads, mode;
  double tole;
  int32_t *winner, *count;
} query_arg;

static int32_t find_box(const obox* boxes, int32_t n, int64_t L1, int64_t U1) {
  int32_t lo = 0, hi = n - 1;
  while (lo <= hi) {
    int32_t mid = (lo + hi) >> 1;
    const obox* b = &boxes[mid];
    if (b->L1 == L1 && b->U1 == U1) return mid;
    if (b->L1 < L1 || (b->L1 == L1 && b->U1 < U1)) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

static void* query_worker(void* p) {
  query_arg* a = (query_arg*)p;
  const int32_t nc = a->nclips > 0 ? a->nclips : 1;
  int32_t* score = (int32_t*)calloc((size_t)nc, sizeof(int32_t));
  int32_t* stamp = (int32_t*)calloc((size_t)nc, sizeof(int32_t));
  int32_t* touched = (int32_t*)malloc(sizeof(int32_t) * (size_t)nc);
  fbox* fb = NULL;
  int64_t cap = 0;
  int32_t epoch = 0, q;
  for (q = a->tid; q < a->nq; q += a->nthreads) {
    int64_t f, nb = 0, i, j;
    int32_t nt = 0, best = -1, k;
#define ADD(c, v)                                  \
  do {                                             \
    if (v) {                                       \
      if (!score[c]) touched[nt++] = (c);          \
      score[c] += (v);                             \
    }                                              \
  } while (0)
    if (a->qoff[q + 1] - a->qoff[q] > cap) {
      cap = a->qoff[q + 1] - a->qoff[q];
      fb = (fbox*)realloc(fb, sizeof(fbox) * (size_t)cap);
    }
    for (f = a->qoff[q]; f < a->qoff[q + 1]; f++) {
      fbox b;
      memset(&b, 0, sizeof b);
      if (!tfo_frame_box(a->q1[f], a->q2[f], a->coefs, a->tole, a->low, a->high, &b.L1, &b.U1, &b.has2, &b.L2, &b.U2))
        continue;
      b.box = find_box(a->boxes, a->nbox, b.L1, b.U1);
      fb[nb++] = b;
    }
    if (nb > 1) qsort(fb, (size_t)nb, sizeof(fbox), fbox_cmp);
    for (i = 0; i < nb; i = j) {
      const obox* B = &a->boxes[fb[i].box];
      int64_t n0 = 0, h, costA = 0, costB;
      for (j = i; j < nb && fb[j].box == fb[i].box; j++) n0 += !fb[j].has2;
      for (k = 0; n0 && k < B->nclip; k++) ADD(B->clip[k], (int32_t)n0);
      h = i + n0; /* the frames with a max2 condition: fb[h..j), sorted by (L2, U2) */
      if (h == j) continue;
      for (f = h; f < j; f++) costA += lb32(B->bym2_v, B->npts, fb[f].U2 + 1) - lb32(B->bym2_v, B->npts, fb[f].L2);
      costB = B->npts + (int64_t)B->ngroup * (j - h);
      if (a->mode == 1 || (a->mode == 0 && costA <= costB)) { /* each frame's run of max2 values, one count per clip */
        for (f = h; f < j; f++) {
          const int64_t e = lb32(B->bym2_v, B->npts, fb[f].U2 + 1);
          int64_t r;
          epoch++;
          for (r = lb32(B->bym2_v, B->npts, fb[f].L2); r < e; r++) {
            const int32_t c = B->bym2_c[r];
            if (stamp[c] != epoch) { stamp[c] = epoch; ADD(c, 1); }
          }
        }
      } else { /* per clip: its ascending values against the frames in window-start order */
        int32_t g;
        for (g = 0; g < B->ngroup; g++) {
          int64_t pp = B->gbeg[g];
          const int64_t pe = B->gbeg[g + 1];
          int32_t cnt = 0;
          for (f = h; f < j; f++) {
            while (pp < pe && B->pts[pp] < fb[f].L2) pp++;
            if (pp == pe) break;
            cnt += B->pts[pp] <= fb[f].U2;
          }
          ADD(B->gclip[g], cnt);
        }
      }
    }
#undef ADD
    for (k = 0; k < nt; k++) { /* max count, ties to the greatest uuid (tiekey = uuid rank) */
      const int32_t c = touched[k];
      if (best < 0 || score[c] > score[best] || (score[c] == score[best] && a->tiekey[c] > a->tiekey[best])) best = c;
    }
    a->winner[q] = best;
    a->count[q] = best >= 0 ? score[best] : 0;
    for (k = 0; k < nt; k++) score[touched[k]] = 0;
  }
  free(fb); free(score); free(stamp); free(touched);
  return NULL;
}

static int obox_cmp(const void* x, const void* y) {
  const obox *a = (const obox*)x, *b = (const obox*)y;
  if (a->L1 != b->L1) return a->L1 < b->L1 ? -1 : 1;
  if (a->U1 != b->U1) return a->U1 < b->U1 ? -1 : 1;
  return 0;
}

int tfo_search_boxes_batch(const int32_t* m1s, const int32_t* m2s, const int32_t* row_clip, int64_t nrows,
                           const int32_t* tiekey, int32_t nclips, const double* q1, const double* q2,
                           const int64_t* qoff, int32_t nq, int coefs, double tolerance, int low, int high,
                           int32_t* winner, int32_t* match_count, int nthreads, int mode) {
  const double tole = tolerance < 0 ? 0.001 : tolerance; /* fp_handler.c:252-256 */
  obox* boxes = NULL;
  int32_t nbox = 0, i;
  int64_t f, nf = nq ? qoff[nq] - qoff[0] : 0;
  int rc = 0;
  if (coefs < 1 || coefs > TFO_COEFS) { /* fp_handler.c:247-250 */
    for (i = 0; i < nq; i++) { winner[i] = -1; match_count[i] = 0; }
    return 0;
  }
  if (nthreads < 1) nthreads = 1;
  /* the batch's distinct max1 boxes */
  boxes = (obox*)calloc((size_t)(nf + 1), sizeof(obox));
  if (!boxes) return -1;
  for (f = qoff[0]; f < qoff[0] + nf; f++) {
    int64_t L1, U1, L2, U2;
    int has2;
    if (!tfo_frame_box(q1[f], q2[f], coefs, tole, low, high, &L1, &U1, &has2, &L2, &U2)) continue;
    boxes[nbox].L1 = L1;
    boxes[nbox].U1 = U1;
    nbox++;
  }
  if (nbox > 1) qsort(boxes, (size_t)nbox, sizeof(obox), obox_cmp);
  {
    int32_t w = 0;
    for (i = 0; i < nbox; i++)
      if (!w || obox_cmp(&boxes[w - 1], &boxes[i]) != 0) boxes[w++] = boxes[i];
    nbox = w;
  }
  {
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    build_arg* ba = (build_arg*)malloc(sizeof(build_arg) * (size_t)nthreads);
    query_arg* qa = (query_arg*)malloc(sizeof(query_arg) * (size_t)nthreads);
    for (i = 0; i < nthreads; i++) {
      build_arg b = {m1s, m2s, row_clip, nrows, nclips, boxes, nbox, i, nthreads, 0};
      ba[i] = b;
      pthread_create(&th[i], NULL, build_worker, &ba[i]);
    }
    for (i = 0; i < nthreads; i++) {
      pthread_join(th[i], NULL);
      rc |= ba[i].status;
    }
    if (!rc) {
      for (i = 0; i < nthreads; i++) {
        query_arg q = {boxes, nbox, nclips, tiekey, q1, q2, qoff, nq, coefs, low, high, i, nthreads, mode, tole,
                       winner, match_count};
        qa[i] = q;
        pthread_create(&th[i], NULL, query_worker, &qa[i]);
      }
      for (i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    }
    free(th); free(ba); free(qa);
  }
  for (i = 0; i < nbox; i++) {
    free(boxes[i].clip); free(boxes[i].bym2_v); free(boxes[i].bym2_c);
    free(boxes[i].gclip); free(boxes[i].gbeg); free(boxes[i].pts);
  }
  free(boxes);
  return rc;
}
