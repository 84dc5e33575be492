/* TEST HARNESS (tests/test_shim.py; not product code): the Asterisk side that shim/
 * fp_handler_tfp.c + shim/fp_catalog.c run against outside Asterisk — a minimal ast_json and
 * ast_log — and a driver that plays the module's calls from the command line: the dialplan
 * application's search (application_handler.c:180-236), the CLI's context / audio commands
 * (cli_handler.c) and app_tiresias.c's directory enrolment (:365-424, scandir + alphasort):
 *   shim_driver BACKUP_DB CMD...   with CMD one of
 *     init | term | enroll CONTEXT FILE | enrolldir CONTEXT DIR | enrolldir1 CONTEXT DIR |
 *     delete UUID | search CONTEXT FILE COEFS TOL LOW HIGH | ctx NAME DIR | ctxdel NAME |
 *     lists | hash FILE | devices LIST |
 *     psearch NTHREADS REPS CONTEXT COEFS TOL LOW HIGH NFILES FILE... |
 *     chan CONTEXT FILE CHUNK MAXMS COEFS TOL LOW HIGH | cthreads NTHREADS ITERS NFILES FILE...
 * chan plays the record loop (application_handler.c:248-312) on a live channel (fp_channel_*): the
 * file's samples pushed CHUNK at a time (160 = one 20 ms SLIN frame), then searched.
 * psearch plays the module's channel threads: NTHREADS threads (application_handler.c:66, one per
 * call) each run REPS fp_search_fingerprint_info calls at once, thread t's r-th on file
 * (t * 7 + r) % NFILES, and print every result, the wall time and the coalescer's counts.
 * enrolldir batches the scan through fp_create_audio_list_infos, enrolldir1 calls
 * fp_craete_audio_list_info per file as the reference does. Each command prints one JSON line. */
#define _GNU_SOURCE
#include <dirent.h>
#include <inttypes.h>
#include <pthread.h>
#include <time.h>
#include <stdarg.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "asterisk/json.h"
#include "asterisk/logger.h"
#include "fp_catalog.h"
#include "fp_handler_tfp.h"
#include "tiresias_fp.h"

/* ---- ast_json: object / array / integer / real / string / null ---- */
enum { J_OBJ, J_INT, J_STR, J_ARR, J_REAL, J_NULL };
struct ast_json {
  int type;
  intmax_t i;
  double d;
  char* s;
  int n, cap;
  char** keys;
  struct ast_json** vals;
};
static struct ast_json* jnew(int type) {
  struct ast_json* j = calloc(1, sizeof *j);
  j->type = type;
  return j;
}
static void jpush(struct ast_json* o, char* k, struct ast_json* v) {
  if (o->n == o->cap) {
    o->cap = o->cap ? 2 * o->cap : 8;
    o->keys = realloc(o->keys, sizeof(char*) * o->cap);
    o->vals = realloc(o->vals, sizeof(struct ast_json*) * o->cap);
  }
  o->keys[o->n] = k;
  o->vals[o->n++] = v;
}
struct ast_json* ast_json_object_create(void) { return jnew(J_OBJ); }
struct ast_json* ast_json_array_create(void) { return jnew(J_ARR); }
struct ast_json* ast_json_null(void) { return jnew(J_NULL); }
struct ast_json* ast_json_integer_create(intmax_t v) {
  struct ast_json* j = jnew(J_INT);
  j->i = v;
  return j;
}
struct ast_json* ast_json_real_create(double v) {
  struct ast_json* j = jnew(J_REAL);
  j->d = v;
  return j;
}
struct ast_json* ast_json_string_create(const char* s) {
  struct ast_json* j = jnew(J_STR);
  j->s = strdup(s);
  return j;
}
int ast_json_object_set(struct ast_json* o, const char* k, struct ast_json* v) {
  if (!o || o->type != J_OBJ) { ast_json_unref(v); return -1; }
  jpush(o, strdup(k), v);
  return 0;
}
struct ast_json* ast_json_object_get(struct ast_json* o, const char* k) {
  int i;
  for (i = 0; o && o->type == J_OBJ && i < o->n; i++)
    if (!strcmp(o->keys[i], k)) return o->vals[i];
  return NULL;
}
int ast_json_array_append(struct ast_json* a, struct ast_json* v) {
  if (!a || a->type != J_ARR) { ast_json_unref(v); return -1; }
  jpush(a, NULL, v);
  return 0;
}
size_t ast_json_array_size(const struct ast_json* a) { return a && a->type == J_ARR ? (size_t)a->n : 0; }
struct ast_json* ast_json_array_get(const struct ast_json* a, size_t i) {
  return a && a->type == J_ARR && i < (size_t)a->n ? a->vals[i] : NULL;
}
intmax_t ast_json_integer_get(const struct ast_json* v) { return v && v->type == J_INT ? v->i : 0; }
double ast_json_real_get(const struct ast_json* v) { return v && v->type == J_REAL ? v->d : 0.0; }
const char* ast_json_string_get(const struct ast_json* v) { return v && v->type == J_STR ? v->s : NULL; }
void ast_json_unref(struct ast_json* v) {
  int i;
  if (!v) return;
  for (i = 0; i < v->n; i++) { free(v->keys[i]); ast_json_unref(v->vals[i]); }
  free(v->keys);
  free(v->vals);
  free(v->s);
  free(v);
}
/* ast_json_load_string: a small JSON reader (objects, arrays, strings with the common escapes,
 * numbers, true / false / null); as jansson with flags 0, only an array or object at the top. */
static const char* jws(const char* p) {
  while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r') p++;
  return p;
}
static struct ast_json* jparse(const char** pp);
static char* jstr(const char** pp) {
  const char* p = *pp + 1;
  char* out = malloc(strlen(p) + 1);
  size_t n = 0;
  while (*p && *p != '"') {
    if (*p == '\\') {
      p++;
      switch (*p) {
        case 'n': out[n++] = '\n'; break;
        case 't': out[n++] = '\t'; break;
        case '"': case '\\': case '/': out[n++] = *p; break;
        default: free(out); return NULL;
      }
      p++;
    } else {
      out[n++] = *p++;
    }
  }
  if (*p != '"') { free(out); return NULL; }
  out[n] = 0;
  *pp = p + 1;
  return out;
}
static struct ast_json* jparse(const char** pp) {
  const char* p = jws(*pp);
  struct ast_json* j = NULL;
  if (*p == '{' || *p == '[') {
    const int obj = *p == '{';
    j = jnew(obj ? J_OBJ : J_ARR);
    p = jws(p + 1);
    if (*p == (obj ? '}' : ']')) { *pp = p + 1; return j; }
    for (;;) {
      char* k = NULL;
      struct ast_json* v;
      if (obj) {
        if (*p != '"' || !(k = jstr(&p))) break;
        p = jws(p);
        if (*p != ':') { free(k); break; }
        p++;
      }
      if (!(v = jparse(&p))) { free(k); break; }
      jpush(j, k, v);
      p = jws(p);
      if (*p == ',') { p = jws(p + 1); continue; }
      if (*p == (obj ? '}' : ']')) { *pp = p + 1; return j; }
      break;
    }
    ast_json_unref(j);
    return NULL;
  }
  if (*p == '"') {
    char* s = jstr(&p);
    if (!s) return NULL;
    j = jnew(J_STR);
    j->s = s;
  } else if (!strncmp(p, "true", 4) || !strncmp(p, "false", 5) || !strncmp(p, "null", 4)) {
    j = *p == 'n' ? jnew(J_NULL) : ast_json_integer_create(*p == 't');
    p += *p == 'f' ? 5 : 4;
  } else {
    char* e;
    const double d = strtod(p, &e);
    if (e == p) return NULL;
    j = ast_json_real_create(d);
    p = e;
  }
  *pp = p;
  return j;
}
struct ast_json* ast_json_load_string(const char* input, struct ast_json_error* error) {
  const char* p;
  struct ast_json* j;
  (void)error;
  if (!input) return NULL;
  p = jws(input);
  if (*p != '{' && *p != '[') return NULL;
  j = jparse(&p);
  if (j && *jws(p) != 0) { ast_json_unref(j); return NULL; }
  return j;
}
enum ast_json_type ast_json_typeof(const struct ast_json* v) {
  switch (v->type) {
    case J_OBJ: return AST_JSON_OBJECT;
    case J_ARR: return AST_JSON_ARRAY;
    case J_STR: return AST_JSON_STRING;
    case J_INT: return AST_JSON_INTEGER;
    case J_REAL: return AST_JSON_REAL;
    default: return AST_JSON_NULL;
  }
}

static void jprint(const struct ast_json* j) {
  int i;
  if (!j) { printf("null"); return; }
  switch (j->type) {
    case J_INT: printf("%jd", j->i); break;
    case J_REAL: printf("%.17g", j->d); break;
    case J_STR: {
      const char* c;
      putchar('"');
      for (c = j->s; *c; c++) {
        if (*c == '"' || *c == '\\') putchar('\\');
        if (*c == '\n') { printf("\\n"); continue; }
        putchar(*c);
      }
      putchar('"');
      break;
    }
    case J_NULL: printf("null"); break;
    case J_ARR:
      printf("[");
      for (i = 0; i < j->n; i++) { if (i) printf(", "); jprint(j->vals[i]); }
      printf("]");
      break;
    default:
      printf("{");
      for (i = 0; i < j->n; i++) { if (i) printf(", "); printf("\"%s\": ", j->keys[i]); jprint(j->vals[i]); }
      printf("}");
  }
}
void ast_log(int level, const char* file, int line, const char* function, const char* fmt, ...) {
  va_list ap;
  fprintf(stderr, "[%d] %s:%d %s: ", level, file, line, function);
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
}

/* ---- driver: application_handler.c:180-236's use of the result ---- */
static void print_search(const char* file, struct ast_json* j) {
  if (!j) {
    printf("{\"file\": \"%s\", \"TIRSTATUS\": \"NOTFOUND\"}\n", file);
    return;
  }
  printf("{\"file\": \"%s\", \"TIRSTATUS\": \"FOUND\", \"TIRFRAMECOUNT\": %d, \"TIRMATCHCOUNT\": %d, "
         "\"TIRFILEUUID\": \"%s\", \"TIRFILENAME\": \"%s\", \"TIRCONTEXT\": \"%s\", \"TIRFILEHASH\": \"%s\"}\n",
         file, (int)ast_json_integer_get(ast_json_object_get(j, "frame_count")),
         (int)ast_json_integer_get(ast_json_object_get(j, "match_count")),
         ast_json_string_get(ast_json_object_get(j, "uuid")), ast_json_string_get(ast_json_object_get(j, "name")),
         ast_json_string_get(ast_json_object_get(j, "context")), ast_json_string_get(ast_json_object_get(j, "hash")));
  ast_json_unref(j);
}

/* ---- psearch: concurrent channel threads ---- */
typedef struct {
  int found, fc, mc;
  char uuid[64];
} psres;
typedef struct {
  int t, reps, nfiles, coefs, low, high;
  double tol;
  const char* ctx;
  char** files;
  psres* out;  /* [reps] */
  pthread_barrier_t* go;
} psarg;

static void* psearch_thread(void* p) {
  psarg* a = p;
  int r;
  pthread_barrier_wait(a->go);
  for (r = 0; r < a->reps; r++) {
    struct ast_json* j = fp_search_fingerprint_info(a->ctx, a->files[(a->t * 7 + r) % a->nfiles], a->coefs, a->tol,
                                                    a->low, a->high);
    psres* o = &a->out[r];
    memset(o, 0, sizeof *o);
    if (j) {
      o->found = 1;
      o->fc = (int)ast_json_integer_get(ast_json_object_get(j, "frame_count"));
      o->mc = (int)ast_json_integer_get(ast_json_object_get(j, "match_count"));
      snprintf(o->uuid, sizeof o->uuid, "%s", ast_json_string_get(ast_json_object_get(j, "uuid")));
      ast_json_unref(j);
    }
  }
  return NULL;
}

static void psearch(int nth, int reps, const char* ctx, int coefs, double tol, int low, int high, int nfiles,
                    char** files) {
  pthread_t* th = calloc(nth, sizeof *th);
  psarg* args = calloc(nth, sizeof *args);
  psres* out = calloc((size_t)nth * reps, sizeof *out);
  pthread_barrier_t go;
  struct timespec t0, t1;
  int64_t c0 = 0, b0 = 0, c1 = 0, b1 = 0;
  int t, r;
  pthread_barrier_init(&go, NULL, nth + 1);
  fp_get_search_stats(&c0, &b0);
  for (t = 0; t < nth; t++) {
    psarg a = {t, reps, nfiles, coefs, low, high, tol, ctx, files, out + (size_t)t * reps, &go};
    args[t] = a;
    pthread_create(&th[t], NULL, psearch_thread, &args[t]);
  }
  clock_gettime(CLOCK_MONOTONIC, &t0);
  pthread_barrier_wait(&go);
  for (t = 0; t < nth; t++) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  fp_get_search_stats(&c1, &b1);
  {
    const double s = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    printf("{\"psearch\": %d, \"reps\": %d, \"seconds\": %.6f, \"per_s\": %.1f, \"calls\": %" PRId64
           ", \"batches\": %" PRId64 ", \"results\": [", nth, reps, s, nth * reps / s, c1 - c0, b1 - b0);
  }
  for (t = 0; t < nth; t++)
    for (r = 0; r < reps; r++) {
      const psres* o = &out[(size_t)t * reps + r];
      printf("%s[%d, %d, \"%s\", %d, %d]", t || r ? ", " : "", (t * 7 + r) % nfiles, o->found, o->uuid, o->mc, o->fc);
    }
  printf("]}\n");
  pthread_barrier_destroy(&go);
  free(th);
  free(args);
  free(out);
}

/* ---- cthreads: the catalog from many threads (tests/test_sanitizers.py, under TSan / ASan) ----
 * thread t, iteration i: file (t + i) % NFILES into context "ctx": create (dedup: of threads racing
 * on one file exactly one creates it), store rows, read the row and the lists back, delete. */
typedef struct {
  int t, iters, nfiles;
  char** files;
  int created, dup;
} cthr;

static void* cthread_main(void* v) {
  cthr* a = v;
  int i;
  for (i = 0; i < a->iters; i++) {
    char* uuid = fp_generate_uuid();
    int32_t m1[3] = {1000000 + i, INT32_MIN, -5}, m2[3] = {a->t, 7, INT32_MIN};
    int ret;
    if (uuid == NULL) continue;
    ret = fpc_create_audio_list_info("ctx", a->files[(a->t + i) % a->nfiles], uuid);
    if (ret == 1) {
      struct ast_json* j;
      a->created++;
      fpc_store_fingerprints("ctx", uuid, m1, m2, 3);
      j = fpc_get_audio_list_info(uuid);
      ast_json_unref(j);
      j = fp_get_audio_lists_all();
      ast_json_unref(j);
      fpc_delete_audio_list_info(uuid);
    } else if (ret == 0) {
      a->dup++;
    }
    free(uuid);
  }
  return NULL;
}

static void cthreads(int nth, int iters, int nfiles, char** files) {
  pthread_t* th = calloc(nth, sizeof *th);
  cthr* a = calloc(nth, sizeof *a);
  int t, created = 0, dup = 0;
  for (t = 0; t < nth; t++) {
    a[t].t = t;
    a[t].iters = iters;
    a[t].nfiles = nfiles;
    a[t].files = files;
    pthread_create(&th[t], NULL, cthread_main, &a[t]);
  }
  for (t = 0; t < nth; t++) {
    pthread_join(th[t], NULL);
    created += a[t].created;
    dup += a[t].dup;
  }
  printf("{\"cthreads\": %d, \"calls\": %d, \"created\": %d, \"dup\": %d}\n", nth, nth * iters, created, dup);
  free(th);
  free(a);
}

/* ---- chan: a live channel fed frame by frame ---- */
static void chan_search(const char* ctx, const char* file, int chunk, int max_ms, int coefs, double tol, int low,
                        int high) {
  int64_t n = 0, i;
  int32_t sr = 0;
  int16_t* pcm;
  fp_channel* ch;
  char label[600];
  snprintf(label, sizeof label, "chan:%s", file);
#ifdef SHIM_HARNESS_NO_ENGINE  /* (catalog_harness.c: no engine library linked) */
  (void)pcm; (void)ch; (void)i; (void)n; (void)chunk; (void)max_ms; (void)ctx; (void)coefs; (void)tol; (void)low;
  (void)high; (void)sr;
  print_search(label, NULL);
  return;
#else
  if (tfp_wav_read(file, NULL, 0, &n, &sr) != TFP_OK || chunk <= 0) {
    print_search(label, NULL);
    return;
  }
  pcm = malloc(sizeof(int16_t) * (size_t)(n ? n : 1));
  ch = fp_channel_open(sr, max_ms);
  if (!pcm || !ch || tfp_wav_read(file, pcm, n, &n, &sr) != TFP_OK) {
    free(pcm);
    fp_channel_close(ch);
    print_search(label, NULL);
    return;
  }
  fp_channel_push(ch, pcm, 7);  /* a previous call's audio, dropped by the reset below */
  fp_channel_reset(ch);
  for (i = 0; i < n; i += chunk) fp_channel_push(ch, pcm + i, (int)(n - i < chunk ? n - i : chunk));
  print_search(label, fp_channel_search(ch, ctx, coefs, tol, low, high));
  fp_channel_close(ch);
  free(pcm);
#endif
}

static int file_select(const struct dirent* e) { return strcmp(e->d_name, ".") && strcmp(e->d_name, ".."); }

/* app_tiresias.c:365-424: the context's directory, alphasort; batched or file by file */
static void enroll_dir(const char* context, const char* dir, bool batched) {
  struct dirent** names;
  int n = scandir(dir, &names, file_select, alphasort), i, done = 0;
  char** paths;
  bool* ok;
  if (n < 0) { printf("{\"enrolldir\": \"%s\", \"ok\": false}\n", dir); return; }
  paths = calloc(n + 1, sizeof(char*));
  ok = calloc(n + 1, sizeof(bool));
  for (i = 0; i < n; i++) {
    if (asprintf(&paths[i], "%s/%s", dir, names[i]->d_name) < 0) paths[i] = NULL;
    free(names[i]);
  }
  free(names);
  if (batched) {
    done = fp_create_audio_list_infos(context, (const char* const*)paths, n, ok);
  } else {
    for (i = 0; i < n; i++) ok[i] = fp_craete_audio_list_info(context, paths[i]);
  }
  printf("{\"enrolldir\": \"%s\", \"batched\": %s, \"enrolled\": %d, \"ok\": [", dir, batched ? "true" : "false", done);
  for (i = 0; i < n; i++) printf("%s%s", i ? ", " : "", ok[i] ? "true" : "false");
  printf("]}\n");
  for (i = 0; i < n; i++) free(paths[i]);
  free(paths);
  free(ok);
}

int main(int argc, char** argv) {
  int i = 2;
  if (argc < 2) return 2;
  fpc_set_backup_path(argv[1]);
  while (i < argc) {
    const char* cmd = argv[i++];
    if (!strcmp(cmd, "init")) {
      printf("{\"init\": %s}\n", fp_init() ? "true" : "false");
    } else if (!strcmp(cmd, "term")) {
      printf("{\"term\": %s}\n", fp_term() ? "true" : "false");
    } else if (!strcmp(cmd, "enroll") && i + 1 < argc) {
      bool ok = fp_craete_audio_list_info(argv[i], argv[i + 1]);
      printf("{\"enroll\": \"%s\", \"ok\": %s}\n", argv[i + 1], ok ? "true" : "false");
      i += 2;
    } else if ((!strcmp(cmd, "enrolldir") || !strcmp(cmd, "enrolldir1")) && i + 1 < argc) {
      enroll_dir(argv[i], argv[i + 1], !strcmp(cmd, "enrolldir"));
      i += 2;
    } else if (!strcmp(cmd, "delete") && i < argc) {
      bool ok = fp_delete_audio_list_info(argv[i]);
      printf("{\"delete\": \"%s\", \"ok\": %s}\n", argv[i], ok ? "true" : "false");
      i += 1;
    } else if (!strcmp(cmd, "search") && i + 5 < argc) {
      const char* ctx = strcmp(argv[i], "NULL") ? argv[i] : NULL;
      print_search(argv[i + 1], fp_search_fingerprint_info(ctx, argv[i + 1], atoi(argv[i + 2]), atof(argv[i + 3]),
                                                           atoi(argv[i + 4]), atoi(argv[i + 5])));
      i += 6;
    } else if (!strcmp(cmd, "ctx") && i + 1 < argc) {
      bool ok = fp_create_context_list_info(argv[i], argv[i + 1], true);
      printf("{\"ctx\": \"%s\", \"ok\": %s}\n", argv[i], ok ? "true" : "false");
      i += 2;
    } else if (!strcmp(cmd, "ctxdel") && i < argc) {
      bool ok = fp_delete_context_list_info(argv[i]);
      printf("{\"ctxdel\": \"%s\", \"ok\": %s}\n", argv[i], ok ? "true" : "false");
      i += 1;
    } else if (!strcmp(cmd, "lists")) {
      struct ast_json* a = fp_get_audio_lists_all();
      struct ast_json* c = fp_get_context_lists_all();
      printf("{\"audio_lists\": ");
      jprint(a);
      printf(", \"context_lists\": ");
      jprint(c);
      printf("}\n");
      ast_json_unref(a);
      ast_json_unref(c);
    } else if (!strcmp(cmd, "hash") && i < argc) {
      char* h = fp_create_hash(argv[i]);
      printf("{\"hash\": \"%s\"}\n", h ? h : "");
      free(h);
      i += 1;
    } else if (!strcmp(cmd, "psearch") && i + 7 < argc && i + 8 + atoi(argv[i + 7]) <= argc) {
      const int nf = atoi(argv[i + 7]);
      const char* ctx = strcmp(argv[i + 2], "NULL") ? argv[i + 2] : NULL;
      psearch(atoi(argv[i]), atoi(argv[i + 1]), ctx, atoi(argv[i + 3]), atof(argv[i + 4]), atoi(argv[i + 5]),
              atoi(argv[i + 6]), nf, argv + i + 8);
      i += 8 + nf;
    } else if (!strcmp(cmd, "cthreads") && i + 2 < argc && i + 3 + atoi(argv[i + 2]) <= argc) {
      const int nf = atoi(argv[i + 2]);
      cthreads(atoi(argv[i]), atoi(argv[i + 1]), nf, argv + i + 3);
      i += 3 + nf;
    } else if (!strcmp(cmd, "chan") && i + 7 < argc) {
      chan_search(argv[i], argv[i + 1], atoi(argv[i + 2]), atoi(argv[i + 3]), atoi(argv[i + 4]), atof(argv[i + 5]),
                  atoi(argv[i + 6]), atoi(argv[i + 7]));
      i += 8;
    } else if (!strcmp(cmd, "devices") && i < argc) {
      fp_set_gpu_devices(argv[i]);
      printf("{\"devices\": \"%s\"}\n", argv[i]);
      i += 1;
    } else {
      fprintf(stderr, "bad command %s\n", cmd);
      return 2;
    }
    fflush(stdout);
  }
  return 0;
}
