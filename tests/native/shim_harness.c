/* TEST HARNESS (tests/test_shim.py; not product code): the Asterisk side that shim/
 * fp_handler_tfp.c runs against outside Asterisk — a minimal ast_json and ast_log, an in-memory
 * catalog behind shim/fp_catalog.h (audio_list + audio_fingerprint, with a snapshot file standing
 * in for the SQLite backup that fp_term writes and fp_init restores), and a driver that plays the
 * dialplan application's calls (application_handler.c:180-236) from the command line:
 *   shim_driver SNAPSHOT CMD...   with CMD one of
 *     init | term | enroll CONTEXT FILE | delete UUID | search CONTEXT FILE COEFS TOL LOW HIGH
 * Each search prints one JSON line: the channel variables TIRSTATUS ... TIRFILEHASH. */
#define _GNU_SOURCE
#include <inttypes.h>
#include <stdarg.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "asterisk/json.h"
#include "asterisk/logger.h"
#include "fp_catalog.h"

/* the facade (src/fp_handler.h:13-38) the shim implements */
bool fp_init(void);
bool fp_term(void);
bool fp_craete_audio_list_info(const char* context, const char* filename);
bool fp_delete_audio_list_info(const char* uuid);
struct ast_json* fp_search_fingerprint_info(const char* context, const char* filename, const int coefs,
                                            const double tolerance, const int freq_ignore_low,
                                            const int freq_ignore_high);

/* ---- ast_json ---- */
struct ast_json {
  int type; /* 0 object, 1 integer, 2 string */
  intmax_t i;
  char* s;
  int n;
  char* keys[16];
  struct ast_json* vals[16];
};
struct ast_json* ast_json_object_create(void) { return calloc(1, sizeof(struct ast_json)); }
struct ast_json* ast_json_integer_create(intmax_t v) {
  struct ast_json* j = calloc(1, sizeof *j);
  j->type = 1;
  j->i = v;
  return j;
}
struct ast_json* ast_json_string_create(const char* s) {
  struct ast_json* j = calloc(1, sizeof *j);
  j->type = 2;
  j->s = strdup(s);
  return j;
}
int ast_json_object_set(struct ast_json* o, const char* k, struct ast_json* v) {
  if (!o || o->type != 0 || o->n == 16) { ast_json_unref(v); return -1; }
  o->keys[o->n] = strdup(k);
  o->vals[o->n++] = v;
  return 0;
}
struct ast_json* ast_json_object_get(struct ast_json* o, const char* k) {
  int i;
  for (i = 0; o && i < o->n; i++)
    if (!strcmp(o->keys[i], k)) return o->vals[i];
  return NULL;
}
intmax_t ast_json_integer_get(const struct ast_json* v) { return v && v->type == 1 ? v->i : 0; }
const char* ast_json_string_get(const struct ast_json* v) { return v && v->type == 2 ? v->s : NULL; }
void ast_json_unref(struct ast_json* v) {
  int i;
  if (!v) return;
  for (i = 0; i < v->n; i++) { free(v->keys[i]); ast_json_unref(v->vals[i]); }
  free(v->s);
  free(v);
}
void ast_log(int level, const char* file, int line, const char* function, const char* fmt, ...) {
  va_list ap;
  fprintf(stderr, "[%d] %s:%d %s: ", level, file, line, function);
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
}

/* ---- catalog ---- */
typedef struct {
  char uuid[64], name[512], context[128];
  uint64_t hash;
  int64_t n;
  int32_t *m1, *m2;
  bool alive;
} clip_t;
static clip_t g_clips[4096];
static int g_nclips;
static const char* g_snapshot;
static int g_uuid_seq;

static uint64_t file_hash(const char* path) { /* stands in for the MD5 of fp_create_hash */
  FILE* f = fopen(path, "rb");
  uint64_t h = 1469598103934665603ull;
  int c;
  if (!f) return 0;
  while ((c = fgetc(f)) != EOF) h = (h ^ (uint64_t)(unsigned char)c) * 1099511628211ull;
  fclose(f);
  return h;
}
static clip_t* find(const char* uuid) {
  int i;
  for (i = 0; i < g_nclips; i++)
    if (g_clips[i].alive && !strcmp(g_clips[i].uuid, uuid)) return &g_clips[i];
  return NULL;
}
char* fp_generate_uuid(void) {
  char* s = malloc(40);
  snprintf(s, 40, "%08x-0000-4000-8000-%012d", (unsigned)(g_uuid_seq * 2654435761u), g_uuid_seq);
  g_uuid_seq++;
  return s;
}
bool fpc_db_init(void) { /* load the snapshot (the restored DB) */
  FILE* f = fopen(g_snapshot, "rb");
  int n, i;
  g_nclips = 0;
  if (!f) return true;
  if (fscanf(f, "%d %d\n", &n, &g_uuid_seq) != 2) { fclose(f); return false; }
  for (i = 0; i < n; i++) {
    clip_t* c = &g_clips[g_nclips++];
    int64_t k;
    memset(c, 0, sizeof *c);
    if (fscanf(f, "%63s %511s %127s %" SCNu64 " %" SCNd64 "\n", c->uuid, c->name, c->context, &c->hash, &c->n) != 5) {
      fclose(f);
      return false;
    }
    c->m1 = malloc(sizeof(int32_t) * (c->n + 1));
    c->m2 = malloc(sizeof(int32_t) * (c->n + 1));
    for (k = 0; k < c->n; k++)
      if (fscanf(f, "%" SCNd32 " %" SCNd32 "\n", &c->m1[k], &c->m2[k]) != 2) { fclose(f); return false; }
    c->alive = true;
  }
  fclose(f);
  return true;
}
bool fpc_db_term(void) { /* the backup */
  FILE* f = fopen(g_snapshot, "wb");
  int i, n = 0;
  int64_t k;
  if (!f) return false;
  for (i = 0; i < g_nclips; i++) n += g_clips[i].alive;
  fprintf(f, "%d %d\n", n, g_uuid_seq);
  for (i = 0; i < g_nclips; i++) {
    clip_t* c = &g_clips[i];
    if (!c->alive) continue;
    fprintf(f, "%s %s %s %" PRIu64 " %" PRId64 "\n", c->uuid, c->name, c->context, c->hash, c->n);
    for (k = 0; k < c->n; k++) fprintf(f, "%" PRId32 " %" PRId32 "\n", c->m1[k], c->m2[k]);
  }
  return fclose(f) == 0;
}
int fpc_create_audio_list_info(const char* context, const char* filename, const char* uuid) {
  uint64_t h = file_hash(filename);
  const char* base = strrchr(filename, '/');
  int i;
  if (!h) return -1;
  for (i = 0; i < g_nclips; i++)
    if (g_clips[i].alive && g_clips[i].hash == h && !strcmp(g_clips[i].context, context)) return 0;
  if (g_nclips == 4096) return -1;
  memset(&g_clips[g_nclips], 0, sizeof(clip_t));
  snprintf(g_clips[g_nclips].uuid, 64, "%s", uuid);
  snprintf(g_clips[g_nclips].name, 512, "%s", base ? base + 1 : filename);
  snprintf(g_clips[g_nclips].context, 128, "%s", context);
  g_clips[g_nclips].hash = h;
  g_clips[g_nclips++].alive = true;
  return 1;
}
struct ast_json* fpc_get_audio_list_info(const char* uuid) {
  clip_t* c = find(uuid);
  struct ast_json* j;
  char hs[32];
  if (!c) return NULL;
  j = ast_json_object_create();
  snprintf(hs, sizeof hs, "%016" PRIx64, c->hash);
  ast_json_object_set(j, "uuid", ast_json_string_create(c->uuid));
  ast_json_object_set(j, "name", ast_json_string_create(c->name));
  ast_json_object_set(j, "context", ast_json_string_create(c->context));
  ast_json_object_set(j, "hash", ast_json_string_create(hs));
  return j;
}
bool fpc_delete_audio_list_info(const char* uuid) {
  clip_t* c = find(uuid);
  if (!c) return false;
  c->alive = false;
  free(c->m1);
  free(c->m2);
  c->m1 = c->m2 = NULL;
  return true;
}
bool fpc_store_fingerprints(const char* context, const char* uuid, const int32_t* m1, const int32_t* m2, int64_t n) {
  clip_t* c = find(uuid);
  (void)context;
  if (!c) return false;
  c->m1 = malloc(sizeof(int32_t) * (n + 1));
  c->m2 = malloc(sizeof(int32_t) * (n + 1));
  memcpy(c->m1, m1, sizeof(int32_t) * n);
  memcpy(c->m2, m2, sizeof(int32_t) * n);
  c->n = n;
  return true;
}
bool fpc_for_each_fingerprint_clip(fpc_clip_rows_cb cb, void* arg) {
  int i;
  for (i = 0; i < g_nclips; i++)
    if (g_clips[i].alive && !cb(arg, g_clips[i].uuid, g_clips[i].m1, g_clips[i].m2, g_clips[i].n)) return false;
  return true;
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

int main(int argc, char** argv) {
  int i = 2;
  if (argc < 2) return 2;
  g_snapshot = argv[1];
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
    } else if (!strcmp(cmd, "delete") && i < argc) {
      bool ok = fp_delete_audio_list_info(argv[i]);
      printf("{\"delete\": \"%s\", \"ok\": %s}\n", argv[i], ok ? "true" : "false");
      i += 1;
    } else if (!strcmp(cmd, "search") && i + 5 < argc) {
      const char* ctx = strcmp(argv[i], "NULL") ? argv[i] : NULL;
      print_search(argv[i + 1], fp_search_fingerprint_info(ctx, argv[i + 1], atoi(argv[i + 2]), atof(argv[i + 3]),
                                                           atoi(argv[i + 4]), atoi(argv[i + 5])));
      i += 6;
    } else {
      fprintf(stderr, "bad command %s\n", cmd);
      return 2;
    }
    fflush(stdout);
  }
  return 0;
}
