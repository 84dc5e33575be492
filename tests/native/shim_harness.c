/* TEST HARNESS (tests/test_shim.py; not product code): the Asterisk side that shim/
 * fp_handler_tfp.c + shim/fp_catalog.c run against outside Asterisk — a minimal ast_json and
 * ast_log — and a driver that plays the module's calls from the command line: the dialplan
 * application's search (application_handler.c:180-236), the CLI's context / audio commands
 * (cli_handler.c) and app_tiresias.c's directory enrolment (:365-424, scandir + alphasort):
 *   shim_driver BACKUP_DB CMD...   with CMD one of
 *     init | term | enroll CONTEXT FILE | enrolldir CONTEXT DIR | enrolldir1 CONTEXT DIR |
 *     delete UUID | search CONTEXT FILE COEFS TOL LOW HIGH | ctx NAME DIR | ctxdel NAME |
 *     lists | hash FILE | devices LIST
 * enrolldir batches the scan through fp_create_audio_list_infos, enrolldir1 calls
 * fp_craete_audio_list_info per file as the reference does. Each command prints one JSON line. */
#define _GNU_SOURCE
#include <dirent.h>
#include <inttypes.h>
#include <stdarg.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "asterisk/json.h"
#include "asterisk/logger.h"
#include "fp_catalog.h"
#include "fp_handler_tfp.h"

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
static void jprint(const struct ast_json* j) {
  int i;
  if (!j) { printf("null"); return; }
  switch (j->type) {
    case J_INT: printf("%jd", j->i); break;
    case J_REAL: printf("%.17g", j->d); break;
    case J_STR: printf("\"%s\"", j->s); break;
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
