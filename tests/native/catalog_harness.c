/* TEST HARNESS (tests/test_catalog.py; not product code): shim/fp_catalog.c alone, on the CPU,
 * driven from the command line. Reuses shim_harness.c's ast_json / ast_log stubs by including it
 * with its main renamed; fp_delete_audio_list_info (the hot half's) is the catalog's own delete.
 *   catalog_driver BACKUP_DB CMD...   with CMD one of
 *     init | term | close | create CONTEXT FILE UUID | store CONTEXT UUID ROWS_BIN | load |
 *     delete UUID | ctx NAME DIR | ctxdel NAME | lists | hash FILE | uuid |
 *     cthreads NTHREADS ITERS NFILES FILE...  (the catalog from many threads, shim_harness.c)
 * ROWS_BIN: n int32 m1 values then n int32 m2 values. */
#define main shim_harness_main
#define SHIM_HARNESS_NO_ENGINE
#include "shim_harness.c"
#undef main

/* the shim's stand-ins: the catalog test needs no engine */
bool fp_init(void) { return false; }
bool fp_term(void) { return false; }
bool fp_craete_audio_list_info(const char* c, const char* f) { (void)c; (void)f; return false; }
int fp_create_audio_list_infos(const char* c, const char* const* f, int n, bool* ok) {
  (void)c; (void)f; (void)n; (void)ok;
  return -1;
}
struct ast_json* fp_search_fingerprint_info(const char* c, const char* f, const int co, const double t, const int l,
                                            const int h) {
  (void)c; (void)f; (void)co; (void)t; (void)l; (void)h;
  return NULL;
}
bool fp_delete_audio_list_info(const char* uuid) { return fpc_delete_audio_list_info(uuid); }
void fp_set_gpu_devices(const char* list) { (void)list; }
fp_channel* fp_channel_open(int sr, int ms) {
  (void)sr; (void)ms;
  return NULL;
}
bool fp_channel_push(fp_channel* ch, const int16_t* s, int n) {
  (void)ch; (void)s; (void)n;
  return false;
}
void fp_channel_reset(fp_channel* ch) { (void)ch; }
struct ast_json* fp_channel_search(fp_channel* ch, const char* c, const int co, const double t, const int l, const int h) {
  (void)ch; (void)c; (void)co; (void)t; (void)l; (void)h;
  return NULL;
}
void fp_channel_close(fp_channel* ch) { (void)ch; }
bool fp_get_search_stats(int64_t* calls, int64_t* batches) {
  (void)calls; (void)batches;
  return false;
}

static void print_ints(const int32_t* v, int64_t n) {
  int64_t k;
  printf("[");
  for (k = 0; k < n; k++) printf("%s%" PRId32, k ? ", " : "", v[k]);
  printf("]");
}

int main(int argc, char** argv) {
  int i = 2;
  if (argc < 2) return 2;
  fpc_set_backup_path(argv[1]);
  while (i < argc) {
    const char* cmd = argv[i++];
    if (!strcmp(cmd, "init")) {
      printf("{\"init\": %s}\n", fpc_db_init() ? "true" : "false");
    } else if (!strcmp(cmd, "term")) {
      printf("{\"term\": %s}\n", fpc_db_term() ? "true" : "false");
    } else if (!strcmp(cmd, "close")) {
      fpc_db_close();
      printf("{\"close\": true}\n");
    } else if (!strcmp(cmd, "create") && i + 2 < argc) {
      printf("{\"create\": %d}\n", fpc_create_audio_list_info(argv[i], argv[i + 1], argv[i + 2]));
      i += 3;
    } else if (!strcmp(cmd, "store") && i + 2 < argc) {
      FILE* f = fopen(argv[i + 2], "rb");
      long bytes;
      int64_t n;
      int32_t* v;
      bool ok = false;
      if (f && !fseek(f, 0, SEEK_END) && (bytes = ftell(f)) >= 0 && !fseek(f, 0, SEEK_SET)) {
        n = bytes / 8;
        v = malloc(sizeof(int32_t) * (2 * n + 1));
        if (fread(v, sizeof(int32_t), 2 * n, f) == (size_t)(2 * n)) ok = fpc_store_fingerprints(argv[i], argv[i + 1], v, v + n, n);
        free(v);
      }
      if (f) fclose(f);
      printf("{\"store\": %s}\n", ok ? "true" : "false");
      i += 3;
    } else if (!strcmp(cmd, "load")) {
      fpc_rows r;
      int32_t c;
      if (!fpc_load_fingerprints(&r)) {
        printf("{\"load\": false}\n");
        continue;
      }
      printf("{\"load\": true, \"clips\": [");
      for (c = 0; c < r.nclips; c++) {
        const int64_t b = r.frame_offsets[c], n = r.frame_offsets[c + 1] - b;
        printf("%s{\"uuid\": \"%s\", \"m1\": ", c ? ", " : "", r.uuids[c]);
        print_ints(r.m1 + b, n);
        printf(", \"m2\": ");
        print_ints(r.m2 + b, n);
        printf("}");
      }
      printf("]}\n");
      fpc_rows_free(&r);
    } else if (!strcmp(cmd, "delete") && i < argc) {
      printf("{\"delete\": %s}\n", fpc_delete_audio_list_info(argv[i]) ? "true" : "false");
      i += 1;
    } else if (!strcmp(cmd, "ctx") && i + 1 < argc) {
      printf("{\"ctx\": %s}\n", fp_create_context_list_info(argv[i], argv[i + 1], false) ? "true" : "false");
      i += 2;
    } else if (!strcmp(cmd, "ctxdel") && i < argc) {
      printf("{\"ctxdel\": %s}\n", fp_delete_context_list_info(argv[i]) ? "true" : "false");
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
    } else if (!strcmp(cmd, "cthreads") && i + 2 < argc && i + 3 + atoi(argv[i + 2]) <= argc) {
      const int nf = atoi(argv[i + 2]);
      cthreads(atoi(argv[i]), atoi(argv[i + 1]), nf, argv + i + 3);  /* (shim_harness.c) */
      i += 3 + nf;
    } else if (!strcmp(cmd, "uuid")) {
      char* u = fp_generate_uuid();
      printf("{\"uuid\": \"%s\"}\n", u ? u : "");
      free(u);
    } else {
      fprintf(stderr, "bad command %s\n", cmd);
      return 2;
    }
    fflush(stdout);
  }
  return 0;
}
