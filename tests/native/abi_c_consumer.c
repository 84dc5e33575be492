/* A C99 consumer of include/tiresias_fp.h, as the reference's fp_handler.c shim would be
 * (INTEGRATION.md): plain C, no C++ or HIP headers, linked against libtiresias_fp.so.
 *
 *   abi_c_consumer host          host-only entry points (no GPU needed)
 *   abi_c_consumer gpu OUT.bin   enrol 8 synthetic clips, fingerprint one excerpt and search it;
 *                                writes the excerpt's frames and the result for the test to check
 *
 * Built and run by tests/test_cabi.py (host) and tests/test_gpu_parity.py (gpu). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tiresias_fp.h"

#define NCLIPS 8
#define CLIP_SAMPLES (8000 * 6)
#define Q_SAMPLES (8000 * 3)
#define Q_OFFSET 4096

static int fail(const char* what, int rc, tfp_engine* e) {
  fprintf(stderr, "%s failed: %d %s\n", what, rc, e ? tfp_engine_last_error(e) : "");
  return 1;
}

static int run_host(void) {
  tfp_synth_spec spec;
  int16_t* pcm;
  int rc;
  if (tfp_abi_version() != TFP_ABI_VERSION) return fail("abi version", tfp_abi_version(), NULL);
  if (tfp_frame_count(0) != 0 || tfp_frame_count(1) != 1 || tfp_frame_count(256) != 1 || tfp_frame_count(257) != 2)
    return fail("frame_count", 0, NULL);
  pcm = (int16_t*)malloc(sizeof(int16_t) * 1024);
  spec.seed = 7;
  spec.clip = 3;
  spec.offset = 0;
  rc = tfp_synth_pcm(&spec, 1, 1024, pcm);
  if (rc != TFP_OK) return fail("synth", rc, NULL);
  if (tfp_synth_pcm(NULL, 1, 1024, pcm) != TFP_E_ARG) return fail("synth NULL specs", 0, NULL);
  {
    /* audio ingest: the 44-byte header Asterisk's format_wav writes, then 2 samples */
    static const unsigned char wav[48] = {'R', 'I', 'F', 'F', 40, 0, 0, 0, 'W', 'A', 'V', 'E', 'f', 'm', 't', ' ',
                                          16, 0, 0, 0, 1, 0, 1, 0, 0x40, 0x1f, 0, 0, 0x80, 0x3e, 0, 0, 2, 0, 16, 0,
                                          'd', 'a', 't', 'a', 4, 0, 0, 0, 0x34, 0x12, 0xff, 0xff};
    unsigned char stereo[48];
    int16_t s[2];
    int64_t ns = 0;
    int32_t sr = 0;
    rc = tfp_wav_decode(wav, sizeof wav, s, 2, &ns, &sr);
    if (rc != TFP_OK || ns != 2 || sr != 8000 || s[0] != 0x1234 || s[1] != -1) return fail("wav_decode", rc, NULL);
    memcpy(stereo, wav, sizeof wav);
    stereo[22] = 2;
    stereo[32] = 4;
    rc = tfp_wav_decode(stereo, sizeof stereo, s, 2, &ns, &sr);
    if (rc != TFP_E_FORMAT || !tfp_engine_last_error(NULL)[0]) return fail("wav_decode stereo", rc, NULL);
  }
  printf("host ok: abi %d, first sample %d\n", tfp_abi_version(), (int)pcm[0]);
  free(pcm);
  return 0;
}

static int run_gpu(const char* out_path) {
  tfp_engine* e = NULL;
  tfp_synth_spec specs[NCLIPS];
  int16_t* pcm = (int16_t*)malloc(sizeof(int16_t) * (size_t)NCLIPS * CLIP_SAMPLES);
  int64_t offsets[NCLIPS + 1];
  const int64_t fpc = tfp_frame_count(CLIP_SAMPLES);
  tfp_frame* rows = (tfp_frame*)malloc(sizeof(tfp_frame) * (size_t)NCLIPS * fpc);
  int32_t* m1 = (int32_t*)malloc(sizeof(int32_t) * fpc);
  int32_t* m2 = (int32_t*)malloc(sizeof(int32_t) * fpc);
  int64_t got = 0, nq;
  tfp_frame* qrows;
  tfp_search_params p;
  tfp_result r;
  FILE* f;
  int c, rc;
  int64_t i;
  char uuid[64];

  if ((rc = tfp_engine_create(0, &e)) != TFP_OK) return fail("engine_create", rc, NULL);
  for (c = 0; c < NCLIPS; c++) {
    specs[c].seed = 0xC0FFEE;
    specs[c].clip = c;
    specs[c].offset = 0;
    offsets[c] = (int64_t)c * CLIP_SAMPLES;
  }
  offsets[NCLIPS] = (int64_t)NCLIPS * CLIP_SAMPLES;
  if ((rc = tfp_synth_pcm(specs, NCLIPS, CLIP_SAMPLES, pcm)) != TFP_OK) return fail("synth", rc, e);
  if ((rc = tfp_fingerprint_batch(e, pcm, offsets, NCLIPS, 8000, rows, NCLIPS * fpc, &got)) != TFP_OK)
    return fail("fingerprint_batch", rc, e);
  if (got != NCLIPS * fpc) return fail("frame total", (int)got, e);
  for (c = 0; c < NCLIPS; c++) {
    for (i = 0; i < fpc; i++) {
      m1[i] = rows[c * fpc + i].m1;
      m2[i] = rows[c * fpc + i].m2;
    }
    snprintf(uuid, sizeof uuid, "00000000-0000-4000-8000-%012d", c);
    if ((rc = tfp_index_add(e, uuid, m1, m2, (int32_t)fpc, NULL)) != TFP_OK) return fail("index_add", rc, e);
  }
  /* query: an excerpt of clip 5 */
  nq = tfp_frame_count(Q_SAMPLES);
  qrows = (tfp_frame*)malloc(sizeof(tfp_frame) * nq);
  if ((rc = tfp_fingerprint_pcm(e, pcm + 5 * CLIP_SAMPLES + Q_OFFSET, Q_SAMPLES, 8000, qrows, nq, &got)) != TFP_OK)
    return fail("fingerprint_pcm", rc, e);
  memset(&p, 0, sizeof p);
  p.coefs = 1;
  p.tolerance = 0.5;
  p.freq_ignore_low = -1;
  p.freq_ignore_high = -1;
  if ((rc = tfp_search(e, qrows, (int32_t)nq, &p, &r)) != TFP_OK) return fail("search", rc, e);
  f = fopen(out_path, "wb");
  if (!f) return fail("fopen", 0, e);
  fwrite(&nq, sizeof nq, 1, f);
  fwrite(qrows, sizeof(tfp_frame), (size_t)nq, f);
  fwrite(&r, sizeof r, 1, f);
  fclose(f);
  printf("gpu ok: found %d uuid %s match_count %d frame_count %d\n", r.found, r.uuid, r.match_count, r.frame_count);
  tfp_engine_destroy(e);
  free(pcm); free(rows); free(m1); free(m2); free(qrows);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && strcmp(argv[1], "host") == 0) return run_host();
  if (argc >= 3 && strcmp(argv[1], "gpu") == 0) return run_gpu(argv[2]);
  fprintf(stderr, "usage: %s host | gpu OUT.bin\n", argv[0]);
  return 2;
}
